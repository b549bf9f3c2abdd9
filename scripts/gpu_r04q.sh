#!/bin/bash
# 8 AMRadio channels on one GPU: streams per channel and hardware queues
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in "fused 1" "unfused 1" "fused 2" "fused 1 split"; do
  timeout -k 10 300 python scripts/fused_front.py channels $v > gpurun_out/r04q_ch.log 2>&1
  rc=$?; grep "^{" gpurun_out/r04q_ch.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
for q in 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python scripts/fused_front.py channels fused 2 > gpurun_out/r04q_ch.log 2>&1
  rc=$?; grep "^{" gpurun_out/r04q_ch.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
