#!/bin/bash
# channels per GPU: 1, 2, 4, 8, 12 channels with 2 streams each (fused front)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for c in 1 2 4 8 12; do
  timeout -k 10 300 python scripts/fused_front.py channels fused 2 c=$c > gpurun_out/r04v_ch.log 2>&1
  rc=$?; grep "^{" gpurun_out/r04v_ch.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
