#!/bin/bash
# the whole GPU suite after the walker cleanup (incl. the bench's RCCL path at world
# size 1 and filter_resample at other rates), long-J IIR timing, 3-stream channels,
# the walker's tuning variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04p_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r04p_pytest.log; [ $rc -eq 0 ] || exit $rc
LDSP_PKG_DIR=build_tuning timeout -k 10 300 python scripts/iir_variants.py 0,7,3,24,40,56,88,0 > gpurun_out/r04p_iir_variants.log 2>&1
rc=$?; tail -1 gpurun_out/r04p_iir_variants.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/iir_longJ.py > gpurun_out/r04p_iir_longJ.log 2>&1
rc=$?; tail -2 gpurun_out/r04p_iir_longJ.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/fused_front.py channels fused 3 > gpurun_out/r04p_channels3.log 2>&1
rc=$?; grep "^{" gpurun_out/r04p_channels3.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/walk_variants.py > gpurun_out/r04p_walk_variants.log 2>&1
rc=$?; tail -1 gpurun_out/r04p_walk_variants.log | cut -c1-800; [ $rc -eq 0 ] || exit $rc
# 8 channels: front / back stages on separate streams, the back ones at high priority
for v in "2" "2 split" "2 split prio" "1 split prio"; do
  timeout -k 10 300 python scripts/fused_front.py channels fused $v > gpurun_out/r04p_ch.log 2>&1
  rc=$?; grep "^{" gpurun_out/r04p_ch.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04p_prof_ch -o ch -- python3 scripts/fused_front.py channels fused 2 > gpurun_out/r04p_prof_ch.log 2>&1
rc=$?; find gpurun_out/r04p_prof_ch -name "*kernel_stats.csv"; exit $rc
