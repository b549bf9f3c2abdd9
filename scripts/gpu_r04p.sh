#!/bin/bash
# the whole GPU suite after the walker cleanup (incl. the bench's RCCL path at world
# size 1 and filter_resample at other rates), long-J IIR timing, 3-stream channels,
# the walker's tuning variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04p_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r04p_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/iir_longJ.py > gpurun_out/r04p_iir_longJ.log 2>&1
rc=$?; tail -2 gpurun_out/r04p_iir_longJ.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/fused_front.py channels fused 3 > gpurun_out/r04p_channels3.log 2>&1
rc=$?; grep "^{" gpurun_out/r04p_channels3.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/walk_variants.py > gpurun_out/r04p_walk_variants.log 2>&1
rc=$?; tail -1 gpurun_out/r04p_walk_variants.log | cut -c1-800; exit $rc
