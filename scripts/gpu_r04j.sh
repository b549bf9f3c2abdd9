#!/bin/bash
# IIR -> resampler fusion: GPU tests, front timing, 8 channels per GPU fused / unfused
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -k filter_resample > gpurun_out/r04j_pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r04j_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/fused_front.py > gpurun_out/r04j_fused_front.log 2>&1
rc=$?; cat gpurun_out/r04j_fused_front.log | cut -c1-600; exit $rc
