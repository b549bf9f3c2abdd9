#!/bin/bash
# fused front: tests, timing, 8 channels fused / unfused in separate processes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -k "filter_resample" > gpurun_out/r04l_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04l_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/fused_front.py front > gpurun_out/r04l_fused_front.log 2>&1 || exit $?
timeout -k 10 300 python scripts/fused_front.py channels fused >> gpurun_out/r04l_fused_front.log 2>&1 || exit $?
timeout -k 10 300 python scripts/fused_front.py channels unfused >> gpurun_out/r04l_fused_front.log 2>&1
rc=$?; grep "^{" gpurun_out/r04l_fused_front.log | cut -c1-400; exit $rc
