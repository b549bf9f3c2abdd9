#!/bin/bash
# NCO table row rotation in the fused NCO + FFT FIR: mix / fused tests, then config 3 timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04s_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r04s_pytest.log; [ $rc -eq 0 ] || exit $rc
FIRBENCH_TAPS=255 timeout -k 10 300 python scripts/firbench.py > gpurun_out/r04s_fir.log 2>&1
rc=$?; grep "^{" gpurun_out/r04s_fir.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
FIRBENCH_TAPS=255 timeout -k 10 300 python scripts/firbench.py > gpurun_out/r04s_fir2.log 2>&1
rc=$?; grep "^{" gpurun_out/r04s_fir2.log | cut -c1-900; exit $rc
