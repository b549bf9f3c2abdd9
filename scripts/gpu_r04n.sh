#!/bin/bash
# exact IIR tile pipeline (tests + 64 Mi timing) and the fused front (tests, timing, channels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_chain.py tests/test_golden.py -x -q --timeout 120 --timeout-method thread -k "iir or filter_resample or exact or deemph or golden" > gpurun_out/r04n_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04n_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/iir_exact_time.py > gpurun_out/r04n_iir_exact.log 2>&1
rc=$?; tail -1 gpurun_out/r04n_iir_exact.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/fused_front.py front > gpurun_out/r04n_fused_front.log 2>&1 || exit $?
timeout -k 10 300 python scripts/fused_front.py channels fused >> gpurun_out/r04n_fused_front.log 2>&1
rc=$?; grep "^{" gpurun_out/r04n_fused_front.log | cut -c1-400; exit $rc
