#!/bin/bash
# FFT-FIR GPU check: the FIR/NCO-fused parity tests on the product build, the
# kernel variants of the tuning build on firbench (VARIANTS, LDSP_FFT_VARIANT
# values; repeat one to see the run-to-run spread), then with PMC=1 the
# config-3 counter passes (scripts/fir_c3_pmc.sh) of the product build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_boundary.py > gpurun_out/fft_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fft_tests.log; [ $rc -eq 0 ] || exit $rc
FIRBENCH_TAPS=127,255 bash scripts/fir_variants.sh ${VARIANTS:-0 4 6 32 0 4 32} || exit 1
if [ "${PMC:-0}" = 1 ]; then
  bash scripts/fir_c3_pmc.sh && python3 scripts/pmc_kernel.py gpurun_out/c3pmc > gpurun_out/c3pmc/summary.json
fi
