#!/bin/bash
# k_pll_seqh: the short-call PLL tests on the product build, then the horizon sweep
# (tuning build) and the README block timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_pll_seqc.py tests/test_gpu_smallcalls.py > gpurun_out/seqh_tests.log 2>&1
rc=$?; tail -2 gpurun_out/seqh_tests.log; [ $rc -eq 0 ] || exit $rc
for D in ${DS:-0}; do
  LDSP_PKG_DIR=$PWD/build_tuning LDSP_PLL_SEQH_D=$D timeout -k 10 120 python3 scripts/seqh_sweep.py || exit 1
done
timeout -k 10 200 python3 scripts/readme_blocks.py
