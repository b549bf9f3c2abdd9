#!/bin/bash
# k_pll_seqc: the short-call PLL tests on the product build, the per-call timing
# and the README block timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_pll_seqc.py tests/test_gpu_smallcalls.py > gpurun_out/seqh_tests.log 2>&1
rc=$?; tail -2 gpurun_out/seqh_tests.log; [ $rc -eq 0 ] || exit $rc
for D in 0; do
  timeout -k 10 120 python3 scripts/seqc_calls.py || exit 1
done
timeout -k 10 200 python3 scripts/readme_blocks.py
