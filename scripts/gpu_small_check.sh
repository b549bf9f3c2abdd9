#!/bin/bash
# Small-call path check: AGC / IIR / chain / small-call GPU tests, then the README
# block kernel trace (scripts/block_trace.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_smallcalls.py tests/test_gpu_iir_modal.py tests/test_gpu_chain.py tests/test_gpu_parity.py tests/test_gpu_pll_seqc.py > gpurun_out/small_tests.log 2>&1
rc=$?; tail -3 gpurun_out/small_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/block_trace.sh | head -30
