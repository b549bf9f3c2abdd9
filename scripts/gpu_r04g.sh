#!/bin/bash
# re-entry check after the container rebuild: every GPU test, then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04g_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04g_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04g_bench20.log 2>&1
rc=$?; grep "^{" gpurun_out/r04g_bench20.log | cut -c1-900; exit $rc
