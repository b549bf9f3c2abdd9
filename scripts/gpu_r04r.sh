#!/bin/bash
# page-locked numpy outputs: the GPU suite, then the README block rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04r_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r04r_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/readme_blocks.py 2 > gpurun_out/r04r_readme.log 2>&1
rc=$?; grep "^{" gpurun_out/r04r_readme.log | cut -c1-700; exit $rc
