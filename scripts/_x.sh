#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ampmodem or amradio or broadcast or smoke" > gpurun_out/pytest_pll.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_pll.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline --no-components > gpurun_out/pll_bb.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"ms_per_launch": [0-9.]*' gpurun_out/pll_bb.log | tr '\n' ' '; echo
exit $rc
