#!/bin/bash
# PLL-focused GPU check: AmpModem/BroadcastAM/chain parity tests, walker
# counters (LDSP_DEBUG_PLL), then the bench without components.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-ampmodem or amradio or broadcast or smoke}" > gpurun_out/pytest_pll.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_pll.log
[ $rc -eq 0 ] || exit $rc
LDSP_DEBUG_PLL=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-components > gpurun_out/pll_dbg.log 2>&1
rc=$?; echo "dbg rc=$rc"; grep "ldsp pll" gpurun_out/pll_dbg.log | tail -2
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-components > gpurun_out/bench_pll.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_pll.log | cut -c1-700
exit $rc
