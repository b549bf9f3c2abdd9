#!/bin/bash
# PLL-focused GPU check: AmpModem/BroadcastAM/chain parity tests (sparse walker,
# then every lane-block forced through the generic path), walker counters
# (LDSP_DEBUG_PLL), then the bench without components.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
K="${PYTEST_K:-ampmodem or amradio or broadcast or smoke}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_pll.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_pll.log
[ $rc -eq 0 ] || exit $rc
LDSP_DEBUG_PLL=2 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_pll_fb.log 2>&1
rc=$?; echo "pytest (all generic) rc=$rc"; grep -v "ldsp pll" gpurun_out/pytest_pll_fb.log | tail -5
[ $rc -eq 0 ] || exit $rc
for m in 1 2; do
LDSP_DEBUG_PLL=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-components > gpurun_out/pll_dbg$m.log 2>&1
rc=$?; echo "dbg$m rc=$rc"; grep "ldsp pll" gpurun_out/pll_dbg$m.log | tail -1; grep -o '"k_pll_walk": {[^}]*}' gpurun_out/pll_dbg$m.log
[ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-components > gpurun_out/bench_pll.log 2>&1
rc=$?; echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench_pll.log | cut -c1-900
exit $rc
