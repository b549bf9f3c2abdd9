#!/bin/bash
# Walker diagnostics: counters (LDSP_DEBUG_PLL=1), every lane-block through the
# generic path (=2, exact, slow),
# and the bench at 1..4 rotating streams (no components, no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for m in 1 2; do
  LDSP_DEBUG_PLL=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-components > gpurun_out/pll_dbg$m.log 2>&1
  rc=$?; echo "dbg$m rc=$rc"; grep "ldsp pll" gpurun_out/pll_dbg$m.log | tail -1
  grep -o '"k_pll_walk": {[^}]*}' gpurun_out/pll_dbg$m.log
  [ $rc -eq 0 ] || exit $rc
done
for s in 1 2 3 4 6; do
  timeout -k 10 300 python bench.py --steps 20 --streams $s --no-cpu-baseline --no-components > gpurun_out/bench_s$s.log 2>&1
  rc=$?; echo "streams $s rc=$rc"; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_s$s.log
  [ $rc -eq 0 ] || exit $rc
done
