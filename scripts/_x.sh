#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for m in 1 3; do
  LDSP_DEBUG_PLL=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-components > gpurun_out/pll_dbg$m.log 2>&1
  rc=$?; echo "dbg$m rc=$rc"; grep "ldsp pll" gpurun_out/pll_dbg$m.log | tail -2
  grep -o '"k_pll_walk": {[^}]*}' gpurun_out/pll_dbg$m.log
  [ $rc -eq 0 ] || exit $rc
done
