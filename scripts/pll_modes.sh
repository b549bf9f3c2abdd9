#!/bin/bash
# Walker timing experiments (debug modes produce wrong output; timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for m in 0 1; do
  LDSP_DEBUG_PLL=1 LDSP_DEBUG_PLL_MODE=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pll_mode$m.log 2>&1 || exit $?
  echo "mode $m"; grep "ldsp pll" gpurun_out/pll_mode$m.log | tail -1
done
