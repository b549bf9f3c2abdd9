cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for m in 1; do
LDSP_DEBUG_PLL=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-components > gpurun_out/dbg$m.log 2>&1 || exit $?
echo "mode $m $(grep 'ldsp pll' gpurun_out/dbg$m.log | tail -1) $(grep -o '"k_pll_walk": {[^}]*}' gpurun_out/dbg$m.log)"
done
