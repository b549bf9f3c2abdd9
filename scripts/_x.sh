cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ampmodem or amradio or broadcast" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for m in 1; do
LDSP_DEBUG_PLL=$m timeout -k 10 300 python bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-components > gpurun_out/dbg$m.log 2>&1 || exit $?
echo "mode $m $(grep 'ldsp pll' gpurun_out/dbg$m.log | tail -1)"
done
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --streams 1 --no-cpu-baseline --no-components > gpurun_out/b1.log 2>&1 || exit $?
echo "$(grep -o '"k_pll_walk": {[^}]*}' gpurun_out/b1.log)"
