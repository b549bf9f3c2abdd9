cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ampmodem or amradio or broadcast or smoke" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
LDSP_DEBUG_PLL=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --streams 1 --no-cpu-baseline --no-components > gpurun_out/dbg1.log 2>&1 || exit $?
echo "$(grep 'ldsp pll' gpurun_out/dbg1.log | tail -1)"
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --streams 1 --no-cpu-baseline --no-components > gpurun_out/b1.log 2>&1 || exit $?
echo "solo $(grep -o '"k_pll_walk": {[^}]*}' gpurun_out/b1.log)"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-components > gpurun_out/b3.log 2>&1 || exit $?
echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b3.log) $(grep -o '"k_pll_walk": {[^}]*}' gpurun_out/b3.log)"
