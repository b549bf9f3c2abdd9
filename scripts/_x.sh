cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ampmodem or amradio or broadcast" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-components > gpurun_out/b$i.log 2>&1 || exit $?
echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b$i.log) $(grep -o '"k_pll_walk": {[^}]*}' gpurun_out/b$i.log)"
done
