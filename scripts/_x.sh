cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-components > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/b.log; grep -o '"roofline": {.*}, "streams' gpurun_out/b.log
