cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fir" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 200 python scripts/firbench.py 2>&1 | tail -3
