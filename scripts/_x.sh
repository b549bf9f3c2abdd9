cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "agc or amradio or smoke" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 400 python scripts/block_sweep.py > gpurun_out/block_sweep.log 2>&1; rc=$?; grep streams gpurun_out/block_sweep.log | head -10; exit $rc
