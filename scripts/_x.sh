cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "agc or ampmodem or amradio or broadcast or smoke" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
BLK=65536 timeout -k 10 200 python scripts/readme_blocks.py 2>&1 | tail -1
