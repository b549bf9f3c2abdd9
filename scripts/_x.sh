cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "iir or amradio" > gpurun_out/pt.log 2>&1 || { tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --streams 1 --no-cpu-baseline --no-components > gpurun_out/b1.log 2>&1 || exit $?
echo "$(grep -o '"k_iir_blk_local": {[^}]*}' gpurun_out/b1.log) $(grep -o '"k_iir_blk_final": {[^}]*}' gpurun_out/b1.log)"
