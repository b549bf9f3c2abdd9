cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -5 gpurun_out/bench_full.log; exit 1; }
timeout -k 10 300 python scripts/chains_bench.py > gpurun_out/chains.log 2>&1 || { tail -5 gpurun_out/chains.log; exit 1; }
grep '^{' gpurun_out/bench_full.log | tail -1 > gpurun_out/bench_full.json
grep '^{' gpurun_out/chains.log | tail -1 > gpurun_out/chains.json
cut -c1-600 gpurun_out/bench_full.json
