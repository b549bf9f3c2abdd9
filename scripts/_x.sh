cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for kp in "" "--no-kprof"; do
timeout -k 10 300 python bench.py $kp --no-cpu-baseline --no-components > gpurun_out/k.log 2>&1 || exit $?
echo "kprof=$kp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/k.log) $(grep -o '"k_pll_walk": {[^}]*}' gpurun_out/k.log)"
done
