cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for s in 3; do for st in 20 50; do
timeout -k 10 300 python bench.py --steps $st --streams $s --no-kprof --no-cpu-baseline --no-components > gpurun_out/b_${s}_$st.log 2>&1 || exit $?
echo "streams $s steps $st $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_${s}_$st.log) $(grep -o '"host_ms[a-z_]*": [0-9.]*' gpurun_out/b_${s}_$st.log)"
done; done
