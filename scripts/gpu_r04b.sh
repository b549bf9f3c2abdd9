cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssb.py tests/test_gpu_parity.py tests/test_gpu_pll_seqc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04b_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-components > gpurun_out/r04b_bench20.log 2>&1
rc=$?; grep "^{" gpurun_out/r04b_bench20.log | cut -c1-700; exit $rc
