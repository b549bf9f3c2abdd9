set -o pipefail
O=gpurun_out/fold; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_many.py tests/test_gpu_chain.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || exit $rc
for f in 1 0 1 0; do
  LDSP_PLL_FOLD=$f LDSP_PKG_DIR=build_tuning LDSP_PROF_TIMELINE=$O/single_f$f.txt timeout -k 10 200 python3 scripts/single_call_timeline.py > $O/single_f$f.out 2>&1 || exit $?
  echo "fold $f $(tail -1 $O/single_f$f.out | cut -c1-40)"
done
