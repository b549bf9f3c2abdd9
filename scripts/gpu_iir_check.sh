# modal IIR: parity tests, then timings (product build and the tuning build's variants)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_iir_modal.py tests/test_gpu_bytes.py tests/test_gpu_parity.py tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread -k "iir or modal or bytes or chain" > gpurun_out/t_modal.log 2>&1
rc=$?; tail -15 gpurun_out/t_modal.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/iir_bench.py > gpurun_out/iir_bench.json 2> gpurun_out/iir_bench.err; rc=$?; cat gpurun_out/iir_bench.json; [ $rc -eq 0 ] || exit $rc
if [ -d build_tuning ]; then LDSP_PKG_DIR=build_tuning timeout -k 10 200 python scripts/iir_variants.py; fi
