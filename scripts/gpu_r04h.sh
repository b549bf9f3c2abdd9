#!/bin/bash
# exec-masked walker repair loop: micro-benchmark, AmpModem / chain GPU tests, walker timing, bench 20 steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench/walk_loop > gpurun_out/r04h_walk_loop.txt 2>&1
rc=$?; cat gpurun_out/r04h_walk_loop.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pll_seqc.py tests/test_gpu_ssb.py tests/test_gpu_chain.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread -k "ampmodem or pll or ssb or chain or broadcast or amradio" > gpurun_out/r04h_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04h_pytest.log; [ $rc -eq 0 ] || exit $rc
LDSP_PKG_DIR=build_tuning timeout -k 10 300 python scripts/walk_variants.py 0,0 > gpurun_out/r04h_walk_variants.log 2>&1
rc=$?; grep "^[0-9]" gpurun_out/r04h_walk_variants.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-components > gpurun_out/r04h_bench20.log 2>&1
rc=$?; grep "^{" gpurun_out/r04h_bench20.log | cut -c1-400; exit $rc
