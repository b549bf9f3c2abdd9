#!/bin/bash
# walker rewrite check: AmpModem / chain GPU tests, walker timing (tuning build), bench 20 steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pll_seqc.py tests/test_gpu_ssb.py tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread -k "ampmodem or pll or ssb or chain or broadcast" > gpurun_out/r04e_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04e_pytest.log; [ $rc -eq 0 ] || exit $rc
LDSP_PKG_DIR=build_tuning timeout -k 10 300 python scripts/walk_variants.py 0,8,9,0 > gpurun_out/r04e_walk_variants.log 2>&1
rc=$?; grep -v "^{" gpurun_out/r04e_walk_variants.log | tail -5 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-components > gpurun_out/r04e_bench20.log 2>&1
rc=$?; grep "^{" gpurun_out/r04e_bench20.log | cut -c1-330; exit $rc
