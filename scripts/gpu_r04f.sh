#!/bin/bash
# exact pipelined IIR + walker exec-window tweak: tests, timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "iir or ampmodem or amradio" > gpurun_out/r04f_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04f_pytest.log; [ $rc -eq 0 ] || exit $rc
LDSP_PKG_DIR=build_tuning timeout -k 10 300 python scripts/walk_variants.py 0,0 > gpurun_out/r04f_walk_variants.log 2>&1
rc=$?; grep -v "^{" gpurun_out/r04f_walk_variants.log | tail -2 | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/iir_exact_time.py > gpurun_out/r04f_iir_exact.log 2>&1
rc=$?; tail -5 gpurun_out/r04f_iir_exact.log; exit $rc
