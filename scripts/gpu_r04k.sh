#!/bin/bash
# fused front (tests, timing, channels) + walker timing variants (tuning build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "filter_resample or ampmodem" > gpurun_out/r04k_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04k_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/fused_front.py > gpurun_out/r04k_fused_front.log 2>&1
rc=$?; cut -c1-600 gpurun_out/r04k_fused_front.log; [ $rc -eq 0 ] || exit $rc
LDSP_PKG_DIR=build_tuning timeout -k 10 300 python scripts/walk_variants.py 0,32,64,96,128,0 > gpurun_out/r04k_walk_variants.log 2>&1
rc=$?; grep "^[0-9]" gpurun_out/r04k_walk_variants.log | cut -c1-250; exit $rc
