#!/bin/bash
# walker: readfirstlane loop variant (ubench) and the product loop's timing split (tuning build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench/walk_loop > gpurun_out/r04i_walk_loop.txt 2>&1
rc=$?; tail -6 gpurun_out/r04i_walk_loop.txt; [ $rc -eq 0 ] || exit $rc
LDSP_PKG_DIR=build_tuning timeout -k 10 300 python scripts/walk_variants.py 0,32,64,0 > gpurun_out/r04i_walk_variants.log 2>&1
rc=$?; grep "^[0-9]" gpurun_out/r04i_walk_variants.log | cut -c1-250; exit $rc
