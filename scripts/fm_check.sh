#!/bin/bash
# FMStereo: the FM / IIR GPU tests, then MS/s and per-kernel times of the
# product build on noise and an FM composite (scripts/fm_time.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "fmstereo or fm_ or iir or deemph" \
    tests/ > gpurun_out/fm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/fm_tests.log; [ $rc -eq 0 ] || exit $rc
for D in 0; do
  timeout -k 10 120 python3 scripts/fm_time.py || exit 1
done
