#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/channels_prof.py 1 4 8 > gpurun_out/r04w_chprof.log 2>&1
rc=$?; grep "^{" gpurun_out/r04w_chprof.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04w_chprof.log; exit $rc; }
