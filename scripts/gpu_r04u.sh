#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/channels_host.py > gpurun_out/r04u_host.log 2>&1
rc=$?; grep "^{" gpurun_out/r04u_host.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/r04u_host.log; exit $rc; }
