#!/bin/bash
# kernel trace of the fused front (k_iir_modal_rs / k_iir_resamp_edges durations)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r04m
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04m -o ff -- python3 scripts/fused_front.py front > gpurun_out/r04m/log.txt 2>&1
rc=$?; tail -2 gpurun_out/r04m/log.txt
f=$(find gpurun_out/r04m -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -12
exit $rc
