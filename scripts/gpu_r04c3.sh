#!/bin/bash
# config 3 launch spread: per-launch durations + GRBM busy cycles + SQ counters (scripts/fir_c3_pmc.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
FIRBENCH_REPS=16 PMC_OUT=gpurun_out/r04c3 bash scripts/fir_c3_pmc.sh > gpurun_out/r04c3.log 2>&1
rc=$?; cat gpurun_out/r04c3.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/c3_spread.py gpurun_out/r04c3 > gpurun_out/r04c3_spread.json && cut -c1-200 gpurun_out/r04c3_spread.json | head -60
