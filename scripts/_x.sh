#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
LDSP_PROF_TIMELINE=gpurun_out/tl.txt timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --no-components > gpurun_out/tl_bench.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"ms_per_launch": [0-9.]*' gpurun_out/tl_bench.log | tr '\n' ' '; echo
python scripts/prof_timeline.py gpurun_out/tl.txt > gpurun_out/tl_summary.txt
exit $rc
