#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run -> gpurun_out/prof/<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=${1:-bench}
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$tag -o $tag -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_$tag.log
python3 - "$tag" <<'PY'
import csv, re, sys
t = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/prof/{t}/{t}_kernel_stats.csv")):
    m = re.search(r'(k_\w+)', r['Name'])
    print(f"{(m.group(1) if m else r['Name'][:40]):40s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:10.1f} pct={float(r['Percentage']):6.2f}")
PY
exit $rc
