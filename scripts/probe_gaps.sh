#!/bin/bash
# Kernel trace of the driver-setting bench (walk-to-walk gaps), then AGC
# warm-up sweep with the tuning build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/gaps
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps/tr -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-components --no-kprof > gpurun_out/gaps/bench.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/gaps/bench.log; exit $rc; }
f=$(find gpurun_out/gaps/tr -name '*kernel_trace.csv' | head -1)
python3 scripts/walk_gaps.py "$f" 22 > gpurun_out/gaps/gaps.txt; tail -25 gpurun_out/gaps/gaps.txt
gzip -c "$f" > gpurun_out/gaps/kernel_trace.csv.gz
[ -n "$SWEEP" ] && bash scripts/knob_sweep.sh "base" "wa30 LDSP_AGC_WAMUL=30" "wa25 LDSP_AGC_WAMUL=25" "wa30w15 LDSP_AGC_WAMUL=30 LDSP_AGC_WMUL=15"
exit 0
