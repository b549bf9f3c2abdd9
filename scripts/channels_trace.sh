#!/bin/bash
# rocprofv3 kernel trace of the bench's 8-channel component (scripts/channels_run.py)
# summarised by scripts/trace_summary.py from the 17th walker launch on (after
# warm-up), plus the driver-setting bench line (20 steps, 5 warm-up).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/chtrace; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o ch -- python3 scripts/channels_run.py > $out/run.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/run.log; exit $rc; }
grep '^{' $out/run.log | tail -1
python3 scripts/trace_summary.py $out/trace k_pll_walk:16 > $out/summary.json && head -c 1500 $out/summary.json
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-components > $out/bench20.log 2>&1
rc=$?; echo "bench20 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench20.log; exit $rc; }
grep '^{' $out/bench20.log | tail -1 | cut -c1-300
