#!/bin/bash
# Kernel trace of the README small-call path (one stream, 65 536-sample blocks,
# scripts/readme_blocks.py) and its per-block timeline (scripts/block_timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/blocktrace; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o blk -- python3 scripts/readme_blocks.py > $out/run.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/run.log; exit $rc; }
grep '^{' $out/run.log | tail -1
python3 scripts/block_timeline.py $out/trace k_iir_modal 8 > $out/timeline.txt && cat $out/timeline.txt
