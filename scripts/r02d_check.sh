#!/bin/bash
# Round-2 (d) GPU pass: GPU tests, smoke, the driver-setting bench, the default
# bench with components, the walk-gap kernel trace and the README blocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
o=gpurun_out/r02d; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 $o/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-components > $o/bench20.log 2>&1
rc=$?; echo "bench20 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $o/bench20.log; exit $rc; }
grep '^{' $o/bench20.log | tail -1 | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/tr -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-components --no-kprof > $o/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $o/tr -name '*kernel_trace.csv' | head -1)
python3 scripts/walk_gaps.py "$f" 22 > $o/gaps.txt; tail -8 $o/gaps.txt; gzip "$f"
timeout -k 10 300 python scripts/readme_blocks.py > $o/readme.log 2>&1
rc=$?; echo "readme rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' $o/readme.log | tail -1 > $o/readme_blocks.json; cut -c1-600 $o/readme_blocks.json | tail -c 300
timeout -k 10 600 python bench.py > $o/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $o/bench_full.log; exit $rc; }
grep '^{' $o/bench_full.log | tail -1 > $o/bench_full.json; cut -c1-300 $o/bench_full.json
