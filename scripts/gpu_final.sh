#!/bin/bash
# Round-end evidence on one GPU: every GPU test, smoke(), the default bench line
# (100 steps, components, CPU baseline), the driver-setting line (20 steps), the
# helper chains, and rocprofv3 kernel stats + PMC passes (scripts/prof_round.sh TAG).
#   bash scripts/gpu_final.sh r04o  -> gpurun_out/final_r04o/, gpurun_out/prof/r04o/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
tag=${1:-r04o}
o=gpurun_out/final_$tag
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -1 $o/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $o/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-components > $o/bench20.log 2>&1
rc=$?; echo "bench20 rc=$rc"; [ $rc -eq 0 ] || { tail -5 $o/bench20.log; exit $rc; }
grep '^{' $o/bench20.log | tail -1 > $o/bench_steps20.json; cut -c1-300 $o/bench_steps20.json
timeout -k 10 700 python bench.py > $o/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $o/bench_full.log; exit $rc; }
grep '^{' $o/bench_full.log | tail -1 > $o/bench.json; cut -c1-300 $o/bench.json
timeout -k 10 300 python scripts/chains_bench.py > $o/chains.log 2>&1 && grep '^{' $o/chains.log | tail -1 > $o/chains.json
echo "chains rc=$?"
bash scripts/prof_round.sh $tag > $o/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 $o/prof.log; exit $rc
