#!/bin/bash
# Round-end rehearsal on one GPU: the GPU test suite, smoke(), the default bench
# line, and the rocprofv3 evidence (kernel stats + PMC passes) into gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -1 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_full.log; exit $rc; }
grep '^{' gpurun_out/bench_full.log | tail -1 > gpurun_out/bench_full.json; cut -c1-400 gpurun_out/bench_full.json
timeout -k 10 300 python scripts/chains_bench.py > gpurun_out/chains.log 2>&1 && grep '^{' gpurun_out/chains.log | tail -1 > gpurun_out/chains.json
[ -n "$PROF" ] && bash scripts/prof_round.sh ${PROF} > gpurun_out/prof.log 2>&1; echo "prof rc=$?"
