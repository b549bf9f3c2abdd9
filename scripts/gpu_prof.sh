#!/bin/bash
# rocprofv3 kernel-trace summaries for the bench and the component benchmarks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python scripts/components.py --reps 10 > gpurun_out/components.json 2> gpurun_out/components.err
rc=$?; echo "components rc=$rc"; cat gpurun_out/components.json; tail -3 gpurun_out/components.err
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/bench -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof bench rc=$rc"; tail -3 gpurun_out/prof_bench.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/comp -o comp -- python3 scripts/components.py --reps 5 > gpurun_out/prof_comp.log 2>&1
rc=$?; echo "rocprof comp rc=$rc"
find gpurun_out/prof -name "*stats*"
exit $rc
