#!/bin/bash
# First-line GPU validation: parity tests, smoke, short bench.
# Each GPU step has its own time limit; a crash-like exit (fault/abort/timeout)
# ends the script so nothing else touches the GPU after it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
ok() { case "$1" in 0|1) return 0;; *) return 1;; esac; }
echo "host: $(nproc) cpus; $(lscpu | grep 'Model name' | head -1)"
ldconfig -p | grep -i liquid || echo "no system libliquid"
timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
