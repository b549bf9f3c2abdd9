#!/bin/bash
# Bench step time vs rotating streams, with and without per-kernel HIP events in the timed steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for s in ${STREAMS:-2 3 4}; do for kp in "" "--no-kprof"; do
  timeout -k 10 300 python bench.py --steps 20 --streams $s $kp --no-cpu-baseline --no-components ${BENCH_ARGS} > gpurun_out/sw_s$s$kp.log 2>&1
  rc=$?; echo "streams $s $kp rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sw_s$s$kp.log) $(grep -o '"host_ms_per_step": [0-9.]*' gpurun_out/sw_s$s$kp.log) $(grep -o '"k_pll_walk": {[^}]*}' gpurun_out/sw_s$s$kp.log)"
  [ $rc -eq 0 ] || exit $rc
done; done
