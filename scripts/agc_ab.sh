#!/bin/bash
# AGC approximate-step A/B: the bench chain at the driver setting (single-call
# latency, per-kernel times) and the batched channels on the product build and
# on build_agc (the fused-series approximate step), alternating twice, then the
# AGC / chain tests on build_agc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/agcab; mkdir -p $O
B="python3 bench.py --no-cpu-baseline --no-components --steps 20 --warmup 5"
for r in 1 2; do
  for v in old new; do
    if [ $v = new ]; then export LDSP_PKG_DIR=$PWD/build_agc; else unset LDSP_PKG_DIR; fi
    timeout -k 10 300 $B > $O/t20_$v$r.json 2> $O/t20_$v$r.err || exit $?
    timeout -k 10 300 python3 scripts/batched_run.py > $O/b_$v$r.json 2> $O/b_$v$r.err || exit $?
    python3 -c "
import json
d=json.loads(open('$O/t20_$v$r.json').read().strip().splitlines()[-1]); b=json.load(open('$O/b_$v$r.json'))
k=d['kernels']
print('$v', d['ms_per_step'], d['single_stream_ms_per_step'], 'agc_chunks', k['k_agc_chunks']['ms'], 'runfix', k['k_agc_runfix']['ms'], 'verify', k['k_agc_verify']['ms'], 'batched', b['batched_8']['Msamples_s'], b['batched_16']['Msamples_s'])"
  done
done
export LDSP_PKG_DIR=$PWD/build_agc
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_agc_rounds.py tests/test_gpu_chain.py tests/test_gpu_many.py -k "agc or AGC or chain or amradio or many" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
