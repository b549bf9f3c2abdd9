#!/bin/bash
# A/B of the folded PLL chunk scan (LDSP_PLL_FOLD, tuning build), alternating:
# the batched channel components (scripts/batched_run.py), 8 per-channel chains
# (scripts/channels_run.py) and the bench chain at the driver setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/foldb; mkdir -p $O
for r in 1 2; do
  for f in 1 0; do
    export LDSP_PLL_FOLD=$f LDSP_PKG_DIR=build_tuning
    timeout -k 10 300 python3 scripts/batched_run.py > $O/b_f${f}_$r.json 2> $O/b_f${f}_$r.err || exit $?
    timeout -k 10 300 python3 scripts/channels_run.py > $O/c_f${f}_$r.json 2> $O/c_f${f}_$r.err || exit $?
    timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-components --steps 20 --warmup 5 > $O/t20_f${f}_$r.json 2> $O/t20_f${f}_$r.err || exit $?
    echo "fold $f run $r batched $(python3 -c "import json; d=json.load(open('$O/b_f${f}_$r.json')); print(d['batched_8'].get('Msamples_s'), d['batched_16'].get('Msamples_s'))") channels $(tail -c 300 $O/c_f${f}_$r.json | tr '\n' ' ' | cut -c1-160) t20 $(python3 -c "import json; d=json.loads(open('$O/t20_f${f}_$r.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('single_stream_ms_per_step'))")"
  done
done
