#!/bin/bash
# k_iir_sect A/B: the per-wave clock trace (scripts/iir_sect_trace.py) of the
# previous build (build_ab) and this one, alternating twice, then the exact-mode
# parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/sab; mkdir -p $O
for r in 1 2; do
  LDSP_PKG_DIR=$PWD/build_ab timeout -k 10 120 python3 scripts/iir_sect_trace.py > $O/old$r.json 2>/dev/null || exit $?
  timeout -k 10 120 python3 scripts/iir_sect_trace.py > $O/new$r.json 2>/dev/null || exit $?
  for v in old new; do python3 -c "import json; d=json.load(open('$O/$v$r.json')); print('$v', d['ms'], d['Msamples_s'], [w['clk_per_sample']['loop'] for w in d['waves']])"; done
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_many.py -k "exact" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
