#!/bin/bash
# FMStereo A/B: scripts/fm_time.py on the product build and on build_fm (the
# chain recording table indices), alternating twice, then the FMStereo parity
# tests on build_fm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/fmab; mkdir -p $O
for r in 1 2; do
  timeout -k 10 200 python3 scripts/fm_time.py > $O/old$r.jsonl 2>/dev/null || exit $?
  LDSP_PKG_DIR=$PWD/build_fm timeout -k 10 200 python3 scripts/fm_time.py > $O/new$r.jsonl 2>/dev/null || exit $?
  for v in old new; do echo "$v $(python3 -c "
import json
for l in open('$O/$v$r.jsonl'):
    d=json.loads(l); print(d['input'], d['Msamples_s'], d['fm_pll_Msamples_s'], end='; ')")"; done
done
LDSP_PKG_DIR=$PWD/build_fm timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "fmstereo or FMStereo or fm_" > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; exit $rc
