#!/bin/bash
# Batched channels (scripts/batched_run.py): the product build against the
# previous one (build_ab), alternating twice, after the fused-front and PLL tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/front3; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_many.py > $O/pytest.log 2>&1; rc=$?; tail -1 $O/pytest.log; [ $rc = 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python3 scripts/batched_run.py > $O/b$r.json 2> $O/b$r.err || exit $?
  LDSP_PKG_DIR=$PWD/build_ab timeout -k 10 300 python3 scripts/batched_run.py > $O/ab$r.json 2> $O/ab$r.err || exit $?
  echo "new $(python3 -c "import json; d=json.load(open('$O/b$r.json')); print(d['batched_8']['Msamples_s'], d['batched_16']['Msamples_s'])")  old $(python3 -c "import json; d=json.load(open('$O/ab$r.json')); print(d['batched_8']['Msamples_s'], d['batched_16']['Msamples_s'])")"
done
