#!/bin/bash
# A/B timing of the IIR kernels: scripts/iir_bench.py on a saved build of the
# package (OLD, default build_ab: libldsp.so + liquiddsp/ copied before a
# change) and on the tree's build, alternated twice; then the modal GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OLD=${OLD:-build_ab}
out=gpurun_out/iir_ab; mkdir -p $out
for r in 1 2; do
    LDSP_PKG_DIR=$PWD/$OLD timeout -k 10 120 python3 scripts/iir_bench.py > $out/old$r.json || exit $?
    timeout -k 10 120 python3 scripts/iir_bench.py > $out/new$r.json || exit $?
    echo "old$r $(cut -c1-400 $out/old$r.json)"
    echo "new$r $(cut -c1-400 $out/new$r.json)"
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_iir_modal.py tests/test_gpu_bytes.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
exit $rc
