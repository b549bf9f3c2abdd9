#!/bin/bash
# A/B timing of the IIR kernels: scripts/iir_bench.py on a saved build of the
# package (OLD, default build_ab: libldsp.so + liquiddsp/ copied before a
# change), on the saved builds in VARIANTS and on the tree's build, alternated
# twice (PERSIST: LDSP_IIR_PERSIST settings, read by tuning builds only -- the
# knob of the persistent experiment in DESIGN.md section 4, since removed); then the
# modal GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OLD=${OLD:-build_ab}
out=gpurun_out/iir_ab; mkdir -p $out
for r in 1 2; do
    LDSP_PKG_DIR=$PWD/$OLD timeout -k 10 120 python3 scripts/iir_bench.py > $out/old$r.json || exit $?
    echo "old$r $(cut -c1-120 $out/old$r.json)"
    for V in $VARIANTS; do             # other saved builds (directories)
        LDSP_PKG_DIR=$PWD/$V timeout -k 10 120 python3 scripts/iir_bench.py > $out/$V$r.json || exit $?
        echo "$V $r $(cut -c1-120 $out/$V$r.json)"
    done
    for P in ${PERSIST:-default}; do
        if [ "$P" = default ]; then timeout -k 10 120 python3 scripts/iir_bench.py > $out/new${P}_$r.json || exit $?
        else LDSP_IIR_PERSIST=$P timeout -k 10 120 python3 scripts/iir_bench.py > $out/new${P}_$r.json || exit $?; fi
        echo "new$P $r $(cut -c1-120 $out/new${P}_$r.json)"
    done
done
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_iir_modal.py tests/test_gpu_bytes.py > $out/pytest.log 2>&1; rc=$?
tail -3 $out/pytest.log
exit $rc
