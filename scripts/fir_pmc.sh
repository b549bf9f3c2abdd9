#!/bin/bash
# Where the FFT-FIR kernel spends its time: kernel-trace stats over many calls
# (launch-to-launch variance) and SQ / GRBM counters of the same workload
# (FIR-127 at 64 Mi, firbench.py), each in its own rocprofv3 pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp FIRBENCH_TAPS=${FIRBENCH_TAPS:-127} FIRBENCH_C3=${FIRBENCH_C3:-0} FIRBENCH_REPS=${FIRBENCH_REPS:-40}
out=gpurun_out/firpmc; mkdir -p $out
F="python3 scripts/firbench.py"
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }; }
run trace --kernel-trace --stats --output-format csv -d $out/trace -o fir -- $F
run sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $out/sq -o fir -- $F
run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $out/grbm -o fir -- $F
