#!/bin/bash
# BASELINE config 3 (NCO.mix_down + 255-tap FIR, 256 Mi) fused kernel alone (or
# another firbench workload: FIRBENCH_* and PMC_OUT):
# kernel-trace stats, HBM bytes (FETCH_SIZE x2 per the gfx950 correction,
# WRITE_SIZE) and SQ / GRBM counters, each in its own rocprofv3 pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp FIRBENCH_TAPS=${FIRBENCH_TAPS:-255} FIRBENCH_N=${FIRBENCH_N:-1048576} FIRBENCH_REPS=${FIRBENCH_REPS:-6} FIRBENCH_C3=${FIRBENCH_C3:-1}
out=${PMC_OUT:-gpurun_out/c3pmc}; mkdir -p $out
F="python3 scripts/firbench.py"
run() { local name=$1; shift; timeout -s KILL 120 rocprofv3 "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }; }
run trace --kernel-trace --stats --output-format csv -d $out/trace -o c3 -- $F
run fetch --pmc FETCH_SIZE --output-format csv -d $out/fetch -o c3 -- $F
run write --pmc WRITE_SIZE --output-format csv -d $out/write -o c3 -- $F
run sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $out/sq -o c3 -- $F
run sq2 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $out/sq2 -o c3 -- $F
run lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT --output-format csv -d $out/lds -o c3 -- $F
run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $out/grbm -o c3 -- $F
