#!/bin/bash
# Where k_iir_modal spends its time: kernel-trace stats, HBM bytes (FETCH_SIZE x2
# per the gfx950 correction, WRITE_SIZE) and SQ / GRBM counters of iir_bench.py
# (64 Mi cheby2 order 8), each in its own rocprofv3 pass; the f64 / valu2 passes
# split the VALU instructions by type (IIRPMC_OUT: output directory).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp REPS=${REPS:-10}
out=${IIRPMC_OUT:-gpurun_out/iirpmc}; mkdir -p $out
B="python3 scripts/iir_bench.py"
run() { local name=$1; shift; timeout -s KILL 120 rocprofv3 "$@" > $out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }; }
run trace --kernel-trace --stats --output-format csv -d $out/trace -o iir -- $B
run fetch --pmc FETCH_SIZE --output-format csv -d $out/fetch -o iir -- $B
run write --pmc WRITE_SIZE --output-format csv -d $out/write -o iir -- $B
run sq --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $out/sq -o iir -- $B
run sq2 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d $out/sq2 -o iir -- $B
run grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $out/grbm -o iir -- $B
run f64 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU --output-format csv -d $out/f64 -o iir -- $B
run valu2 --pmc SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $out/valu2 -o iir -- $B
