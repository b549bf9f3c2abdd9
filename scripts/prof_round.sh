#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the bench and of the
# FIR benchmark, then FETCH_SIZE and WRITE_SIZE in separate --pmc passes (no
# trace domains beside --pmc), summarised per kernel by scripts/pmc_summary.py.
#   bash scripts/prof_round.sh r01   -> gpurun_out/prof/r01_*  (copy to profiles/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
tag=${1:-r01}
out=gpurun_out/prof/$tag
mkdir -p $out
B="python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-components"
F="python3 scripts/firbench.py"
run() {   # name, rocprof args..., -- cmd
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" > $out/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $out/$name.log; exit $rc; }
}
run bench_trace --kernel-trace --stats --output-format csv -d $out/bench_trace -o bench -- $B
run fir_trace --kernel-trace --stats --output-format csv -d $out/fir_trace -o fir -- $F
run bench_fetch --pmc FETCH_SIZE --output-format csv -d $out/bench_fetch -o bench -- $B
run bench_write --pmc WRITE_SIZE --output-format csv -d $out/bench_write -o bench -- $B
run bench_sq --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM --output-format csv -d $out/bench_sq -o bench -- $B
run fir_fetch --pmc FETCH_SIZE --output-format csv -d $out/fir_fetch -o fir -- $F
run fir_write --pmc WRITE_SIZE --output-format csv -d $out/fir_write -o fir -- $F
# the fused front (filter_resample) and its two-call form at 64 Mi (scripts/fused_front.py front)
R="python3 scripts/fused_front.py front"
run front_trace --kernel-trace --stats --output-format csv -d $out/front_trace -o front -- $R
# the walk's duration cross-check: with the early hand-off off every walker waits in
# stream order, so rocprof's k_pll_walk duration is the walk itself; the same run's
# JSON line (in the log) carries the walker's own clock (roofline.ms_per_launch)
run walk0_trace --kernel-trace --stats --output-format csv -d $out/walk0_trace -o walk0 -- $B --walk-early 0
# the exact SOS cascade (k_iir_sect) and the fast modal IIR at 64 Mi (scripts/iir_exact_time.py)
run iirx_trace --kernel-trace --stats --output-format csv -d $out/iirx_trace -o iirx -- python3 scripts/iir_exact_time.py
run front_fetch --pmc FETCH_SIZE --output-format csv -d $out/front_fetch -o front -- $R
run front_write --pmc WRITE_SIZE --output-format csv -d $out/front_write -o front -- $R
python3 scripts/pmc_summary.py $out > $out/summary.json && cat $out/summary.json
