#!/bin/bash
# SQ issue counters of k_iir_modal (iir_bench.py, 64 Mi cheby2-8) for several
# package builds (LDSP_PKG_DIR), one rocprofv3 pass per build:
#   bash scripts/iir_sq_ab.sh OUTDIR build_a build_b ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp REPS=${REPS:-6}
out=$1; shift; mkdir -p "$out"
for pk in "$@"; do
  n=$(basename "$pk")
  LDSP_PKG_DIR=$pk timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_SALU --output-format csv -d "$out/$n" -o iir -- \
      python3 scripts/iir_bench.py > "$out/$n.log" 2>&1 || { echo "$n failed"; tail -5 "$out/$n.log"; exit 1; }
  echo "== $n"; python3 scripts/pmc_kernel.py "$out/$n" | python3 -c "
import json,sys; d=json.load(sys.stdin)
for k,v in d.items():
    if k.startswith('k_iir_modal<2, 4, false'): print(k, {c: round(x/65536,1) for c,x in v.items()})"
done
