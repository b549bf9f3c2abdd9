#!/bin/bash
# Tuning sweep on the GPU box with the tuning build (python-liquiddsp_amd/Makefile:
# make OUT=../build_tuning OBJDIR=../build_tuning/obj EXTRA=-DLDSP_TUNING).
# Each argument is one configuration "NAME VAR=VALUE ...":
#   bash scripts/knob_sweep.sh "base" "warm512 LDSP_PLL_WARM=512"
# Prints the bench step time, the chain stages and the walker's repair count.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/sweep
export LDSP_PKG_DIR=$PWD/build_tuning
for cfg in "$@"; do
  set -- $cfg
  name=$1; shift
  env "$@" timeout -k 10 180 python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-components --no-cpu-baseline \
      > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err
  rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -3 gpurun_out/sweep/$name.err; exit $rc; }
  python3 - gpurun_out/sweep/$name.json "$name" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = r["kernels"]
pick = ["k_iir_blk_local", "k_iir_blk_final", "k_resamp", "k_agc_chunks", "k_agc_runfix", "k_agc_verify", "k_pll_cand",
        "k_pll_walk", "k_iir_spec_chunks"]
print(sys.argv[2], "ms/step", r["ms_per_step"], "single", r["single_stream_ms_per_step"],
      "repairs", r["roofline"].get("serial_chain", {}).get("repairs"),
      {n: k[n]["ms"] for n in pick if n in k}, "stages", r["stage_ms"], flush=True)
PY
done
