#!/bin/bash
# AGC speculation tuning on the bench workload: per (W, Wa, rounds) the AGC
# stage time (bench stage_ms) and, in a separate debug run, the re-run counts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/agc_sweep; mkdir -p $out
for cfg in "20 40 2" "14 40 2" "10 40 2" "7 40 2" "10 30 2" "10 40 3"; do
  set -- $cfg
  tag="w$1_wa$2_r$3"
  LDSP_AGC_WMUL=$1 LDSP_AGC_WAMUL=$2 LDSP_AGC_ROUNDS=$3 timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 \
      --no-components --no-cpu-baseline > $out/$tag.json 2> $out/$tag.err || { echo "$tag failed"; tail -3 $out/$tag.err; exit 1; }
  LDSP_DEBUG_AGC=1 LDSP_AGC_WMUL=$1 LDSP_AGC_WAMUL=$2 LDSP_AGC_ROUNDS=$3 timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 \
      --no-components --no-cpu-baseline > /dev/null 2> $out/$tag.dbg || exit 1
  python3 - "$out/$tag.json" "$out/$tag.dbg" "$tag" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = r["kernels"]
dbg = [l.strip() for l in open(sys.argv[2]) if "[ldsp agc]" in l][-1:]
print(sys.argv[3], "value", r["value"], "agc_ms", r["stage_ms"]["agc"], "chunks", k["k_agc_chunks"]["ms"],
      "runfix", k.get("k_agc_runfix", {}).get("ms"), "verify", k["k_agc_verify"]["ms"], dbg)
PY
done
