#!/bin/bash
# FFT-FIR kernel variants (tuning build PKG, default build_tuning; LDSP_FFT_VARIANT bits: see k_firfft.hip)
# on firbench's workloads; one JSON line per variant into gpurun_out/firvar/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/firvar
P=${PKG:-build_tuning}
export LDSP_PKG_DIR=$PWD/$P
for v in "$@"; do
  LDSP_FFT_VARIANT=$v FIRBENCH_REPS=${FIRBENCH_REPS:-20} timeout -k 10 120 python3 scripts/firbench.py \
      > gpurun_out/firvar/$P.v$v.json 2> gpurun_out/firvar/$P.v$v.err || { echo "variant $v failed"; tail -3 gpurun_out/firvar/$P.v$v.err; exit 1; }
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], {k: (v.get('ms'), v.get('kernel') or v.get('kernels')) for k, v in r.items() if isinstance(v, dict)})" gpurun_out/firvar/$P.v$v.json $v $P
done
