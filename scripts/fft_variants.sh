#!/bin/bash
# FFT-FIR experiment variants (LDSP_FFT_VARIANT), one process each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3}; do
  LDSP_FFT_VARIANT=$v timeout -k 10 120 python scripts/firbench.py > gpurun_out/fftv_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/fftv_$v.log; exit 1; }
  grep variant gpurun_out/fftv_$v.log
done
