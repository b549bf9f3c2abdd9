#!/bin/bash
# AGC repair rounds (tuning knob LDSP_AGC_ROUNDS, default 3): 8 channels and the single-chain bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in 3 1 3 1; do
  LDSP_PKG_DIR=build_tuning LDSP_AGC_ROUNDS=$r timeout -k 10 300 python scripts/fused_front.py channels fused 2 > gpurun_out/r04y_ch.log 2>&1
  rc=$?; echo "rounds=$r $(grep '^{' gpurun_out/r04y_ch.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
done
for r in 3 1; do
  LDSP_PKG_DIR=build_tuning LDSP_AGC_ROUNDS=$r timeout -k 10 300 python scripts/channels_prof.py 8 > gpurun_out/r04y_chprof.log 2>&1
  rc=$?; echo "rounds=$r $(grep '^{' gpurun_out/r04y_chprof.log | cut -c1-600)"; [ $rc -eq 0 ] || exit $rc
done
