#!/bin/bash
# large modal scans on a CU-masked stream: GPU suite, 8-channel A/B (tuning build
# knob LDSP_IIR_CUMASK), per-kernel times under 8 channels, single-chain bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04x_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r04x_pytest.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1 0 1; do
  LDSP_PKG_DIR=build_tuning LDSP_IIR_CUMASK=$m timeout -k 10 300 python scripts/fused_front.py channels fused 2 > gpurun_out/r04x_ch.log 2>&1
  rc=$?; echo "cumask=$m $(grep '^{' gpurun_out/r04x_ch.log | cut -c1-260)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python scripts/fused_front.py channels unfused 2 > gpurun_out/r04x_ch.log 2>&1
rc=$?; echo "product unfused $(grep '^{' gpurun_out/r04x_ch.log | cut -c1-260)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/channels_prof.py 1 8 > gpurun_out/r04x_chprof.log 2>&1
rc=$?; grep "^{" gpurun_out/r04x_chprof.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-components > gpurun_out/r04x_b20.log 2>&1
rc=$?; grep '^{' gpurun_out/r04x_b20.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline --no-components > gpurun_out/r04x_b100.log 2>&1
rc=$?; grep '^{' gpurun_out/r04x_b100.log | cut -c1-250; exit $rc
