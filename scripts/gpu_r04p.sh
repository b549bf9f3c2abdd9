#!/bin/bash
# the bench's RCCL path at world size 1 under torch.distributed.run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_fused.py -k "rccl or other_rates" -x -v --timeout 300 --timeout-method thread > gpurun_out/r04p_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/r04p_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/iir_longJ.py > gpurun_out/r04p_iir_longJ.log 2>&1
rc=$?; tail -2 gpurun_out/r04p_iir_longJ.log | cut -c1-600; exit $rc
