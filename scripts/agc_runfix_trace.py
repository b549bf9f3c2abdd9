"""Per-run trace of the AGC run-fix (k_agc_runfix_wide) on the bench chain:
needs a build with -DLDSP_AGC_TRACE (each run's workgroup prints its chunk
count, in-order lane re-runs and elapsed time).  Knobs from argv K=V pairs.
    make OUT=../build_e1 OBJDIR=../build_e1/obj EXTRA="-DLDSP_TUNING -DLDSP_AGC_TRACE"
    LDSP_PKG_DIR=build_e1 python3 scripts/agc_runfix_trace.py LDSP_AGC_WMUL=5"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for kv in sys.argv[1:]:
    k, v = kv.split("=", 1)
    os.environ[k] = v
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "build_e1")]
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402
from bench import AMRadio, synth_channel  # noqa: E402

dev = torch.device("cuda", 0)
x = synth_channel(64 << 20, 0, dev)
r = AMRadio(L)
for i in range(3):
    print(f"--- call {i}", flush=True)
    r(x)
    torch.cuda.synchronize()
