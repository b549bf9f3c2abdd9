"""Timing decomposition of the PLL walker k_pll_walk (tuning build:
LDSP_PKG_DIR=build_tuning).  The AmpModem input of the bench chain (BASELINE
C4: 64 Mi IQ -> IIR -> resampler -> AGC, 1.61 M samples) is demodulated by a
fresh AmpModem per variant, 5 calls, walker time averaged over calls 2-5.
LDSP_WALK_VARIANT (the block-loop asm, walk_asm_loop<VAR / 32>): 0 product, 32 no
repairs, 64 no per-lane-block store (32 and 64 give wrong outputs: timing only), 96
the store issued by a helper wave's scratch slot (timing only)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "build_tuning"))]
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import numpy as np  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402
from bench import AMRadio, synth_channel  # noqa: E402

dev = torch.device("cuda", 0)
x = synth_channel(64 << 20, 0, dev)
r = AMRadio(L)
a = r.agc(r.resample(r.bandpass(x)))
torch.cuda.synchronize()
del x
variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "0,32,64,96,0".split(","))]
ref = None
out = {}
for v in variants:
    os.environ["LDSP_WALK_VARIANT"] = str(v)
    am = L.AmpModem(modulation=0.5, type="dsb", carrier=True)
    ys = []
    for k in range(5):
        if k == 1:
            L._profile_reset()
            L._profile_enable(True)
        ys.append(am(a))
    torch.cuda.synchronize()
    L._profile_enable(False)
    rep = L._profile_report()
    e, rp, fb = am._walk_stats()
    cw, cb = am._walk_clocks()
    y = torch.cat(ys).cpu().numpy()
    if ref is None and v == 0:
        ref = y
    same = bool(np.array_equal(y.view(np.uint32), ref.view(np.uint32))) if ref is not None else None
    w = rep["k_pll_walk"]
    out[str(v)] = {"walk_ms": round(w[1] / w[0], 4), "entries": e, "repairs": rp, "fallbacks": fb,
                   "clk_walk": cw, "clk_wait": cb, "bitwise_v0": same}
    print(v, json.dumps(out[str(v)]), flush=True)
print(json.dumps(out))
