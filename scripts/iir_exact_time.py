"""Exact-mode IIR timing: the chain's cheby2 order-8 filter (BASELINE C4) with
bandpass.exact = True on 64 Mi complex samples in one call (k_iir_sect) and on
the README's 65 536-sample blocks, next to the fast modal scan."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

n = int(os.environ.get("N", str(64 << 20)))
x = torch.randn(n, dtype=torch.complex64, device="cuda") * 0.1
res = {}
for exact in (False, True):
    f = L.ComplexIIRFilter(filter_type="cheby2", order=8, Fc=15000 / 2000000)
    f.exact = exact
    f(x[:65536])
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    t0 = time.perf_counter()
    f(x)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    L._profile_enable(False)
    rep = {k: round(v[1] / v[0], 3) for k, v in L._profile_report().items()}
    blocks = [x[i:i + 65536] for i in range(0, 64 * 65536, 65536)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in blocks:
        f(b)
    torch.cuda.synchronize()
    eb = (time.perf_counter() - t0) / len(blocks)
    res["exact" if exact else "fast"] = {"n": n, "ms": round(el * 1e3, 3), "Msamples_s": round(n / el / 1e6, 2),
                                          "kernels_ms": rep, "readme_block_ms": round(eb * 1e3, 3)}
    print(json.dumps(res), flush=True)
