"""Where the exact SOS cascade's time goes: per section wave of k_iir_sect, shader
clocks per sample spent waiting (input / ring space), forming the input tile and
in the recursion (ldsp_debug_iir_sect_trace), for the chain's cheby2 order-8
filter (BASELINE C4) in exact mode.  N (default 16 Mi) complex samples, one call."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

n = int(os.environ.get("N", str(16 << 20)))
order = int(os.environ.get("ORDER", "8"))
x = torch.randn(n, dtype=torch.complex64, device="cuda") * 0.1
f = L.ComplexIIRFilter(filter_type="cheby2", order=order, Fc=15000 / 2000000)
f.exact = True
f(x[:4096])
buf = torch.zeros(2 * 9 * 4, dtype=torch.int64, device="cuda")
L._debug_iir_sect_trace(buf.data_ptr())
torch.cuda.synchronize()
t0 = time.perf_counter()
f(x)
torch.cuda.synchronize()
el = time.perf_counter() - t0
L._debug_iir_sect_trace(0)
t = buf.cpu().numpy().reshape(2, 9, 4)
nsec = (order + 1) // 2
out = {"n": n, "ms": round(el * 1e3, 2), "Msamples_s": round(n / el / 1e6, 2), "waves": []}
for c in range(2):
    for w in range(nsec):
        wait, u, loop, tot = (int(v) for v in t[c, w])
        out["waves"].append({"comp": c, "wave": w, "clk_per_sample": {"wait": round(wait / n, 2), "u": round(u / n, 2),
                             "loop": round(loop / n, 2), "total": round(tot / n, 2)}})
print(json.dumps(out), flush=True)
