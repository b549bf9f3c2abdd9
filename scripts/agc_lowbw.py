"""AGC at a low bandwidth (1e-4): the chunk-parallel threshold grows to ~620 k
samples, so every shorter call runs tsa mode (chunks approximating from the
call's true start state).  Times each call size, counts in-kernel / runfix
re-runs and checks every call bitwise against the restatement.  Run once as is
and once with LDSP_AGC_TSAMIN=1000000000 (tsa off: those calls take the
sequential / speculative path) to compare -- the LDSP_* knobs are read only by
a tuning build (Makefile EXTRA=-DLDSP_TUNING; LDSP_PKG_DIR points at it)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")]
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker only)

bw = float(os.environ.get("BW", "1e-4"))
rng = np.random.default_rng(7)
fs = 48000.0
sizes = [2_000, 20_000, 100_000, 300_000, 600_000]
n = sum(sizes) * 2
t = np.arange(n) / fs
msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t)) / 2
env = 0.1 * (1 + 0.5 * msg) * (1 + 0.8 * (np.sin(2 * np.pi * 0.7 * t) > 0))
x = (env * np.exp(2j * np.pi * 300 / fs * np.arange(n))
     + 0.003 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
xd = torch.from_numpy(x).cuda()
g = L.AGC()
g.bandwidth = bw
g.lock = False
g.scale = 0.01
o = O.AGC()
o.bandwidth = np.float32(bw)
o.scale = np.float32(0.01)
rows, a, ok = [], 0, True
for rep in range(2):
    for s in sizes:
        torch.cuda.synchronize()
        r0 = g._tsa_reruns()
        t0 = time.perf_counter()
        y = g(xd[a:a + s])
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ref = o(x[a:a + s])
        same = bool((y.cpu().numpy().view(np.uint32) == ref.view(np.uint32)).all())
        ok &= same
        rows.append({"rep": rep, "n": s, "ms": round(el * 1e3, 2), "reruns": g._tsa_reruns() - r0, "bitwise": same})
        a += s
print(json.dumps({"bandwidth": bw, "tsamin": os.environ.get("LDSP_AGC_TSAMIN"), "all_bitwise": ok, "calls": rows}))
sys.exit(0 if ok else 1)
