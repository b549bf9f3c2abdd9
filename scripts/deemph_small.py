"""DeemphasisFilter (48 kHz) on README-sized calls (1 573 samples, device
tensors): per-call kernel times and wall time per call.  One JSON line;
LDSP_IIR_SPEC_MIN (tuning build) moves small calls to the sequential loop."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

n, calls = int(os.environ.get("N", "1573")), 200
x = torch.from_numpy(np.random.default_rng(1).standard_normal(n * calls).astype(np.float32)).cuda()
if os.environ.get("EXACT") == "1":   # the same first-order filter as an exact-mode RIIRFilter
    xd = np.float32(np.exp(-1.0 / (75.0e-6 * 48000.0)))
    f = L.RIIRFilter(np.array([1.0 - xd], np.float32), np.array([1.0, -xd], np.float32))
    f.exact = True
else:
    f = L.DeemphasisFilter(48000)
for i in range(4):
    f(x[i * n:(i + 1) * n])
torch.cuda.synchronize()
L._profile_reset()
L._profile_enable(True)
t0 = time.perf_counter()
for i in range(calls):
    f(x[i * n:(i + 1) * n])
torch.cuda.synchronize()
el = time.perf_counter() - t0
L._profile_enable(False)
print(json.dumps({"spec_min": os.environ.get("LDSP_IIR_SPEC_MIN", "default"), "n": n,
                  "us_per_call": round(el / calls * 1e6, 1),
                  "kernel_us": {k: round(v[1] / v[0] * 1e3, 1) for k, v in L._profile_report().items()}}))
