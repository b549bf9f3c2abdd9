"""FMStereo throughput (product or LDSP_PKG_DIR build) on two 4 Mi-sample
inputs: complex Gaussian noise (scripts/chains_bench.py's input) and an FM
stereo broadcast composite (pilot 19 kHz, L+R, L-R on 38 kHz, deviation 75 kHz
at 600 kS/s): wall MS/s and per-kernel ms.  One line per input."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

n = int(os.environ.get("FM_N", str(1 << 22)))
fs = 600e3
rng = np.random.default_rng(1)
t = np.arange(n) / fs
left = np.sin(2 * np.pi * 440 * t)
right = np.sin(2 * np.pi * 1000 * t)
comp = 0.45 * (left + right) / 2 + 0.1 * np.sin(2 * np.pi * 19e3 * t) + 0.45 * (left - right) / 2 * np.sin(2 * np.pi * 38e3 * t)
fmx = np.exp(1j * 2 * np.pi * 75e3 * np.cumsum(comp) / fs).astype(np.complex64)
noise = ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)).astype(np.complex64)
for name, x in (("noise", noise), ("fm_composite", fmx)):
    xd = torch.from_numpy(x).cuda()
    f = L.FMStereo()
    f(xd[: 1 << 16])
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    t0 = time.perf_counter()
    f(xd)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    L._profile_enable(False)
    ker = {k: round(v[1] / v[0], 2) for k, v in L._profile_report().items()}
    print(json.dumps({"input": name, 
                      "Msamples_s": round(n / el / 1e6, 2), "kernels_ms": ker,
                      "fm_pll_Msamples_s": round(n / ker.get("k_fm_pll", 1e9) / 1e3, 2)}))
