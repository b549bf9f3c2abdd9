"""Device throughput of the receive-path helpers either side of the hot path
(SURVEY 8f): bytes_to_iq, Delay, FreqDem, BroadcastAM, FMStereo, the default
resamplers; per-kernel HIP-event times from libldsp's profiler, inputs
resident in HBM.  One JSON line.  CHAINS_N overrides the IQ block size."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "python-liquiddsp_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import liquiddsp as L  # noqa: E402

N = int(os.environ.get("CHAINS_N", str(16 << 20)))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(5)


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    L._profile_enable(False)
    ker = {k: round(v[1] / v[0], 4) for k, v in L._profile_report().items()}
    return {"wall_ms": round(el * 1e3, 3), "Msamples_s": round(N / el / 1e6, 1), "kernels_ms": ker}


res = {"iq_samples": N}
raw = torch.randint(-32768, 32767, (2 * N,), dtype=torch.int16, device=dev, generator=g)
res["bytes_to_iq"] = timed(lambda: L.bytes_to_iq(raw))
x = torch.complex(torch.randn(N, generator=g, device=dev), torch.randn(N, generator=g, device=dev))
d = L.Delay(25)
res["delay25"] = timed(lambda: d(x))
fd = L.FreqDem(0.1)
res["freqdem"] = timed(lambda: fd(x))
t = torch.arange(N, device=dev, dtype=torch.float64) / 48000.0
am = ((1 + 0.5 * torch.sin(2 * np.pi * 700 * t)) * torch.exp(1j * (2 * np.pi * 3.0 * t + 0.3))).to(torch.complex64)
bam = L.BroadcastAM()
res["broadcast_am"] = timed(lambda: bam(am))
cr = L.CResampler(0.5)
res["cresampler_0.5"] = timed(lambda: cr(x))
n_fm = min(N, 1 << 22)
xf = x[:n_fm].contiguous()
fm = L.FMStereo()
r = timed(lambda: fm(xf), reps=1)
r["Msamples_s"] = round(n_fm / (r["wall_ms"] * 1e-3) / 1e6, 2)
r["iq_samples"] = n_fm
res["fmstereo"] = r
print(json.dumps(res), flush=True)
