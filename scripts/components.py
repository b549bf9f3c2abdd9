"""Component benchmarks on one GPU (HIP events on torch's current stream):

  fir127   ComplexFIRFilter, 127 taps (Kaiser fc=0.1, As=60), 64 Mi complex64   (north-star FIR)
  resamp   ComplexResampler rate=48k/2M, 64 Mi complex64                          (BASELINE config 2)
  nco_fir  NCO.mix_down + ComplexFIRFilter 255 taps, 256 Mi complex64             (BASELINE config 3)

Algorithmic bytes: read input once + write output once.
Usage: python scripts/components.py [--reps R] [--json]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "python-liquiddsp_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM = 8000.0
FP32 = 157.3


def _time(fn, reps, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def kaiser(n, fc, As):
    """Windowed-sinc lowpass taps (numpy); any 127/255 real taps exercise the kernel."""
    beta = 0.1102 * (As - 8.7)
    t = np.arange(n) - (n - 1) / 2
    r = 2 * t / n
    return (np.sinc(2 * fc * t) * np.i0(beta * np.sqrt(1 - r * r)) / np.i0(beta)).astype(np.float32)


def run(reps=10, sizes=None):
    import liquiddsp as L
    dev = torch.device("cuda", 0)
    sizes = sizes or {}
    out = {}
    g = torch.Generator(device=dev)
    g.manual_seed(1)

    n = sizes.get("fir127", 64 << 20)
    x = torch.complex(torch.randn(n, generator=g, device=dev), torch.randn(n, generator=g, device=dev))
    f = L.ComplexFIRFilter(kaiser(127, 0.1, 60.0))
    ms = _time(lambda: f(x), reps)
    byt = 16 * n
    flops = 4 * 127 * n
    out["fir127"] = {"n": n, "ms": round(ms, 4), "Msamples_s": round(n / ms / 1e3, 1),
                     "GBs": round(byt / ms / 1e6, 1), "hbm_frac": round(byt / ms / 1e6 / HBM, 4),
                     "TFLOPs": round(flops / ms / 1e9, 2), "valu_frac": round(flops / ms / 1e9 / FP32, 4)}
    del x

    n = sizes.get("resamp", 64 << 20)
    x = torch.complex(torch.randn(n, generator=g, device=dev), torch.randn(n, generator=g, device=dev))
    r = L.ComplexResampler(rate=48000 / 2000000, Fc=48000 / 2000000)
    ms = _time(lambda: r(x), reps)
    k = int(n * 0.024)
    byt = 8 * n + 8 * k
    out["resamp"] = {"n": n, "ms": round(ms, 4), "Msamples_s": round(n / ms / 1e3, 1),
                     "GBs": round(byt / ms / 1e6, 1), "hbm_frac": round(byt / ms / 1e6 / HBM, 4)}
    del x

    n = sizes.get("nco_fir", 256 << 20)
    x = torch.complex(torch.randn(n, generator=g, device=dev), torch.randn(n, generator=g, device=dev))
    nco = L.NCO("nco")
    nco.freq = float(2 * np.pi * 0.05)
    f2 = L.ComplexFIRFilter(kaiser(255, 0.05, 60.0))
    ms_n = _time(lambda: nco.mix_down(x), reps)
    ms = _time(lambda: f2(nco.mix_down(x)), reps)
    byt = 32 * n                      # unfused: NCO read+write, FIR read+write
    flops = (6 + 4 * 255) * n
    out["nco_fir"] = {"n": n, "ms": round(ms, 4), "nco_ms": round(ms_n, 4), "Msamples_s": round(n / ms / 1e3, 1),
                      "GBs": round(byt / ms / 1e6, 1), "TFLOPs": round(flops / ms / 1e9, 2),
                      "valu_frac": round(flops / ms / 1e9 / FP32, 4)}
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    print(json.dumps(run(a.reps)))
