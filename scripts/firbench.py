"""FIR kernel timing on the GPU (per-kernel HIP events): ComplexFIRFilter at
64 Mi complex64 samples for a few tap counts and modes.  Prints one JSON line."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-liquiddsp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402


def kaiser(n, fc, As):
    beta = 0.1102 * (As - 8.7)
    t = np.arange(n) - (n - 1) / 2
    r = 2 * t / n
    return (np.sinc(2 * fc * t) * np.i0(beta * np.sqrt(1 - r * r)) / np.i0(beta)).astype(np.float32)


def main():
    n = int(os.environ.get("FIRBENCH_N", 64 << 20))
    taps = [int(v) for v in os.environ.get("FIRBENCH_TAPS", "127,255").split(",")]
    modes = os.environ.get("FIRBENCH_MODES", "fast").split(",")
    reps = 10
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    x = torch.complex(torch.randn(n, generator=g, device="cuda"), torch.randn(n, generator=g, device="cuda"))
    res = {"variant": os.environ.get("LDSP_FFT_VARIANT", "default"), "n": n}
    for Lt in taps:
        for mode in modes:
            f = L.ComplexFIRFilter(kaiser(Lt, 0.1, 60.0))
            f.mode = mode
            f(x)
            torch.cuda.synchronize()
            L._profile_reset()
            L._profile_enable(True)
            for _ in range(reps):
                f(x)
            torch.cuda.synchronize()
            L._profile_enable(False)
            (k, (c, tot)), = L._profile_report().items()
            ms = tot / c
            res[f"L{Lt}_{mode}"] = {"kernel": k, "ms": round(ms, 4), "GBs": round(16 * n / ms / 1e6, 1),
                                    "hbm_frac": round(16 * n / ms / 1e6 / 8000, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
