"""FIR kernel timing on the GPU (per-kernel HIP events): ComplexFIRFilter at
64 Mi complex64 samples for a few tap counts and modes, and BASELINE config 3
(NCO.mix_down + 255-tap ComplexFIRFilter at 256 Mi samples) unfused and fused
(liquiddsp.mix_down_filter).  Prints one JSON line.  LDSP_PKG_DIR selects the
package build (e.g. the tuning build, whose LDSP_FFT_VARIANT picks the kernel variant)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402


def kaiser(n, fc, As):
    beta = 0.1102 * (As - 8.7)
    t = np.arange(n) - (n - 1) / 2
    r = 2 * t / n
    return (np.sinc(2 * fc * t) * np.i0(beta * np.sqrt(1 - r * r)) / np.i0(beta)).astype(np.float32)


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    L._profile_enable(False)
    return {k: tot / c for k, (c, tot) in L._profile_report().items()}


def main():
    n = int(os.environ.get("FIRBENCH_N", 64 << 20))
    taps = [int(v) for v in os.environ.get("FIRBENCH_TAPS", "127,255").split(",")]
    modes = os.environ.get("FIRBENCH_MODES", "fast").split(",")
    reps = int(os.environ.get("FIRBENCH_REPS", 10))
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    x = torch.complex(torch.randn(n, generator=g, device="cuda"), torch.randn(n, generator=g, device="cuda"))
    res = {"variant": os.environ.get("LDSP_FFT_VARIANT", "default"), "n": n}
    for Lt in taps:
        for mode in modes:
            f = L.ComplexFIRFilter(kaiser(Lt, 0.1, 60.0))
            f.mode = mode
            (k, ms), = timed(lambda: f(x), reps).items()
            res[f"L{Lt}_{mode}"] = {"kernel": k, "ms": round(ms, 4), "GBs": round(16 * n / ms / 1e6, 1),
                                    "hbm_frac": round(16 * n / ms / 1e6 / 8000, 4)}
    if os.environ.get("FIRBENCH_C3", "1") == "1":
        del x
        n3 = 256 << 20
        x = torch.complex(torch.randn(n3, generator=g, device="cuda"), torch.randn(n3, generator=g, device="cuda"))
        for fused in (False, True):
            nco = L.NCO("nco")
            nco.freq = float(2 * np.pi * 0.05)
            f = L.ComplexFIRFilter(kaiser(255, 0.05, 60.0))
            t = timed((lambda: L.mix_down_filter(nco, f, x)) if fused else (lambda: f(nco.mix_down(x))), max(3, reps // 2))
            tot = sum(t.values())
            res["c3_fused" if fused else "c3_unfused"] = {"kernels": {k: round(v, 4) for k, v in t.items()},
                                                          "ms": round(tot, 4), "frac_of_16B_roof":
                                                          round(16 * n3 / tot / 1e6 / 8000, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
