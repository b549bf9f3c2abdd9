"""PLL walker under hard inputs (diagnostic): locked AM, carrier beyond the
lock range, noise only, and Costas (suppressed carrier): walk time and
counters per 1.6 M-sample call, and bit-exactness against the restatement on
a prefix."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "python-liquiddsp_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402
from oracle import oracle as O  # noqa: E402

fs, n = 48000.0, 1610613
rng = np.random.default_rng(5)
t = np.arange(n) / fs
msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t)) / 2
noise = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) / np.sqrt(2)
cases = {
    "locked_1k2": (1 + 0.5 * msg) * np.exp(2j * np.pi * 1200 * t) + 0.03 * noise,
    "unlocked_3k5": (1 + 0.5 * msg) * np.exp(2j * np.pi * 3500 * t) + 0.03 * noise,
    "noise_only": noise,
    "dsbsc_100": msg * np.exp(1j * (2 * np.pi * 100 * t + 0.7)) + 0.03 * noise,
    "dsbsc_5": msg * np.exp(1j * (2 * np.pi * 5 * t + 0.7)) + 0.03 * noise,
}
res = {}
only = os.environ.get("PLL_STRESS_ONLY")
for name, x in cases.items():
    if only and name not in only.split(","):
        continue
    x = x.astype(np.complex64)
    for carrier in (True, False):
        am = L.AmpModem(modulation=0.5, type="dsb", carrier=carrier)
        xd = torch.from_numpy(x).cuda()
        am(xd)                                   # first call: locks / warms up
        torch.cuda.synchronize()
        L._profile_reset()
        L._profile_enable(True)
        t0 = time.perf_counter()
        y = am(xd)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        L._profile_enable(False)
        kp = L._profile_report()
        e, r, f = am._walk_stats()
        ok = None
        if os.environ.get("PLL_STRESS_EXACT") and (name != "locked_1k2" or carrier):   # prefix vs the restatement
            m = 200_000
            g = L.AmpModem(modulation=0.5, type="dsb", carrier=carrier)
            ref = O.AmpModem(0.5, "dsb", carrier=carrier)(x[:m])
            ok = bool(np.array_equal(g(x[:m]).view(np.uint32), ref.view(np.uint32)))
        res[f"{name}_{'carrier' if carrier else 'costas'}"] = {
            "walk_ms": round(kp["k_pll_walk"][1], 3) if "k_pll_walk" in kp else None, "call_ms": round(el * 1e3, 3),
            "entries": int(e), "repairs": int(r), "fallbacks": int(f), "prefix_bitexact": ok}
        print(name, carrier, res[f"{name}_{'carrier' if carrier else 'costas'}"], flush=True)
