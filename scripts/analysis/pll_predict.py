"""How far ahead is the AmpModem carrier PLL's table index predictable?  The
oracle restatement run one sample at a time on a 48 kHz AM signal (carrier
+1.2 kHz, modulation 0.5, 30 dB SNR, after the oracle AGC): per horizon h the
distribution of (true index - index predicted from the state h samples earlier
with the last kicks held), in table cells -- the window a candidate batch must
cover.  CPU only (oracle)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import oracle as ora  # noqa: E402

fs, n = 48000.0, int(os.environ.get("N", "60000"))
rng = np.random.default_rng(4)
t = np.arange(n) / fs
msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t) + np.sin(2 * np.pi * 2500 * t)) / 3
x = 0.1 * (1 + 0.5 * msg) * np.exp(1j * (2 * np.pi * 1200 * t + 0.3))
x = (x + 0.1 * 10 ** (-30 / 20) / np.sqrt(2) * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
agc = ora.AGC()
agc.scale = np.float32(0.01)
y = agc(x)
am = ora.AmpModem(mod_index=0.5, type="dsb", carrier=True)
th = np.empty(n + 1, np.uint64)
dd = np.empty(n + 1, np.uint64)
th[0], dd[0] = am.pll_state
for i in range(n):
    am(y[i:i + 1])
    th[i + 1], dd[i + 1] = am.pll_state
M = 1 << 32
k1 = (dd[1:].astype(np.int64) - dd[:-1].astype(np.int64)) % M
k2 = (th[1:].astype(np.int64) - th[:-1].astype(np.int64) - dd[1:].astype(np.int64)) % M
tidx = lambda v: ((v + (1 << 21)) >> 22) & 1023
skip = 5000                     # after acquisition
print(f"samples {n}, after {skip}: per-sample k2 spread (cells) p1/p50/p99:",
      np.percentile(((k2[skip:] + M // 2) % M - M // 2) / 2 ** 22, [1, 50, 99]).round(2))
for h in (1, 2, 4, 5, 7, 8, 12, 16):
    i = np.arange(max(skip, 1), n - h)
    k1h = k1[i - 1].astype(np.int64)
    k2h = k2[i - 1].astype(np.int64)
    pred = (th[i].astype(np.int64) + h * (k2h + dd[i].astype(np.int64)) + k1h * (h * (h + 1) // 2)) % M
    e = (tidx(th[i + h].astype(np.int64)) - tidx(pred) + 512) % 1024 - 512
    q = np.percentile(np.abs(e), [50, 90, 99, 99.9])
    print(f"h={h:2d}  |err| cells p50 {q[0]:.0f}  p90 {q[1]:.0f}  p99 {q[2]:.0f}  p99.9 {q[3]:.0f}  "
          f"within +-8: {np.mean(np.abs(e) <= 7):.3f}  +-16: {np.mean(np.abs(e) <= 15):.3f}  +-32: {np.mean(np.abs(e) <= 31):.3f}")

# predictor variants for the one-wave kernel's horizons (4..7): the last kicks
# held (k_pll_seqc), no phase kick (k2 = 0, k1 held), kicks averaged over the
# last 4 samples; share of batches whose 4 samples all fall in a 16-cell window
print("batch of 4 at horizons 4..7, all four within the 16-cell window (-8..+7):")
i = np.arange(max(skip, 8), n - 8)
def batch_hit(k1h, k2h):
    ok = np.ones(i.size, bool)
    for h in (4, 5, 6, 7):
        pred = (th[i].astype(np.int64) + h * (k2h + dd[i].astype(np.int64)) + k1h * (h * (h + 1) // 2)) % M
        e = (tidx(th[i + h].astype(np.int64)) - tidx(pred) + 512) % 1024 - 512
        ok &= (e >= -8) & (e <= 7)
    return ok.mean()
s64 = lambda v: (v.astype(np.int64) + M // 2) % M - M // 2
print("  last kicks held:", round(batch_hit(s64(k1[i - 1]), s64(k2[i - 1])), 3))
print("  k2 = 0, k1 held:", round(batch_hit(s64(k1[i - 1]), 0 * i), 3))
avg = lambda k: np.mean([s64(k[i - j]) for j in range(1, 5)], axis=0).astype(np.int64)
print("  kicks averaged over 4:", round(batch_hit(avg(k1), avg(k2)), 3))
avg8 = lambda k: np.mean([s64(k[i - j]) for j in range(1, 9)], axis=0).astype(np.int64)
print("  kicks averaged over 8:", round(batch_hit(avg8(k1), avg8(k2)), 3))

# expected directly-evaluated samples per batch (k_pll_seqc evaluates a step
# whose index is outside its window itself) for ways of splitting the 64 lanes
# into the 4 samples' windows (horizons 4..7)
print("missed samples per batch of 4 by window split (lanes per horizon 4, 5, 6, 7):")
k1h, k2h = s64(k1[i - 1]), s64(k2[i - 1])
errs = []
for h in (4, 5, 6, 7):
    pred = (th[i].astype(np.int64) + h * (k2h + dd[i].astype(np.int64)) + k1h * (h * (h + 1) // 2)) % M
    errs.append((tidx(th[i + h].astype(np.int64)) - tidx(pred) + 512) % 1024 - 512)
for split in ((16, 16, 16, 16), (12, 14, 18, 20), (10, 14, 18, 22), (8, 12, 20, 24), (8, 14, 18, 24)):
    miss = sum(np.mean((e < -(w // 2)) | (e > w - w // 2 - 1)) for e, w in zip(errs, split))
    print(f"  {split}: {miss:.3f}")
