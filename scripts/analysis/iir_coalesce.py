"""Do float32 DF-II trajectories of the chain's cheby2 order-8 lowpass (BASELINE
C4: Fc = 15 kHz / 2 MS/s, the restatement's exact iirfilt) started W samples
before a chunk from zero state coalesce bit for bit with the true trajectory
by the chunk's start?  The speculative exact chunks of k_iir_spec rely on it
(their verifier re-runs any chunk that does not).  Per W: the share of chunks
whose first C outputs are all bit-identical to the sequential run's.
CPU only (oracle).  python iir_coalesce.py [n_chunks]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
from oracle import oracle as O  # noqa: E402

nchunk = int(sys.argv[1]) if len(sys.argv) > 1 else 200
n = 1 << 23
fs = 2.0e6
t = np.arange(n, dtype=np.float64) / fs
msg = (np.sin(2 * np.pi * 400 * t) + np.sin(2 * np.pi * 1000 * t) + np.sin(2 * np.pi * 2500 * t)) / 3
ph = 2 * np.pi * 1200 * t + 0.3
amp = 0.1 * (1 + 0.5 * msg)
rng = np.random.default_rng(4)
sigma = 0.1 * 10 ** (-30 / 20) / np.sqrt(2)
x = ((amp * np.cos(ph)).astype(np.float32) + 1j * (amp * np.sin(ph)).astype(np.float32)
     + sigma * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
proto = ("cheby2", "lowpass", O.FMT_SOS, 8, np.float32(15000 / 2e6), 0.0, 0.7, 60.0)
ref = O.IIRFilter(prototype=proto)(x)
C = 256
starts = np.linspace(40000, n - C - 1, nchunk).astype(np.int64)
print(f"{nchunk} chunks of {C} outputs over {n} samples of the C4 IQ input")
for W in (1024, 2048, 4096, 6144, 8192, 12288, 16384, 24576, 32768):
    ok = 0
    first = []
    for s in starts:
        f = O.IIRFilter(prototype=proto)
        y = f(x[s - W:s + C])
        eq = y.view(np.uint64)[W:] == ref.view(np.uint64)[s:s + C]
        ok += bool(eq.all())
        # how far into the warm-up the trajectories agree from there on
        e = y.view(np.uint64) == ref.view(np.uint64)[s - W:s + C]
        bad = np.nonzero(~e)[0]
        first.append(W + C if bad.size == 0 else (W + C - 1 - bad[-1]))
    first = np.array(first)
    print(f"W {W:6d}: chunks bit-identical {ok}/{nchunk} ({100.0 * ok / nchunk:.1f} %); "
          f"samples from the last difference to the chunk end: min {first.min()} median {int(np.median(first))}",
          flush=True)
