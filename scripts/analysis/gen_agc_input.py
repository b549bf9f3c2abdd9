import sys, numpy as np, time
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", ".."))
from oracle import oracle as O
n = 1 << 26
fs = 2.0e6
t = np.arange(n, dtype=np.float64) / fs
msg = (np.sin(2*np.pi*400*t) + np.sin(2*np.pi*1000*t) + np.sin(2*np.pi*2500*t)) / 3
ph = 2*np.pi*1200*t + 0.3
amp = 0.1*(1 + 0.5*msg)
rng = np.random.default_rng(4)
sigma = 0.1 * 10**(-30/20) / np.sqrt(2)
x = ((amp*np.cos(ph)).astype(np.float32) + 1j*(amp*np.sin(ph)).astype(np.float32) + sigma*(rng.standard_normal(n)+1j*rng.standard_normal(n))).astype(np.complex64)
t0 = time.time()
iir = O.IIRFilter(prototype=("cheby2", "lowpass", O.FMT_SOS, 8, 15000/2e6, 0.0, 0.5, 60.0))
y = iir(x)
rs = O.Resampler(np.float32(48000/2e6), 20, 48000/2e6, 60.0, 13)
z = rs(y)
print(len(z), time.time()-t0)
z.tofile("agc_in.c64")
agc = O.AGC(); agc.lock(False); agc.scale = 0.01
a = agc(z)
a.tofile("am_in.c64")
