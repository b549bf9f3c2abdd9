import sys, numpy as np
sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", ".."))
from oracle import oracle as O
n = 1 << 22; fs = 600000.0
rng = np.random.default_rng(1)
t = np.arange(n) / fs
left, right = np.sin(2*np.pi*1000*t), 0.5*np.sin(2*np.pi*3000*t)
comp = 0.45*(left+right) + 0.45*(left-right)*np.cos(2*np.pi*38000*t) + 0.1*np.cos(2*np.pi*19000*t)
x = (np.exp(2j*np.pi*(75000/fs)*np.cumsum(comp)) + 0.01*(rng.standard_normal(n)+1j*rng.standard_normal(n))/np.sqrt(2)).astype(np.complex64)
O.FreqDem(4.0)(x).astype(np.float32).tofile("fm_s.f32")
xn = (rng.standard_normal(n) + 1j*rng.standard_normal(n)).astype(np.complex64)
O.FreqDem(4.0)(xn).astype(np.float32).tofile("fmn_s.f32")
