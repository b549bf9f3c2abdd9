import os, sys, time
REPO = os.getcwd()
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "python-liquiddsp_amd")]
import numpy as np, torch, liquiddsp as L
n = 1 << 20
rng = np.random.default_rng(1)
x = (np.exp(1j * rng.standard_normal(n).cumsum() * 0.3)).astype(np.complex64)
xd = torch.from_numpy(x).cuda()
f = L.FMStereo()
f(xd); torch.cuda.synchronize()
t0 = time.perf_counter(); f(xd); torch.cuda.synchronize(); el = time.perf_counter() - t0
print(os.environ.get("LDSP_PKG_DIR", "product"), f"{n / el / 1e6:.2f} MS/s")
