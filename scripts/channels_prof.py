"""Per-kernel times (libldsp HIP events on each launch's stream) inside the
multi-channel component: N AMRadio chains (fused front, 2 streams each) on one
GPU, against one chain alone -- which kernels stretch when the channels share the GPU.
    python channels_prof.py [channels ...]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
import bench  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
n, per, steps = 64 << 20, 2, 8
counts = [int(a) for a in sys.argv[1:]] or [1, 8]
xs = [bench.synth_channel(n, r, dev) for r in range(max(counts))]
strm = [[torch.cuda.Stream(dev) for _ in range(per)] for _ in range(max(counts))]
for C in counts:
    radios = [bench.AMRadio(L, fused_front=True) for _ in range(C)]
    for k in range(2 * per):
        for c in range(C):
            with torch.cuda.stream(strm[c][k % per]):
                radios[c](xs[c])
    torch.cuda.synchronize()
    L._profile_reset()
    L._profile_enable(True)
    t0 = time.perf_counter()
    for k in range(steps):
        for c in range(C):
            with torch.cuda.stream(strm[c][k % per]):
                radios[c](xs[c])
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    L._profile_enable(False)
    rep = {k: round(v[1] / v[0], 4) for k, v in L._profile_report().items()}
    print(json.dumps({"channels": C, "ms_per_step": round(t / steps * 1e3, 3), "kernel_ms": rep}), flush=True)
    del radios
