"""Host side of the multi-channel component: how long the Python loop takes to
enqueue one step of 8 AMRadio chains (fused front, 2 streams per channel) against
the step's wall time, and the same step issued from one host thread per channel
(the C ABI releases the GIL)."""
import json
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR", os.path.join(REPO, "python-liquiddsp_amd"))]
import bench  # noqa: E402
import torch  # noqa: E402
import liquiddsp as L  # noqa: E402

dev = torch.device("cuda", 0)
C, per, n, steps = 8, 2, 64 << 20, 10
xs = [bench.synth_channel(n, r, dev) for r in range(C)]
radios = [bench.AMRadio(L, fused_front=True) for _ in range(C)]
strm = [[torch.cuda.Stream(dev) for _ in range(per)] for _ in range(C)]


def one(c, k):
    with torch.cuda.stream(strm[c][k % per]):
        radios[c](xs[c])


def run(threaded):
    for k in range(2 * per):
        for c in range(C):
            one(c, k)
    torch.cuda.synchronize()
    enq = []
    t0 = time.perf_counter()
    for k in range(steps):
        a = time.perf_counter()
        if threaded:
            th = [threading.Thread(target=one, args=(c, k)) for c in range(C)]
            for t in th:
                t.start()
            for t in th:
                t.join()
        else:
            for c in range(C):
                one(c, k)
        enq.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    return {"threaded": threaded, "ms_per_step": round(t / steps * 1e3, 3), "enqueue_ms_per_step": round(sum(enq) / steps * 1e3, 3),
            "Msamples_s": round(C * n * steps / t / 1e6, 1)}


for th in (False, True, False):
    print(json.dumps(run(th)), flush=True)
