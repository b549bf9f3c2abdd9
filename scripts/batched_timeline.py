"""Kernel timeline of the batched 8-channel component (bench.multi_channel_batched)
on the tuning build: every launch's start / end (HIP events, LDSP_PROF_TIMELINE),
summarised per kernel (count, busy ms) and as the walks' spans per step.
    LDSP_PKG_DIR=build_tuning LDSP_PROF_TIMELINE=tlb.txt python3 scripts/batched_timeline.py"""
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.environ.get("LDSP_PKG_DIR") or os.path.join(REPO, "build_tuning")]
import torch  # noqa: E402
import bench  # noqa: E402
import liquiddsp as L  # noqa: E402

tl = os.environ["LDSP_PROF_TIMELINE"]
dev = torch.device("cuda", 0)
bs = [torch.cuda.Stream(dev) for _ in range(4)]
bench.multi_channel_batched(L, dev, 8, steps=4, strm=bs)        # warm-up (allocations, objects)
open(tl, "w").close()
L._profile_reset()
L._profile_enable(True)
r = bench.multi_channel_batched(L, dev, 8, steps=10, strm=bs)
torch.cuda.synchronize()
L._profile_enable(False)
L._profile_report()
rows = sorted(((n, s, float(a), float(b)) for n, s, a, b in (l.split() for l in open(tl) if l.strip())),
              key=lambda t: t[2])
t0 = rows[0][2]
busy, cnt = defaultdict(float), defaultdict(int)
for n, s, a, b in rows:
    busy[n] += b - a
    cnt[n] += 1
span = rows[-1][3] - t0
print(json.dumps({"result": r, "span_ms": round(span, 3),
                  "kernels": {k: {"launches": cnt[k], "busy_ms": round(v, 3)} for k, v in
                              sorted(busy.items(), key=lambda kv: -kv[1])}}))
for n, s, a, b in rows:
    print(f"{n:22s} {s[-6:]:>8s} {a - t0:9.3f} {b - t0:9.3f} {b - a:7.3f}")
