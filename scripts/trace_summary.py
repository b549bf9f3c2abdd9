"""Summarise a rocprofv3 kernel trace (kernel_trace.csv under DIR; optional
window NAME:K = from the K-th launch of kernel NAME on): per kernel
the launch count, total / mean duration and the share of the traced span it
was running on some queue; k_pll_walk launches: the wait between the end of
the previous kernel on their queue and their start."""
import csv, glob, json, os, re, sys
from collections import defaultdict

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:30]
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        rows.append((name, q, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows.sort(key=lambda r: r[2])
if len(sys.argv) > 2:                       # window: from the K-th launch of NAME ("NAME:K") to the end
    name, k = sys.argv[2].split(":")
    starts = [r[2] for r in rows if r[0] == name]
    rows = [r for r in rows if r[2] >= starts[int(k)]]
t0, t1 = rows[0][2], max(r[3] for r in rows)
span = (t1 - t0) / 1e6
tot = defaultdict(float)
cnt = defaultdict(int)
iv = defaultdict(list)
for n, q, a, b in rows:
    tot[n] += (b - a) / 1e6
    cnt[n] += 1
    iv[n].append((a, b))
def union(v):
    v = sorted(v)
    s, ca, cb = 0, None, None
    for a, b in v:
        if ca is None or a > cb:
            if ca is not None:
                s += cb - ca
            ca, cb = a, b
        else:
            cb = max(cb, b)
    return (s + (cb - ca)) / 1e6 if ca is not None else 0.0
res = {"span_ms": round(span, 3), "kernels": {}}
for n in sorted(tot, key=lambda k: -tot[k]):
    res["kernels"][n] = {"calls": cnt[n], "total_ms": round(tot[n], 3), "mean_ms": round(tot[n] / cnt[n], 4),
                         "busy_frac_of_span": round(union(iv[n]) / span, 3)}
byq = defaultdict(list)
for r in rows:
    byq[r[1]].append(r)
waits = []
for q, v in byq.items():
    for i, r in enumerate(v):
        if r[0] == "k_pll_walk" and i > 0:
            waits.append((r[2] - v[i - 1][3]) / 1e3)
if waits:
    waits.sort()
    res["walk_start_wait_us"] = {"n": len(waits), "median": round(waits[len(waits) // 2], 1),
                                 "p90": round(waits[int(len(waits) * 0.9)], 1), "max": round(waits[-1], 1)}
print(json.dumps(res, indent=1))
