"""Print a kernel timeline (start/end relative to the first dispatch shown, in
microseconds, per queue) from a rocprofv3 --kernel-trace CSV:
    python scripts/timeline.py <dir>/<name>_kernel_trace.csv [first_kernel_regex] [count]"""
import csv
import re
import sys

path = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_pll_walk"
count = int(sys.argv[3]) if len(sys.argv) > 3 else 80
rows = []
for r in csv.DictReader(open(path)):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), m.group(1) if m else r["Kernel_Name"][:30],
                 r.get("Queue_Id", r.get("Stream_Id", "?"))))
rows.sort()
idx = [i for i, r in enumerate(rows) if re.search(first, r[2])]
if len(idx) > 3:
    i0 = idx[-4]          # a late occurrence (steady state)
else:
    i0 = idx[0] if idx else 0
t0 = rows[i0][0]
for s, e, n, q in rows[max(0, i0 - 20):i0 + count]:
    print(f"q{q:>3} {n:24s} start={(s - t0) / 1e3:10.1f} end={(e - t0) / 1e3:10.1f} dur={(e - s) / 1e3:9.1f}")
