"""Summarise an LDSP_PROF_TIMELINE file (name stream start_ms end_ms per
profiled launch): for every k_pll_walk, the gap since the previous walk ended
and which of its same-stream predecessors ended last."""
import sys
from collections import defaultdict

rows = [l.split() for l in open(sys.argv[1]) if l.strip()]
rows = [(n, s, float(a), float(b)) for n, s, a, b in rows]
rows.sort(key=lambda r: r[2])
walks = [r for r in rows if r[0] == "k_pll_walk"]
prev_end = None
for w in walks:
    same = [r for r in rows if r[1] == w[1] and r[3] <= w[2] + 1e-6 and r is not w]
    last = max(same, key=lambda r: r[3]) if same else None
    gap = (w[2] - prev_end) if prev_end is not None else float("nan")
    print(f"walk {w[1][-6:]} start {w[2]:9.3f} dur {w[3]-w[2]:6.3f} gap {gap:7.3f}  "
          f"last same-stream before: {last[0] if last else '-'} ended {last[3] if last else 0:9.3f}")
    prev_end = w[3]
busy = defaultdict(float)
for n, s, a, b in rows:
    busy[n] += b - a
span = rows[-1][3] - rows[0][2]
print(f"span {span:.3f} ms; walks {len(walks)}; per-kernel busy ms:",
      {k: round(v, 3) for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:8]})
