"""Per-block kernel timeline of the README small-call path from a rocprofv3
kernel trace (scripts/block_trace.sh): the blocks are delimited by launches
of FIRST (default k_iir_modal); for each kernel of a block its start offset,
duration and the idle gap before it, averaged over the traced blocks after
SKIP warm-up blocks.  usage: python3 scripts/block_timeline.py DIR [FIRST] [SKIP]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "k_iir_modal"
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(k_\w+)", r["Kernel_Name"])
            rows.append((m.group(1) if m else r["Kernel_Name"][:24], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda r: r[1])
    starts = [i for i, r in enumerate(rows) if r[0] == first]
    blocks = [rows[a:b] for a, b in zip(starts[:-1], starts[1:])][skip:]
    if not blocks:
        print("no blocks")
        return
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])   # key -> count, start, dur, gap
    span = 0.0
    for blk in blocks:
        t0 = blk[0][1]
        prev_end = t0
        seen = defaultdict(int)
        for name, a, b in blk:
            seen[name] += 1
            key = (name, seen[name])
            e = agg[key]
            e[0] += 1
            e[1] += (a - t0) / 1e3
            e[2] += (b - a) / 1e3
            e[3] += max(0, a - prev_end) / 1e3
            prev_end = max(prev_end, b)
        span += (prev_end - t0) / 1e3
    nb = len(blocks)
    period = (blocks[-1][0][1] - blocks[0][0][1]) / 1e3 / max(1, nb - 1)
    print(f"blocks {nb}, block period {period:.1f} us, first-to-last-end per block {span / nb:.1f} us")
    print(f"{'kernel':28s}{'#':>3s}{'start_us':>10s}{'dur_us':>9s}{'gap_us':>9s}")
    tot_d = tot_g = 0.0
    for (name, k), (c, s, d, g) in sorted(agg.items(), key=lambda kv: kv[1][1] / kv[1][0]):
        print(f"{name:28s}{k:3d}{s / c:10.1f}{d / c:9.1f}{g / c:9.1f}" + ("" if c == nb else f"   (in {c} blocks)"))
        tot_d += d / nb
        tot_g += g / nb
    print(f"sum of durations {tot_d:.1f} us, sum of gaps {tot_g:.1f} us")


if __name__ == "__main__":
    main()
