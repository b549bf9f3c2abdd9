"""Walk-to-walk gaps from a rocprofv3 kernel trace (analysis tooling).

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- python3 bench.py ...
    python scripts/walk_gaps.py D/<...>/run_kernel_trace.csv

Prints, for the last call's steady state, the time from each k_pll_walk's end
to the next one's start and which kernels started or ran in that gap, plus the
span of the whole trace section from the first kernel to the last walk.
"""
import collections
import csv
import sys


def short(name):
    for pre in ("void ", "ldsp::k::(anonymous namespace)::", "(anonymous namespace)::"):
        name = name.replace(pre, "")
    return name.split("(")[0].split("<")[0]


def main(path, last=30):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    walks = [r for r in rows if r[2] == "k_pll_walk"]
    walks = walks[-last:]
    gaps = []
    for a, b in zip(walks, walks[1:]):
        g = b[0] - a[1]
        inside = collections.Counter(r[2] for r in rows if a[1] <= r[0] < b[0])
        gaps.append(g)
        print(f"walk {(a[1]-a[0])/1e3:8.1f} us  gap {g/1e3:7.1f} us  started in gap: "
              + ", ".join(f"{k}x{v}" for k, v in inside.most_common(6)))
    if gaps:
        gaps.sort()
        print(f"walks {len(walks)}: mean walk {sum(w[1]-w[0] for w in walks)/len(walks)/1e3:.1f} us, "
              f"gap median {gaps[len(gaps)//2]/1e3:.1f} us, mean {sum(gaps)/len(gaps)/1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)
