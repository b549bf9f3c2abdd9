"""Config 3's launch-to-launch spread: per launch of the
fused NCO + FFT FIR kernel at 256 Mi, its duration (kernel trace) and the GPU's
busy cycles in the same launch of a separate pass (GRBM_GUI_ACTIVE; kernels in
the same order), so cycles / duration is the clock the launch ran at; and the SQ
issue counters of the fused and plain kernels at the same size.
    python c3_spread.py <scripts/fir_c3_pmc.sh output dir>"""
import csv
import glob
import json
import os
import sys

root = sys.argv[1]


def rows(sub, pat):
    out = []
    for f in glob.glob(os.path.join(root, sub, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def kind(name, grid):
    if "k_fir_fft1024x" not in name or int(grid) != 196352:
        return None
    return "fused" if "k_fir_fft1024x<true" in name else "plain"


tr = [r for r in rows("trace", "*kernel_trace.csv")]
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = {"fused": [], "plain": []}
for r in tr:
    g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    k = kind(r["Kernel_Name"], g)
    if k:
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def counters(sub):
    per = {}
    for r in rows(sub, "*counter_collection.csv"):
        k = kind(r["Kernel_Name"], r["Grid_Size"])
        if k:
            per.setdefault((k, int(r["Dispatch_Id"])), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    out = {"fused": [], "plain": []}
    for (k, d) in sorted(per):
        out[k].append(per[(k, d)])
    return out


gr = counters("grbm")
res = {"what": __doc__.split("\n\n")[0].replace("\n", " ")}
for k in ("plain", "fused"):
    d = dur[k]
    g = gr[k]
    n = min(len(d), len(g))
    mhz = [round(g[i]["GRBM_GUI_ACTIVE"] / d[i], 1) for i in range(n)]   # cycles per us = MHz
    res[k] = {"durations_us": [round(v, 1) for v in d], "gui_active_MHz_per_launch": mhz,
              "duration_min_max_us": [round(min(d), 1), round(max(d), 1)] if d else None}
for sub in ("sq", "sq2", "lds"):
    c = counters(sub)
    for k in ("plain", "fused"):
        if c[k]:
            keys = c[k][0].keys()
            res.setdefault(k, {})[sub] = {q: round(sum(x[q] for x in c[k]) / len(c[k])) for q in keys}
print(json.dumps(res, indent=1))
