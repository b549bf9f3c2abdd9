"""Per-kernel summary of a prof_round.sh directory: average duration (kernel
trace) and HBM bytes per launch from FETCH_SIZE / WRITE_SIZE.

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE (KB) reports half the
bytes of a wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024;
WRITE_SIZE (KB) is exact for streaming stores: write bytes = WRITE_SIZE * 1024.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    if not m:
        return name[:60]
    if m.group(1) == "k_iir_blk" and m.group(2):      # k_iir_blk<NC, D, FINAL, ...>
        return "k_iir_blk_final" if "true" in m.group(2) else "k_iir_blk_local"
    return m.group(1)


def stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    return out


def counters(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def shape_key(name, grid):
    """kernel + template arguments + grid size: one launch shape (the FIR runs
    launch one kernel at several sizes, whose per-launch averages must not mix)"""
    m = re.search(r"(k_\w+)(<[^>]*>)?", name)
    base = (m.group(1) + (m.group(2) or "")) if m else name[:60]
    return f"{base}@{grid}"


def by_shape(root, run):
    """{shape: {calls, avg_us, fetch_bytes_corrected, write_bytes, hbm_bytes, hbm_GBs}}"""
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(root, f"{run}_trace", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_" not in r["Kernel_Name"]:
                continue
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            dur[shape_key(r["Kernel_Name"], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {}
    for counter, field, scale in (("FETCH_SIZE", "fetch_bytes_corrected", 2048.0), ("WRITE_SIZE", "write_bytes", 1024.0)):
        acc = defaultdict(list)
        for f in glob.glob(os.path.join(root, f"{run}_{counter.split('_')[0].lower()}", "**", "*counter_collection.csv"),
                           recursive=True):
            for r in csv.DictReader(open(f)):
                if r.get("Counter_Name") == counter and "k_" in r["Kernel_Name"]:
                    acc[shape_key(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            out.setdefault(k, {})[field] = scale * sum(v) / len(v)
    for k, v in dur.items():
        out.setdefault(k, {}).update(calls=len(v), avg_us=round(sum(v) / len(v), 2))
    for e in out.values():
        if "fetch_bytes_corrected" in e and "write_bytes" in e and "avg_us" in e:
            e["hbm_bytes"] = e["fetch_bytes_corrected"] + e["write_bytes"]
            e["hbm_GBs"] = round(e["hbm_bytes"] / (e["avg_us"] * 1e3), 1)
    return out


def main(root):
    res = {}
    for run in ("fir", "front"):
        if glob.glob(os.path.join(root, f"{run}_trace")):
            res[f"{run}_by_shape"] = by_shape(root, run)
    for run in ("bench", "fir", "front"):
        st = stats(os.path.join(root, f"{run}_trace"))
        fe = counters(os.path.join(root, f"{run}_fetch"), "FETCH_SIZE")
        wr = counters(os.path.join(root, f"{run}_write"), "WRITE_SIZE")
        for k, v in st.items():
            e = dict(v)
            if k in fe:
                e["fetch_bytes_corrected"] = 2.0 * fe[k] * 1024
            if k in wr:
                e["write_bytes"] = wr[k] * 1024
            for cn in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_INSTS_VMEM"):
                sq = counters(os.path.join(root, f"{run}_sq"), cn)
                if k in sq:
                    e[cn.lower()] = round(sq[k])
            if "fetch_bytes_corrected" in e and "write_bytes" in e:
                e["hbm_bytes"] = e["fetch_bytes_corrected"] + e["write_bytes"]
                e["hbm_GBs"] = round(e["hbm_bytes"] / (e["avg_us"] * 1e3), 1)
            res.setdefault(run, {})[k] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
