"""Average counter values per kernel over every counter_collection.csv under a
directory (scripts/iir_pmc.sh, fir_pmc.sh): {kernel: {counter: mean}}."""
import csv, glob, json, os, re, sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)(<[^>]*>)?", r["Kernel_Name"])
        k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)(<[^>]*>)?", r["Name"])
        k = (m.group(1) + (m.group(2) or "")) if m else r["Name"][:40]
        acc[k]["avg_ns"].append(float(r["AverageNs"]))
print(json.dumps({k: {c: round(sum(v) / len(v), 1) for c, v in d.items()} for k, d in acc.items()
                  if k.startswith("k_")}, indent=1))
