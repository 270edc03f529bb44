"""Summarise rocprofv3 --pmc counter_collection.csv: per kernel, the mean of each counter."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName") or "?"
    cname = r.get("Counter_Name") or r.get("Counter-Name")
    val = float(r.get("Counter_Value") or r.get("Counter-Value") or 0)
    agg[name][cname].append(val)
counters = sorted({c for k in agg.values() for c in k})
print("| kernel | " + " | ".join(counters) + " |")
print("|---|" + "---|" * len(counters))
for name, cs in agg.items():
    vals = []
    for c in counters:
        v = cs.get(c, [])
        vals.append(f"{sum(v) / len(v):.4g}" if v else "")
    print(f"| `{name[:70]}` | " + " | ".join(vals) + " |")
