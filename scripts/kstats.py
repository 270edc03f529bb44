"""Summarise a rocprofv3 kernel_stats.csv: top kernels with per-call average (us) and share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
print("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
for x in rows[:n]:
    print(f"| `{x['Name'][:100]}` | {x['Calls']} | {float(x['TotalDurationNs']) / 1e6:.2f} | "
          f"{float(x['AverageNs']) / 1e3:.2f} | {float(x['Percentage']):.1f} |")
