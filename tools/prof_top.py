"""Print per-iteration kernel totals from a rocprofv3 --stats directory: prof_top.py <dir> [steps] [filter...]"""
import csv
import sys
from pathlib import Path

d, steps = Path(sys.argv[1]), float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
flt = sys.argv[3:]
rows = list(csv.DictReader(open(next(d.glob("*kernel_stats.csv")))))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6 / steps:.2f} ms/iter")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if flt and not any(k in r["Name"] for k in flt):
        continue
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:7.3f} {int(r['Calls']) / steps:6.1f} "
          f"{float(r['AverageNs']) / 1e3:8.1f}  {r['Name'][:100]}")
