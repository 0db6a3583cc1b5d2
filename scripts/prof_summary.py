"""Summarise a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time: {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
print(f"{'%':>6} {'total ms':>9} {'calls':>6} {'avg us':>9}  kernel")
for r in rows[:top]:
    name = r["Name"]
    if len(name) > 100:
        name = name[:100] + "…"
    print(f"{float(r['Percentage']):6.2f} {float(r['TotalDurationNs']) / 1e6:9.2f} {int(r['Calls']):6d} "
          f"{float(r['AverageNs']) / 1e3:9.1f}  {name}")
