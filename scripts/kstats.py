"""Summarise a rocprofv3 *_kernel_stats.csv: top kernels by total time (names shortened)."""
import csv
import os
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} launches")
for r in rows[:n]:
    name = r["Name"]
    name = re.sub(r"\(.*", "", name) if not name.startswith("_ZN") else name[:60]
    name = (name.replace("prec::", "") if os.environ.get("KEEP_T") else re.sub(r"<.*", "", name))[:90]
    print(f"{float(r['TotalDurationNs']) / 1e6:9.1f} ms {int(r['Calls']):>7} {float(r['AverageNs']) / 1e3:9.1f} us "
          f"{float(r['Percentage']):5.1f}%  {name}")
