"""Summarise a rocprofv3 --stats kernel CSV: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU kernel time: {tot / 1e6:.2f} ms over {sum(int(r['Calls']) for r in rows)} dispatches")
print(f"{'ms':>9s} {'%':>6s} {'calls':>6s} {'avg us':>9s}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    name = r["Name"]
    if len(name) > 100:
        name = name[:100] + "..."
    print(f"{float(r['TotalDurationNs']) / 1e6:9.2f} {float(r['Percentage']):6.2f} {int(r['Calls']):6d} "
          f"{float(r['AverageNs']) / 1e3:9.1f}  {name}")
