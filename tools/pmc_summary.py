"""Mean PMC counter values per kernel (rocprofv3 --pmc counter_collection CSV).

    python tools/pmc_summary.py gpurun_out/pmc/run_counter_collection.csv [name-filter]
"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
order = []
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if filt not in name:
        continue
    key = name if len(name) < 90 else name[:90]
    if key not in vals:
        order.append(key)
    vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key in order:
    cs = vals[key]
    n = len(next(iter(cs.values())))
    print(f"{key}  (x{n})")
    for c, v in sorted(cs.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.0f}")
