"""Per-kernel sums of the PMC counters in a rocprofv3 run_results.db (rocpd SQLite output).

    python tools/pmc_db.py gpurun_out/<dir>/run_results.db [kernel-substring]
"""
import collections
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in con.execute("pragma table_info(counters_collection)")]
kcol = next(c for c in cols if c.lower() in ("kernel_name", "name"))
ncol = next(c for c in cols if c.lower() in ("counter_name",))
vcol = next(c for c in cols if c.lower() in ("counter_value", "value"))
sums = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
for k, n, v in con.execute(f"select {kcol}, {ncol}, {vcol} from counters_collection"):
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    sums[k][n] += float(v)
for k, d in sums.items():
    print(k[:90])
    for n, v in sorted(d.items()):
        print(f"    {n:32s} {v:16.0f}")
