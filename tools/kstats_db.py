"""Per-kernel call count / total / average duration from a rocprofv3 run_results.db (rocpd SQLite output).

    python tools/kstats_db.py gpurun_out/<dir>/run_results.db [name-substring]
"""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
name = next(c for c in ("kernel_name", "name") if c in cols)
rows = con.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start) "
                   f"from kernels group by {name} order by sum(end - start) desc").fetchall()
total = sum(r[2] for r in rows)
print(f"{'calls':>6} {'total us':>10} {'avg us':>9} {'min us':>9} {'%':>6}  kernel")
for k, n, tot, avg, mn in rows:
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    print(f"{n:6d} {tot / 1e3:10.1f} {avg / 1e3:9.1f} {mn / 1e3:9.1f} {100 * tot / total:6.2f}  {k[:110]}")
