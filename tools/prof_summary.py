"""Summarise a rocprofv3 kernel profile: top kernels by total time.

Accepts either the ``--stats`` CSV (``*_kernel_stats.csv``) or the rocpd SQLite
database (``*_results.db``, rocprofv3's default output format).  With a DB,
``--by-grid`` additionally splits each kernel by launch grid (e.g. GEMM shapes).

    python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv 30
    python tools/prof_summary.py gpurun_out/prof/run_results.db 30 --by-grid
"""
import csv
import sqlite3
import sys


def _short(name: str, n: int = 100) -> str:
    return name if len(name) <= n else name[:n] + "..."


def from_csv(path):
    rows = list(csv.DictReader(open(path)))
    return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in rows]


def from_db(path, by_grid):
    c = sqlite3.connect(path)
    if by_grid:
        q = ("select name || ' [grid ' || grid_x || 'x' || grid_y || 'x' || grid_z || ']', count(*), sum(duration) "
             "from kernels group by name, grid_x, grid_y, grid_z")
    else:
        q = "select name, count(*), sum(duration) from kernels group by name"
    return [(n, int(k), float(d)) for n, k, d in c.execute(q)]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    by_grid = "--by-grid" in sys.argv
    path = args[0]
    top = int(args[1]) if len(args) > 1 else 30
    rows = from_db(path, by_grid) if path.endswith(".db") else from_csv(path)
    tot = sum(r[2] for r in rows)
    print(f"total GPU kernel time: {tot / 1e6:.2f} ms over {sum(r[1] for r in rows)} dispatches")
    print(f"{'ms':>9s} {'%':>6s} {'calls':>6s} {'avg us':>9s}  kernel")
    for name, calls, ns in sorted(rows, key=lambda r: -r[2])[:top]:
        print(f"{ns / 1e6:9.2f} {100 * ns / tot:6.2f} {calls:6d} {ns / calls / 1e3:9.1f}  {_short(name, 130)}")


if __name__ == "__main__":
    main()
