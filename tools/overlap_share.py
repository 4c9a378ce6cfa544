"""How much of one kernel family's time overlaps other kernels, from a
rocprofv3 kernel trace (rocpd SQLite DB; ``kernels`` view: name, start, end).

    python tools/overlap_share.py gpurun_out/prof/run_results.db adam

Prints the family's summed kernel time, the wall time it covers (union of its
intervals), the part of that union during which some OTHER kernel also ran,
and the device's overall busy union.
"""
import sqlite3
import sys


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    path, key = sys.argv[1], sys.argv[2].lower()
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end from kernels"))
    fam = [(s, e) for n, s, e in rows if key in n.lower()]
    other = [(s, e) for n, s, e in rows if key not in n.lower()]
    fu, ou = union(fam), union(other)
    both = intersect(fu, ou)
    allu = union(fam + other)
    span = (max(e for _, _, e in rows) - min(s for _, s, _ in rows)) if rows else 0
    print(f"{key}: {len(fam)} kernels, {sum(e - s for s, e in fam) / 1e6:.2f} ms summed, union {length(fu) / 1e6:.2f} ms, "
          f"of which {length(both) / 1e6:.2f} ms ({100 * length(both) / max(1, length(fu)):.1f} %) overlap other kernels")
    print(f"device busy union {length(allu) / 1e6:.2f} ms over a {span / 1e6:.2f} ms trace "
          f"({100 * length(allu) / max(1, span):.1f} %); other kernels alone {length(ou) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
