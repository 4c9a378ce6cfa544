"""Reads the rocprofv3 database of tools/micro/small_copy_probe.hip: for each (copy kind, size) group between
two marker kernels, how many __amd_rocclr_copyBuffer kernels ran (copies on the CUs) and how many DMA copies
(the memory-copy trace) -- i.e. the size from which the runtime stops turning a copy into a kernel."""
import glob
import sqlite3
import sys

ipc = "--ipc" in sys.argv
dbs = sorted(p for p in glob.glob(sys.argv[1], recursive=True))
ks, cps = [], []
for db in dbs:  # a forked child may write its own database
    c = sqlite3.connect(db)
    ks += c.execute("select start, name from kernels order by start").fetchall()
    cps += c.execute("select start, size from memory_copies order by start").fetchall()
ks.sort()
cps.sort()
marks = [(a, n) for a, n in ks if "marker" in n]
names = ["IPC_NoCU"] if ipc else ["D2D_NoCU", "D2D"]
sizes = [8, 4096, 65536, 262144, 1048576, 4194304, "8 (4K->4K)", "8 (4K->8M)", "8 (8M->4K)"] if ipc else [8, 64, 1024, 4096, 16384, 65536, 262144, 1048576,
                                                                  4194304]
print(f"{'kind':<10} {'bytes':>9} {'copy kernels':>13} {'DMA copies':>11}")
for j, (t0, _) in enumerate(marks):
    t1 = marks[j + 1][0] if j + 1 < len(marks) else float("inf")
    nk = sum(1 for a, n in ks if t0 < a < t1 and "copyBuffer" in n)
    nd = sum(1 for a, z in cps if t0 < a < t1)
    k, i = divmod(j, len(sizes))
    if k >= len(names):
        break
    print(f"{names[k]:<10} {sizes[i]:>9} {nk:>13} {nd:>11}")
