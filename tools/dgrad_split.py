"""Which K = 4096 dgrad of the enc12 step is slow?  Labels each dgrad dispatch of a rocprofv3 trace by the
kernel issued right before it on the GPU (enc12 post-norm layer backward order: LN2 bwd -> fc2 dgrad (ReLU mask
folded) -> fc1 dgrad (+ residual gradient) -> LN1 bwd -> out dgrad -> attention bwd -> qkv dgrad (+ residual)),
and prints the duration statistics per label, next to the same-shape forward GEMMs."""
import statistics
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
c = sqlite3.connect(db)
ks = c.execute("select start, end, name, grid_x from kernels order by start").fetchall()
groups = defaultdict(list)
for i, (a, b, n, g) in enumerate(ks):
    if "gemm256_kernel<true, false, 0, 0" in n and g == 524288:
        prev = ks[i - 1][2]
        prevs = ("ln_bwd" if "ln_bwd" in prev else "dgrad" if "gemm256_kernel<true, false, 0, 0" in prev else
                 "attn_bwd" if "attn_bwd" in prev else prev[:40])
        groups[f"dgrad after {prevs}"].append(b - a)
    elif "gemm256_kernel<true, true, 0, 0" in n and g == 524288:
        groups["fwd out/fc2 (K 4096)"].append(b - a)
    elif "gemm256_kernel<true, true, 0, 1" in n and g == 524288:
        groups["fwd fc1 relu+dropout"].append(b - a)
for k, v in sorted(groups.items()):
    print(f"{k:<40} n={len(v):5d} median {statistics.median(v) / 1e3:8.1f} us  mean {statistics.mean(v) / 1e3:8.1f}")
