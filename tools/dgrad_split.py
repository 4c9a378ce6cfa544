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
        nxt = ks[i + 1][2] if i + 1 < len(ks) else ""
        if "attn_bwd" in prev:
            label = "qkv dgrad (after attention bwd)"
        elif "gemm256_kernel<true, false, 0, 0" in prev:
            label = "fc1 dgrad (+ residual gradient; after fc2's dgrad)"
        elif "gemm256_kernel<true, false, 0, 0" in nxt:
            label = "fc2 dgrad (ReLU mask folded; before fc1's)"
        elif "attn_bwd" in nxt:
            label = "out-proj dgrad (plain; before attention bwd)"
        else:
            label = f"dgrad between {prev[:30]} and {nxt[:30]}"
        groups[label].append(b - a)
    elif "gemm256_kernel<true, true, 0, 0" in n and g == 524288:
        groups["fwd out/fc2 (K 4096)"].append(b - a)
    elif "gemm256_kernel<true, true, 0, 1" in n and g == 524288:
        groups["fwd fc1 relu+dropout"].append(b - a)
for k, v in sorted(groups.items()):
    q = statistics.quantiles(v, n=10) if len(v) > 1 else [v[0]] * 9
    print(f"{k:<52} n={len(v):5d} median {statistics.median(v) / 1e3:8.1f} us  p10 {q[0] / 1e3:8.1f}  "
          f"p90 {q[-1] / 1e3:8.1f}")
