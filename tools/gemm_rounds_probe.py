"""Multi-round GEMM probe: one launch of 4096 x 12288 x 4096 (768 tiles = 3 rounds of the 256
CUs) vs three back-to-back launches of 4096 x 4096 x 4096 (one round each) on the same data,
and the same for the LM-head shape.  Per-round cost tells whether round transitions inside one
launch cost more than launch boundaries."""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts) * 1e3


# clocks up before anything is timed (the first timings of a process otherwise read slow)
_x = torch.randn(4096, 4096, device="cuda").to(torch.bfloat16)
for _ in range(300):
    k.linear_fwd(_x, _x, None, 0, 0.0, False)
torch.cuda.synchronize()

for T, N in ((4096, 12288), (4096, 16384), (4096, 28928), (2048, 12288), (2048, 28928)):
    x = torch.randn(T, 4096, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, 4096, device="cuda").to(torch.bfloat16)
    parts = [w[i:i + 4096].contiguous() for i in range(0, N, 4096)]
    ones, autos = [], []
    for _ in range(2):  # alternated, so neither arm always runs first
        k.gemm_set_rounds(1)
        autos.append(timeit(lambda: k.linear_fwd(x, w, None, 0, 0.0, False)))
        k.gemm_set_rounds(0)
        ones.append(timeit(lambda: k.linear_fwd(x, w, None, 0, 0.0, False)))
    k.gemm_set_rounds(1)
    one, auto = min(ones), min(autos)
    split = timeit(lambda: [k.linear_fwd(x, p, None, 0, 0.0, False) for p in parts])
    hb = timeit(lambda: torch.matmul(x, w.t()))
    fl = 2.0 * T * N * 4096
    print(f"{T}x{N}x4096: one launch {one:7.1f} us ({fl / one / 1e6:5.0f} TF/s) | per-round launches (default) "
          f"{auto:7.1f} us ({fl / auto / 1e6:5.0f}) | {len(parts)} separate GEMMs of <=4096 cols {split:7.1f} us "
          f"({fl / split / 1e6:5.0f}) | hipBLASLt {hb:7.1f} us ({fl / hb / 1e6:5.0f})")
