"""Forward-GEMM timing at the enc12 T=8192 shapes for ONE setting of the
block-ordering group (MIPIPE_GEMM_G, read once per process) -- run it once per
value and compare:

    for g in 4 8 16 32; do MIPIPE_GEMM_G=$g python tools/gemm_group_sweep.py; done
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()


def timeit(fn, iters=30):
    for _ in range(5):
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
    return statistics.median(ts)


xw = torch.randn(4096, 4096, device="cuda").to(torch.bfloat16)
for _ in range(300):  # warm clocks
    k.linear_fwd(xw, xw, None, 0, 0.0, False)
g = os.environ.get("MIPIPE_GEMM_G", "default")
for name, M, N, K in [("qkv fwd", 8192, 12288, 4096), ("out fwd", 8192, 4096, 4096), ("dec fwd", 8192, 28928, 4096)]:
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    t = timeit(lambda: k.linear_fwd(x, w, b, 0, 0.0, False))
    print(f"G={g:8s} {name:8s} {M}x{N}x{K}: {t * 1e3:8.1f} us {2.0 * M * N * K / t / 1e9:7.0f} TF/s", flush=True)
