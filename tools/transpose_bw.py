"""transpose_b16 bandwidth at the flush's shapes (x [T, K_in] -> x^T [K_in, T]) vs torch's x.t().contiguous().

    python tools/transpose_bw.py
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
for R, C in [(8192, 4096), (8192, 1600), (8192, 6400), (32768, 4096)]:
    x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
    res = {}
    for name, fn in (("mipipe", lambda: k.transpose_b16(x)), ("torch", lambda: x.t().contiguous())):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / 20 * 1e3
    gb = 2 * R * C * 2 / 1e9
    print(f"{R:6d} x {C:5d}: mipipe {res['mipipe']:7.1f} us ({gb / res['mipipe'] * 1e3:5.2f} TB/s) | "
          f"torch {res['torch']:7.1f} us ({gb / res['torch'] * 1e3:5.2f} TB/s)", flush=True)
