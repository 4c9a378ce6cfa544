"""Fixed per-tile cost of the forward GEMM: time(K) = fixed + K * slope at M x N
(enc12 qkv: 4096 x 12288, 768 tiles = 3 per CU), mipipe vs hipBLASLt.

    python tools/gemm_k_sweep.py [M N]
"""
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


M, N = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4096, 12288)
print(f"fwd {M} x {N} x K: us (mipipe plain | mipipe bias+relu | mipipe fp32 out | hipBLASLt)")
rows = []
for K in (64, 128, 256, 512, 1024, 2048, 4096):
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    t0 = timeit(lambda: k.linear_fwd(x, w, None, 0, 0.0, False))
    t1 = timeit(lambda: k.linear_fwd(x, w, b, 1, 0.0, False))
    t2 = timeit(lambda: k.gemm_f32(x, w, True, True))
    th = timeit(lambda: torch.matmul(x, w.t()))
    rows.append((K, t0, th))
    print(f"K={K:5d}  {t0:8.1f} {t1:8.1f} {t2:8.1f} {th:8.1f}   ({2 * M * N * K / t0 / 1e6:5.0f} vs {2 * M * N * K / th / 1e6:5.0f} TF/s)")
(k1, a1, h1), (k2, a2, h2) = rows[-3], rows[-1]
sa, sh = (a2 - a1) / (k2 - k1), (h2 - h1) / (k2 - k1)
print(f"fit over K={k1}..{k2}: mipipe fixed {a2 - sa * k2:.1f} us + {sa * 1000:.1f} us/1k K; "
      f"hipBLASLt fixed {h2 - sh * k2:.1f} us + {sh * 1000:.1f} us/1k K")
