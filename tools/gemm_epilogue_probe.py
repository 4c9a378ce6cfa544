"""Fixed (K-independent) cost of the GEMM epilogues: time 4096 x 4096 x K for small K."""
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


M = N = 4096
for K in (64, 128, 256, 512, 1024, 4096):
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    bias = torch.zeros(N, device="cuda").to(torch.bfloat16)
    t_bf = timeit(lambda: k.linear_fwd(a, b, None, 0, 0.0, False))
    t_bias = timeit(lambda: k.linear_fwd(a, b, bias, 1, 0.0, False))
    t_drop = timeit(lambda: k.linear_fwd(a, b, bias, 1, 0.2, False))
    t_f32 = timeit(lambda: k.gemm_f32(a, b, True, True))
    print(f"K={K:5d}  bf16 {t_bf:7.1f} us  +bias+relu {t_bias:7.1f}  +dropout {t_drop:7.1f}  f32 {t_f32:7.1f}")
