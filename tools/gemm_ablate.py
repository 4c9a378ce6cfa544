"""GEMM ablation at 4096^3: layout (K- vs I-contiguous operands) x epilogue."""
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


M = N = K = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
at = a.t().contiguous()
bt = b.t().contiguous()
c = torch.zeros(M, N, device="cuda")
fl = 2.0 * M * N * K
cases = {
    "KC,KC bf16-store (fwd)": lambda: k.linear_fwd(a, b, None, 0, 0.0, False),
    "KC,KC f32-store": lambda: k.gemm_f32(a, b, True, True),
    "KC,IC f32-store (dgrad layout)": lambda: k.gemm_f32(a, bt, True, False),
    "IC,IC f32-store (wgrad layout)": lambda: k.gemm_f32(at, bt, False, False),
    "IC,IC f32-accumulate (wgrad)": lambda: k.linear_wgrad(at.t().contiguous() if False else a.t().contiguous().t(), b, c) if False else k.linear_wgrad(torch.empty(0), torch.empty(0), c) if False else None,
}
# wgrad proper: dW[N,K] += dy[T,N]^T x[T,K]
dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)   # [T=K, M]
xx = torch.randn(K, N, device="cuda").to(torch.bfloat16)   # [T=K, N]
cases["IC,IC f32-accumulate (wgrad)"] = lambda: k.linear_wgrad(dy, xx, c)
cases["hipBLASLt bf16"] = lambda: torch.matmul(a, b.t())
scheds = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [k.gemm_get_schedule()]
for name, fn in cases.items():
    for sc in scheds:
        k.gemm_set_schedule(sc)
        t = timeit(fn)
        print(f"{name:34s} sched={sc} {t * 1e3:8.1f} us  {fl / t / 1e9:7.0f} TF/s")
        if name.startswith("hipBLASLt"):
            break
