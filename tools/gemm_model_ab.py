"""A/B of the GEMM main-loop schedules at the enc12_d4096 training shapes
(micro-batch T = 4096 tokens): forward (KC,KC + bias/ReLU), dgrad (KC,IC),
deferred wgrad (IC,IC, K-segmented over 4 micro-batches, fp32 accumulate).

    python tools/gemm_model_ab.py [SCHED ...]    (default: 0 1; see gemm_set_schedule)"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
SCHEDS = [int(a) for a in sys.argv[1:]] or [0, 1]
T, E, V = 4096, 4096, 28928


def timeit(fn, iters=10):
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


cases = []
for N, K in ((3 * E, E), (E, E), (V, E)):
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.zeros(N, device="cuda").to(torch.bfloat16)
    dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
    mg = torch.zeros(N, K, device="cuda")
    fl = 2.0 * T * N * K
    cases.append((f"fwd   {T}x{N}x{K} relu", fl, lambda x=x, w=w, b=b: k.linear_fwd(x, w, b, 1, 0.0, False)))
    cases.append((f"dgrad {T}x{K}x{N}", fl, lambda dy=dy, w=w: k.linear_dgrad(dy, w)))
    dys = [torch.randn(T, N, device="cuda").to(torch.bfloat16) for _ in range(4)]
    xs = [torch.randn(T, K, device="cuda").to(torch.bfloat16) for _ in range(4)]
    cases.append((f"wgrad {N}x{K}x(4x{T}) seg", 4 * fl, lambda dys=dys, xs=xs, mg=mg: k.linear_wgrad_segments(dys, xs, mg)))

for name, fl, fn in cases:
    res = []
    for sc in SCHEDS:
        k.gemm_set_schedule(sc)
        t = timeit(fn)
        res.append(f"sched={sc} {t:8.1f} us {fl / t / 1e6:6.0f} TF/s")
    print(f"{name:32s} " + " | ".join(res))
k.gemm_set_schedule(2)
