"""GEMM main-loop schedules A/B in ONE process (rule 24): gemm_set_schedule(2) (ping-pong) vs
(3) (ping-pong, B staged two K-tiles ahead), arms alternated per shape, best of 3 rounds of
medians; the enc12 T=8192 shapes and GPT-2-XL's (T=8192, E=1600) forward / dgrad / wgrad.

    python tools/gemm_sched_ab.py [modes...]
"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
modes = [int(m) for m in sys.argv[1:]] or [2, 3]


def timeit(fn, iters=15):
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


_x = torch.randn(4096, 4096, device="cuda").to(torch.bfloat16)
for _ in range(300):  # clocks up before timing
    k.linear_fwd(_x, _x, None, 0, 0.0, False)
torch.cuda.synchronize()

T = 8192
cases = []
for tag, E, outs in (("enc12", 4096, ((12288, "qkv"), (4096, "out"), (28928, "dec"))),
                     ("gpt2xl", 1600, ((4800, "qkv"), (1600, "out"), (6400, "fc1")))):
    for N, name in outs:
        cases.append((f"{tag} {name} fwd", T, N, E, "fwd"))
        cases.append((f"{tag} {name} dgrad", T, E, N, "dgrad"))
        cases.append((f"{tag} {name} wgrad", N, E, T, "wgrad"))
cases.append(("gpt2xl fc2 fwd", T, 1600, 6400, "fwd"))

print(f"{'case':22s} {'M':>6s} {'N':>6s} {'K':>6s} | " + " | ".join(f"sched {m}: us  TF/s" for m in modes), flush=True)
for name, M, N, K, kind in cases:
    if kind == "fwd":
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        b = torch.randn(N, device="cuda").to(torch.bfloat16)
        fn = lambda: k.linear_fwd(x, w, b, 0, 0.0, False)  # noqa: E731
    elif kind == "dgrad":
        dy = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(K, N, device="cuda").to(torch.bfloat16)
        fn = lambda: k.linear_dgrad(dy, w)  # noqa: E731
    else:
        dy = torch.randn(K, M, device="cuda").to(torch.bfloat16)
        x = torch.randn(K, N, device="cuda").to(torch.bfloat16)
        g = torch.zeros(M, N, device="cuda")
        fn = lambda: k.linear_wgrad(dy, x, g, True)  # noqa: E731
    res = {m: [] for m in modes}
    for _ in range(3):
        for m in modes + modes[::-1]:
            k.gemm_set_schedule(m)
            res[m].append(timeit(fn))
    k.gemm_set_schedule(7)
    fl = 2.0 * M * N * K
    print(f"{name:22s} {M:6d} {N:6d} {K:6d} | " +
          " | ".join(f"{min(res[m]):8.1f} {fl / min(res[m]) / 1e6:5.0f}" for m in modes), flush=True)
