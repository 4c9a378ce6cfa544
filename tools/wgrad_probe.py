"""Weight-gradient GEMMs at the sizes of a real deferred flush (K = all tokens of a step), in ONE
process with arms alternated: main-loop schedule 3 (wgrad layout on the per-tile loop) vs 4
(ping-pong with the B lead everywhere).

    python tools/wgrad_probe.py
"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()


def timeit(fn, iters=6):
    for _ in range(2):
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
for _ in range(300):
    k.linear_fwd(_x, _x, None, 0, 0.0, False)
torch.cuda.synchronize()

modes = [int(m) for m in sys.argv[1:]] or [3, 4]
print("weight [N x K], T tokens | " + " | ".join(f"sched {m}: us TF/s" for m in modes), flush=True)
for tag, T, shapes in (("gpt2xl", 4 * 18432, ((4800, 1600), (1600, 1600), (6400, 1600), (1600, 6400))),
                       ("enc12", 4 * 8192, ((12288, 4096), (4096, 4096), (28928, 4096)))):
    for N, K in shapes:
        dy = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        g = torch.zeros(N, K, device="cuda")
        res = {m: [] for m in modes}
        for _ in range(2):
            for m in modes + modes[::-1]:
                k.gemm_set_schedule(m)
                res[m].append(timeit(lambda: k.linear_wgrad(dy, x, g, True)))
        k.gemm_set_schedule(7)
        fl = 2.0 * T * N * K
        print(f"{tag} [{N} x {K}], T={T} | " + " | ".join(f"{min(res[m]):9.1f} {fl / min(res[m]) / 1e6:5.0f}"
                                                          for m in modes), flush=True)
        del dy, x, g
