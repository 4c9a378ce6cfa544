"""Cost of the activation-backward epilogue (GemmArgs::dact) vs a plain dgrad + the separate
bias_act backward kernel, GPT-2-XL fc2 dgrad shape (T=8192, [8192 x 6400] output, K=1600) and the
enc12 ReLU shape ([8192 x 4096], K=4096).  Arms alternated in one process.

    python tools/gemm_dact_probe.py
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


_x = torch.randn(4096, 4096, device="cuda").to(torch.bfloat16)
for _ in range(300):
    k.linear_fwd(_x, _x, None, 0, 0.0, False)
torch.cuda.synchronize()

for name, T, E, F, act, p in (("gpt2xl fc2 dgrad gelu p0.1", 8192, 1600, 6400, 2, 0.1),
                              ("gpt2xl gelu p0", 8192, 1600, 6400, 2, 0.0),
                              ("enc12 ffn dgrad relu p0.2", 8192, 4096, 4096, 1, 0.2)):
    x = torch.randn(T, E, device="cuda").to(torch.bfloat16)
    w1 = (torch.randn(F, E, device="cuda") * 0.05).to(torch.bfloat16)
    b1 = torch.randn(F, device="cuda").to(torch.bfloat16)
    w2 = (torch.randn(E, F, device="cuda") * 0.05).to(torch.bfloat16)
    y, pre, seed, offset = k.linear_fwd(x, w1, b1, act, p, act == 2)
    saved = pre if act == 2 else y
    dy = torch.randn(T, E, device="cuda").to(torch.bfloat16)
    arms = {
        "plain dgrad": lambda: k.linear_dgrad(dy, w2),
        "dgrad + bias_act_bwd": lambda: k.bias_act_bwd(k.linear_dgrad(dy, w2), saved, None, act, p, seed, offset,
                                                        False, None),
        "dgrad with dact epilogue": lambda: k.linear_dgrad(dy, w2, None, None, act, saved, p, seed, offset),
    }
    res = {a: [] for a in arms}
    for _ in range(3):
        for a in list(arms) + list(arms)[::-1]:
            res[a].append(timeit(arms[a]))
    print(name + ": " + " | ".join(f"{a} {min(v):7.1f} us" for a, v in res.items()), flush=True)
