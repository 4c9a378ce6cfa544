"""Repeat the forward GEMM with and without the x^T emission (GemmArgs::at) and count, per arm, the runs whose
output differs from that arm's first run and from the other arm (intermittent-race screen).

    python tools/emit_screen.py [reps] [M N K]
"""
import math
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
M, N, K = (int(a) for a in sys.argv[2:5]) if len(sys.argv) > 4 else (8192, 4096, 4096)
torch.manual_seed(21)
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).to(torch.bfloat16)
b = torch.randn(N, device="cuda").to(torch.bfloat16)
xt = torch.empty((K, M), device="cuda", dtype=torch.bfloat16)
ref = (x.float() @ w.float().t() + b.float())


def plain():
    return k.linear_fwd(x, w, b, 0, 0.0, False)[0]


def emit():
    return k.linear_fwd(x, w, b, 0, 0.0, False, None, xt)[0]


first = {"plain": plain().clone(), "emit": emit().clone()}
print("first runs equal:", torch.equal(first["plain"], first["emit"]),
      "max |plain - fp32 ref|:", (first["plain"].float() - ref).abs().max().item(), flush=True)
bad = {"plain": 0, "emit": 0}
for r in range(reps):
    for name, fn in (("plain", plain), ("emit", emit)):
        y = fn()
        if not torch.equal(y, first[name]):
            bad[name] += 1
            d = (y.float() - first[name].float()).abs()
            idx = (d > 0).nonzero()
            print(f"rep {r} {name}: {idx.shape[0]} elems differ, rows {idx[:, 0].min().item()}-{idx[:, 0].max().item()} "
                  f"cols {idx[:, 1].min().item()}-{idx[:, 1].max().item()} max {d.max().item():.3g}", flush=True)
    if not torch.equal(xt, x.t()):
        print(f"rep {r}: x^T wrong", flush=True)
print(f"{reps} reps: plain differs {bad['plain']}x, emit differs {bad['emit']}x", flush=True)
