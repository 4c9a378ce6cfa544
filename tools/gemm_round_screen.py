"""test_gemm_round_launches_identical as a screen: each output of the round-chunked launches against
the one-launch result AND against a repeat of itself, many times, reporting which outputs differ,
in how many elements and where (systematic vs intermittent).

    python tools/gemm_round_screen.py [reps]
"""
import math
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
DEV = "cuda"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
torch.manual_seed(12)
T, K, N = 2048, 512, 9000
x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
b = torch.randn(N, device=DEV).to(torch.bfloat16)
dy = torch.randn(4096, 1024, device=DEV).to(torch.bfloat16)
w2 = (torch.randn(1024, 4608, device=DEV) / 32).to(torch.bfloat16)
r = torch.randn(4096, 4608, device=DEV).to(torch.bfloat16)
dys = [torch.randn(256, 8200, device=DEV).to(torch.bfloat16) for _ in range(2)]
xs = [torch.randn(256, 2048, device=DEV).to(torch.bfloat16) for _ in range(2)]
x3 = torch.randn(2816, 512, device=DEV).to(torch.bfloat16)
w3 = (torch.randn(6400, 512, device=DEV) / math.sqrt(512)).to(torch.bfloat16)
names = ["fwd relu p0.3", "fwd gelu", "gelu preact", "dgrad+res", "wgrad segs", "fwd 2816x6400"]


def run():
    torch.manual_seed(77)
    y1 = k.linear_fwd(x, w, b, 1, 0.3, False)[0]
    torch.manual_seed(78)
    y2, pre, _, _ = k.linear_fwd(x, w, b, 2, 0.0, True)
    dx = k.linear_dgrad(dy, w2, r)
    mg = torch.zeros(8200, 2048, device=DEV)
    k.linear_wgrad_segments(dys, xs, mg, False)
    y3 = k.linear_fwd(x3, w3, None, 0, 0.0, False)[0]
    return [y1, y2, pre, dx, mg, y3]


def diff(a, bb):
    ne = (a.float() != bb.float()) & ~(torch.isnan(a.float()) & torch.isnan(bb.float()))
    n = int(ne.sum().item())
    if not n:
        return "="
    idx = ne.nonzero()
    rows, cols = idx[:, 0], idx[:, 1]
    return (f"{n} elems rows {rows.min().item()}-{rows.max().item()} cols {cols.min().item()}-{cols.max().item()} "
            f"maxdiff {(a.float() - bb.float()).abs()[ne].max().item():.3g}")


k.gemm_set_rounds(0)
ref = run()
ref2 = run()
print("one launch, repeat:", [diff(a, bb) for a, bb in zip(ref, ref2)], flush=True)
k.gemm_set_rounds(2)  # per-round launches at any K
first = run()
for it in range(reps):
    got = run()
    d_ref = [diff(a, bb) for a, bb in zip(got, ref)]
    d_self = [diff(a, bb) for a, bb in zip(got, first)]
    bad = [(names[i], d_ref[i], d_self[i]) for i in range(len(names)) if d_ref[i] != "=" or d_self[i] != "="]
    print(f"rep {it}: " + ("all identical" if not bad else "; ".join(f"{n}: vs one-launch {a} / vs first {s}"
                                                                      for n, a, s in bad)), flush=True)
