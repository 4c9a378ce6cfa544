"""Intermittent-mismatch screen of the forward GEMM epilogue variants at one shape: each variant run
`reps` times against its first result; a mismatch is broken down by 256x256 tile and by the row /
column position inside the tile (epilogue pass = row half, wave column = col // 64).

    python tools/gemm_gelu_screen.py [reps]
"""
import math
import sys
from collections import Counter

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
DEV = "cuda"
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
torch.manual_seed(12)
T, K, N = 2048, 512, 9000
x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
b = torch.randn(N, device=DEV).to(torch.bfloat16)

VARIANTS = {
    "gelu+aux": lambda: k.linear_fwd(x, w, b, 2, 0.0, True)[:2],
    "gelu": lambda: (k.linear_fwd(x, w, b, 2, 0.0, False)[0], None),
    "gelu p0.1": lambda: (k.linear_fwd(x, w, b, 2, 0.1, False)[0], None),
    "relu p0.3": lambda: (k.linear_fwd(x, w, b, 1, 0.3, False)[0], None),
    "bias only": lambda: (k.linear_fwd(x, w, b, 0, 0.0, False)[0], None),
}


def where(a, bb):
    ne = a.float() != bb.float()
    n = int(ne.sum().item())
    if not n:
        return None
    idx = ne.nonzero()
    r, c = idx[:, 0], idx[:, 1]
    tiles = Counter(zip((r // 256).tolist(), (c // 256).tolist()))
    half = Counter(((r % 256) // 128).tolist())
    wcol = Counter(((c % 256) // 64).tolist())
    return (f"{n} elems in {len(tiles)} tiles {dict(list(tiles.items())[:6])}; row halves {dict(half)}; "
            f"wave cols {dict(wcol)}")


for rounds in (1, 0):
    k.gemm_set_rounds(rounds)
    for name, fn in VARIANTS.items():
        torch.manual_seed(5)
        first = [t.clone() if t is not None else None for t in fn()]
        bad = []
        for it in range(reps):
            torch.manual_seed(5)
            got = fn()
            for j, (g, f) in enumerate(zip(got, first)):
                if g is None:
                    continue
                wdesc = where(g, f)
                if wdesc:
                    bad.append(f"rep {it} out{j}: {wdesc}")
        print(f"rounds {rounds} {name:10s}: {len(bad)} mismatching outputs in {reps} reps", flush=True)
        for line in bad[:4]:
            print("    " + line, flush=True)
k.gemm_set_rounds(1)
