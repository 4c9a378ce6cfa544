"""Repeats GEMMs of one shape many times in every operand layout and block width and counts
results that differ from the first one (bitwise; the kernels are deterministic), to tell an
intermittent wrong tile (a staging race) from a systematic one.

    python tools/gemm_race_screen.py [M N K] [reps]
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (4096, 4800, 1600)
reps = int(sys.argv[4]) if len(sys.argv) >= 5 else 50
torch.manual_seed(1)
a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
b = torch.randn(K, N, device="cuda").to(torch.bfloat16)
ref = a.float() @ b.float()
for width in (0, 128, 256):
    k.gemm_set_width(width)
    for rounds in (1, 0):
        k.gemm_set_rounds(rounds)
        for a_kc, b_kc in [(True, True), (True, False), (False, False), (False, True)]:
            A = a if a_kc else a.t().contiguous()
            B = b.t().contiguous() if b_kc else b
            poison = torch.full((M, N), float("nan"), device="cuda")
            del poison
            first = k.gemm_f32(A, B, a_kc, b_kc)
            err0 = (first - ref).abs().max().item()
            bad, worst = 0, 0.0
            for _ in range(reps):
                # the caching allocator hands the output the block just freed: NaN-filled,
                # so an element the GEMM does not write shows
                poison = torch.full((M, N), float("nan"), device="cuda")
                del poison
                c = k.gemm_f32(A, B, a_kc, b_kc)
                if not torch.equal(c, first):
                    bad += 1
                    worst = max(worst, (c - first).abs().max().item())
            print(f"width {width:3d} rounds {rounds} layout {int(a_kc)}{int(b_kc)}: first err {err0:.3g}, "
                  f"{bad}/{reps} differ (max {worst:.3g})", flush=True)
k.gemm_set_width(0)
k.gemm_set_rounds(1)
