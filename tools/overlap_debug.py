"""Where do the serial and the overlapped FlatAdam steps differ? (debug aid)"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/tests")
import test_gpu_optim_overlap as t  # noqa: E402
from mipipe.optim import _Overlap  # noqa: E402

_Overlap.MIN_CHUNK = 4096
for steps in (1, 2):
    l0, p0, s0, opt0, m0 = t._train(False, "never", steps=steps)
    l1, p1, s1, opt1, m1 = t._train(True, "never", steps=steps)
    g = opt1.groups[0]
    print(f"steps {steps}: losses equal {l0 == l1}; n_lazy {g.n_lazy} n {g.numel}; chunks {opt1._overlap.chunks[0][:4]}...")
    bounds = []
    off = 0
    names = {id(p): n for n, p in m1.named_parameters()}
    for p in g.params:
        bounds.append((off, off + p.numel(), names.get(id(p), "?")))
        off += p.numel()
    for name, a, b in zip(("master", "exp_avg", "exp_avg_sq"), s0, s1):
        d = (a != b).nonzero().flatten()
        print(f"  {name}: {d.numel()} differing elements", end="")
        if d.numel():
            idx = d.tolist()
            hit = sorted({n for i in idx for (s, e, n) in bounds if s <= i < e})
            print(f"; first {idx[:5]}; params {hit[:8]}; max abs diff {(a - b).abs().max().item():.3e}")
        else:
            print()
    g0 = opt0.groups[0]
    print("  main_grad equal:", torch.equal(g0.main_grad, g.main_grad))
