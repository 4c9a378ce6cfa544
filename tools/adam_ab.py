"""Adam kernel variants, interleaved in ONE process (rule 24): a flat 1.44B-
parameter group (the enc12_d4096 PP=1 stage), bf16 model + fp32 master /
grad / moments, 30 B per parameter per step.

    python tools/adam_ab.py [n_params]
"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_444_860_160
dev = "cuda"
master = torch.randn(n, device=dev)
model = master.to(torch.bfloat16)
grad = torch.randn(n, device=dev) * 1e-3
m = torch.zeros(n, device=dev)
v = torch.zeros(n, device=dev)
sq = torch.ones(1, device=dev)


def run():
    k.adam_step(master, model, grad, m, v, 1e-4, 0.9, 0.999, 1e-8, 0.0, 0.1, 0.001, sq, 0.5, False)


def timeit(iters=10):
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        run()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


for _ in range(5):
    run()
VARIANTS = {0: "grid-stride loop", 1: "one tile per block", 2: "one tile per block, streaming stores (default)"}
res = {v_: [] for v_ in VARIANTS}
for rnd in range(3):
    for var in (0, 1, 2, 2, 1, 0):
        k.adam_set_variant(var)
        res[var].append(timeit())
gb = 30.0 * n / 1e9
for var, ts in res.items():
    t = min(ts)
    print(f"variant {var} ({VARIANTS[var]}): {t:7.3f} ms (median {statistics.median(ts):.3f})  {gb / t:6.2f} TB/s "
          f"at 30 B/param", flush=True)
k.adam_set_variant(2)
# the same HBM read / write mix without the math: 16 B read + 14 B written per parameter (grad, master, moments in;
# master, moments, bf16 model out) vs a plain copy (read 1, write 1)
del m, v
a = torch.empty(n // 2, device=dev)
b = torch.empty_like(a)
ts = []
for _ in range(10):
    s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s_.record()
    b.copy_(a)
    e_.record()
    e_.synchronize()
    ts.append(s_.elapsed_time(e_))
t = min(ts)
print(f"torch copy_ {a.numel() * 4 / 1e9:.1f} GB -> {a.numel() * 8 / 1e9 / t:.2f} TB/s (read + write)", flush=True)
