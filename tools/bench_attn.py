"""Attention kernel timing at the enc12 shape (micro-batch 128: B=128, S=128, H=16, D=256): whole-sequence
kernels (1) or the general ones (0)."""
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


B, S, H, D = (int(x) for x in (sys.argv[1:5] if len(sys.argv) > 4 else (128, 128, 16, 256)))
causal = len(sys.argv) > 5 and sys.argv[5] == "causal"
P = float(sys.argv[6]) if len(sys.argv) > 6 else 0.2
qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16)
q, kk, v = (qkv.select(2, i) for i in range(3))
scale = D ** -0.5
o, lse, seed, off, bits = k.attention_fwd(q, kk, v, causal, P, scale)
bits = bits if bits.numel() else None
causal_frac = 0.5 if causal else 1.0
fl_fwd = 4.0 * B * H * S * S * D * causal_frac
fl_bwd = 2.5 * fl_fwd
dout = torch.randn_like(o)
dq = torch.empty_like(qkv)
print(f"B={B} S={S} H={H} D={D} causal={causal} p={P}")
for fused in (0, 1):
    k.attention_set_fused_bwd(fused)
    f = timeit(lambda: k.attention_fwd(q, kk, v, causal, P, scale))
    t = timeit(lambda: k.attention_bwd(dout, q, kk, v, o, lse, causal, P, scale, seed, off,
                                       dq.select(2, 0), dq.select(2, 1), dq.select(2, 2), bits))
    print(f"  whole-sequence kernels={fused}: fwd {f:.1f} us ({fl_fwd / f / 1e6:.0f} TF/s)  "
          f"bwd {t:.1f} us ({fl_bwd / t / 1e6:.0f} TF/s)")
k.attention_set_fused_bwd(1)
