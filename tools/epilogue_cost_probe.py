"""What the forward GEMM's epilogue variants cost at GPT-2-XL's fc1 shape (x [18432, 1600] . W [6400, 1600]^T):
plain bf16, + bias, + GELU, + GELU + dropout 0.1, + pre-activation output, + GELU'(pre) output (aux_grad).
Arms alternate in one process; median of 20 after warm-up.

    python tools/epilogue_cost_probe.py [T K N]
"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
T, K, N = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (18432, 1600, 6400)
torch.manual_seed(0)
x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
b = torch.randn(N, device="cuda").to(torch.bfloat16)
ARMS = {
    "plain": lambda: k.linear_fwd(x, w, None, 0, 0.0, False),
    "bias": lambda: k.linear_fwd(x, w, b, 0, 0.0, False),
    "bias+gelu": lambda: k.linear_fwd(x, w, b, 2, 0.0, False),
    "bias+relu+drop0.1": lambda: k.linear_fwd(x, w, b, 1, 0.1, False),
    "bias+gelu+drop0.1": lambda: k.linear_fwd(x, w, b, 2, 0.1, False),
    "bias+gelu+drop0.1+pre": lambda: k.linear_fwd(x, w, b, 2, 0.1, True),
    "bias+gelu+drop0.1+gelu'": lambda: k.linear_fwd(x, w, b, 2, 0.1, True, None, None, True),
}
times = {a: [] for a in ARMS}
for _ in range(3):
    for fn in ARMS.values():
        fn()
torch.cuda.synchronize()
for rep in range(20):
    for a, fn in ARMS.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        times[a].append(e0.elapsed_time(e1) * 1e3)
flops = 2.0 * T * K * N
base = statistics.median(times["plain"])
print(f"# forward GEMM {T} x {N} x {K} ({flops / 1e9:.0f} GFLOP), median of 20, us (TF/s, + vs plain)")
for a in ARMS:
    t = statistics.median(times[a])
    print(f"{a:26s} {t:8.1f} us  ({flops / t / 1e6:6.0f} TF/s)  {t - base:+7.1f}", flush=True)
