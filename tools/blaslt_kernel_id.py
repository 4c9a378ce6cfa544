#!/usr/bin/env python3
"""Which hipBLASLt kernels torch runs for the enc12 forward GEMM shapes (run under
rocprofv3 --kernel-trace: the kernel names encode macro tile, MFMA shape, waves
and DirectToLds).  Also times them with events, for the main-loop comparison."""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
dev = "cuda"
for (T, N, K) in [(8192, 4096, 4096), (8192, 12288, 4096), (4096, 4096, 4096)]:
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    for _ in range(5):
        y = F.linear(x, w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        y = F.linear(x, w)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"{T}x{N}x{K}: {us:.1f} us  {2*T*N*K/us/1e6:.0f} TF/s", flush=True)
