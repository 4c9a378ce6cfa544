"""Long-sequence attention forward at GPT-2-XL's shape with the keep words made inside the kernel (DM=2) vs read
(DM=1, after the stand-alone mask kernel): run under rocprofv3 --kernel-trace to split the kernels.

    rocprofv3 --kernel-trace --stats -d gpurun_out/dm -o run -- python3 tools/attn_long_dm_probe.py
"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
B, S, H, D, p = 18, 1024, 25, 64, 0.1
qkv = torch.randn(B, S, 3, H, D, device="cuda").to(torch.bfloat16)
q, kk, v = (qkv.select(2, i) for i in range(3))
for fused in (True, False, True, False):
    k.attention_long_set_fused_rng(fused)
    for _ in range(20):
        k.attention_fwd(q, kk, v, True, p, D ** -0.5)
    torch.cuda.synchronize()
k.attention_long_set_fused_rng(True)
print("ok")
