"""Driver for a rocprofv3 --pmc pass: the enc12 forward and dgrad GEMMs at
8192 x 4096 x 4096, 30 launches each, on the 8-wave and the 4-wave kernel
(the kernel names tell them apart: gemm256_kernel / gemm4w_kernel)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
torch.manual_seed(0)
x = torch.randn(8192, 4096, device="cuda").to(torch.bfloat16)
w = torch.randn(4096, 4096, device="cuda").to(torch.bfloat16)
dy = torch.randn(8192, 4096, device="cuda").to(torch.bfloat16)
for waves in (8, 4):
    k.gemm_set_waves(waves)
    for _ in range(30):
        k.linear_fwd(x, w, None, 0, 0.0, False)
    for _ in range(30):
        k.linear_dgrad(dy, w)
    torch.cuda.synchronize()
k.gemm_set_waves(0)
print("done")
