"""Does the HIP runtime torch loads accept hipMemcpyDeviceToDeviceNoCU, and does it run such copies on the DMA
engines?  (The standalone probes link /opt/rocm's runtime; torch ships its own libamdhip64.so.)  Run under
``rocprofv3 --kernel-trace --memory-copy-trace`` and read with tools/small_copy_report.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mipipe  # noqa: F401,E402
from mipipe import _native_loader  # noqa: E402

k = _native_loader.kernels()
print("hip runtime version", k.hip_runtime_version(), "torch.version.hip", torch.version.hip)
s = torch.cuda.current_stream().cuda_stream
for n in (1, 512, 8192, 131072, 524288, 1 << 20):
    a = torch.ones(n, dtype=torch.int64, device="cuda")
    b = torch.zeros_like(a)
    torch.cuda.synchronize()
    err = [k.copy_nocu(b, a, s) for _ in range(3)]
    torch.cuda.synchronize()
    print(f"{8 * n:>9} B: {'accepted' if not any(err) else err[0]}, copied {bool(torch.equal(a, b))}")
