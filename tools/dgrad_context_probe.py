"""Why does the enc12 K=4096 dgrad run ~15 % slower than the same-shape forward inside the step, when the two
are within 2 % in an isolated loop (profiles/gemm_schedules_ab.txt, M = 8192)?  Sustained, interleaved loops of
the forward (x . W^T) and the dgrad (dY . W) at M = 8192 and 16384, alone and with a 512 MiB streaming copy
between launches (what the step's LayerNorm kernels do to the caches), with the window's gfxclk."""
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402
from mipipe.utils.telemetry import GpuTelemetry  # noqa: E402

k = kernels()
dev = "cuda"


def window(fn, flush, seconds=2.0):
    tel = GpuTelemetry(0, period=0.02).start()
    ts = []
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        for _ in range(4):
            if flush is not None:
                flush()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
    t = tel.stop()
    clk = (t or {}).get("gfxclk_mhz", {}).get("mean")
    return statistics.median(ts), clk


def main():
    big = torch.empty(256 << 20, dtype=torch.float16, device=dev)  # 512 MiB
    big2 = torch.empty_like(big)
    flush = lambda: big2.copy_(big)  # noqa: E731
    for M in (8192, 16384):
        N = K = 4096
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        fwd = lambda: k.linear_fwd(x, w, None, 0, 0.0, False)  # noqa: E731
        dgr = lambda: k.linear_dgrad(dy, w)  # noqa: E731
        for _ in range(3):
            fwd(), dgr()
        torch.cuda.synchronize()
        time.sleep(1.0)
        for ctx, fl_fn in (("alone", None), ("after a 512 MiB copy", flush)):
            for rep in range(2):
                for name, fn in (("fwd", fwd), ("dgrad", dgr)):
                    us, clk = window(fn, fl_fn)
                    print(f"M={M:6d} {ctx:<22} {name:<6} {us:8.1f} us {fl / us / 1e6:7.0f} TF/s  gfxclk {clk}",
                          flush=True)


if __name__ == "__main__":
    main()
