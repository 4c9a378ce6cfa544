"""Why a GEMM runs faster "in isolation" than inside the training step
(the transposed QKV weight-gradient GEMM at 1.47 PF/s alone,
1.32 inside the step): the same launches timed as a short burst after idle (what
tools/bench_gemm.py and the A/B scripts measure) and sustained for seconds (what
the step does), with the amdsmi telemetry of each window.

    python tools/gemm_clock_probe.py            # burst vs sustained, the default kernel
    python tools/gemm_clock_probe.py --waves    # sustained only: 8-wave vs 4-wave block, interleaved (energy per
                                                # FLOP decides speed at the power cap; bursts cannot show it)
"""
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402
from mipipe.utils.telemetry import GpuTelemetry  # noqa: E402

k = kernels()
dev = "cuda"
SHAPES = [("fwd 8192x4096x4096", 8192, 4096, 4096), ("qkv fwd 8192x12288x4096", 8192, 12288, 4096)]


def run_window(fn, seconds=None, iters=None):
    tel = GpuTelemetry(0, period=0.002 if iters else 0.02).start()
    ts = []
    t_end = time.perf_counter() + (seconds or 0)
    n = 0
    while (iters is not None and n < iters) or (seconds is not None and time.perf_counter() < t_end):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / 10)
        n += 1
    t = tel.stop()
    return statistics.median(ts), t


def waves_ab():
    for name, M, N, K in SHAPES:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        for case, fn in (("fwd", lambda: k.linear_fwd(x, w, None, 0, 0.0, False)),
                         ("dgrad", lambda: k.linear_dgrad(dy, w))):
            for waves in (8, 4, 4, 8):
                k.gemm_set_waves(waves)
                for _ in range(10):
                    fn()
                torch.cuda.synchronize()
                time.sleep(2.0)
                ms, t = run_window(fn, seconds=3.0)
                clk = (t.get("gfxclk_mhz") or {}).get("mean")
                pw = (t.get("socket_power_w") or {}).get("mean")
                print(f"{name:26s} {case:5s} {waves}-wave sustained 3 s {ms * 1e3:7.1f} us {fl / ms / 1e9:6.0f} TF/s | "
                      f"gfxclk {clk} MHz, power {pw} W, power-limited {t.get('power_limited_pct')} %", flush=True)
        k.gemm_set_waves(0)


if "--waves" in sys.argv:
    waves_ab()
    sys.exit(0)

for name, M, N, K in SHAPES:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = torch.randn(N, K, device=dev).to(torch.bfloat16)
    fl = 2.0 * M * N * K

    def fn():
        k.linear_fwd(x, w, None, 0, 0.0, False)

    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    for label, kw in (("burst after 3 s idle (5 x 10 launches)", {"iters": 5}),
                      ("sustained 4 s", {"seconds": 4.0})):
        time.sleep(3.0)
        ms, t = run_window(fn, **kw)
        clk = (t.get("gfxclk_mhz") or {}).get("mean")
        pw = (t.get("socket_power_w") or {}).get("mean")
        print(f"{name:26s} {label:40s} {ms * 1e3:7.1f} us  {fl / ms / 1e9:6.0f} TF/s | gfxclk {clk} MHz, "
              f"power {pw} W, power-limited {t.get('power_limited_pct')} %", flush=True)
