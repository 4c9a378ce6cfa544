"""A/B: deferred weight-gradient GEMM (main_grad fp32 += dY^T X over 4 micro-batch
segments) on the mipipe K-segmented kernel vs hipBLASLt through torch (bf16 in,
fp32 out).  enc12_d4096 shapes: T = 4 x SEG tokens (argv[1], default 4096; the step's flush today: 16384).
"addmm x4" accumulates one micro-batch segment per call (no concatenation copy)."""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()


def timeit(fn, iters=10):
    for _ in range(2):
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


seg, nseg = (int(sys.argv[1]) if len(sys.argv) > 1 else 4096), 4
for name, N, K in (("out", 4096, 4096), ("qkv", 12288, 4096)):
    dys = [torch.randn(seg, N, device="cuda").to(torch.bfloat16) for _ in range(nseg)]
    xs = [torch.randn(seg, K, device="cuda").to(torch.bfloat16) for _ in range(nseg)]
    main = torch.zeros(N, K, device="cuda")
    fl = 2.0 * N * K * seg * nseg
    t_ours = timeit(lambda: k.linear_wgrad_segments(dys, xs, main, True))
    ref = main.clone()
    line = f"{name:4s} {N}x{K}x{seg * nseg}: mipipe {t_ours:8.1f} us {fl / t_ours / 1e6:6.0f} TF/s"
    dyc, xc = torch.cat(dys), torch.cat(xs)
    for label, fn in (
        ("addmm_out", lambda: torch.addmm(main, dyc.t(), xc, out_dtype=torch.float32, out=main)),
        ("addmm_new", lambda: torch.addmm(main, dyc.t(), xc, out_dtype=torch.float32)),
        ("cat+addmm", lambda: torch.addmm(main, torch.cat(dys).t(), torch.cat(xs), out_dtype=torch.float32, out=main)),
        ("mm_bf16", lambda: torch.mm(dyc.t(), xc)),
        ("addmm x4", lambda: [torch.addmm(main, d.t(), x, out_dtype=torch.float32, out=main) for d, x in zip(dys, xs)]),
    ):
        try:
            t = timeit(fn)
            line += f" | {label} {t:8.1f} us {fl / t / 1e6:6.0f}"
        except Exception as ex:  # noqa: BLE001
            line += f" | {label} ERR {str(ex)[:80]}"
    print(line, flush=True)
    # numerics: one accumulation from zero each way
    main.zero_()
    k.linear_wgrad_segments(dys, xs, main, True)
    try:
        alt = torch.addmm(torch.zeros_like(main), dyc.t(), xc, out_dtype=torch.float32)
        print(f"     max |mipipe - blaslt| = {(main - alt).abs().max().item():.3e} (scale {alt.abs().max().item():.2e})")
    except Exception as ex:  # noqa: BLE001
        print("     numerics skipped:", str(ex)[:80])
    del dys, xs, main, dyc, xc
    torch.cuda.empty_cache()

# plain dgrad of the decoder: dX[T, E] = dY[T, V] W[V, E]
dy = torch.randn(4096, 28928, device="cuda").to(torch.bfloat16)
w = torch.randn(28928, 4096, device="cuda").to(torch.bfloat16)
fl = 2.0 * 4096 * 28928 * 4096
t1 = timeit(lambda: k.linear_dgrad(dy, w, None))
t2 = timeit(lambda: torch.mm(dy, w))
print(f"dec dgrad: mipipe {t1:.1f} us {fl / t1 / 1e6:.0f} TF/s | torch.mm {t2:.1f} us {fl / t2 / 1e6:.0f} TF/s")
