"""4-wave (gemm4w_kernel, 128x128 per wave) vs 8-wave (ping-pong, 128x64 per wave)
256x256 GEMM blocks on the enc12 step's shapes: numerics of the 4-wave kernel
against an fp32 torch reference (sampled rows), then interleaved timing, each
arm twice in the order 8, 4, 4, 8 (the better of each).

    python tools/gemm_waves_ab.py [T]
"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
dev = "cuda"


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
    return statistics.median(ts)


def arm(w, fn):
    k.gemm_set_waves(w)
    return timeit(fn)


def ab(fn):
    a1, b1, b2, a2 = arm(8, fn), arm(4, fn), arm(4, fn), arm(8, fn)
    k.gemm_set_waves(0)
    return min(a1, a2), min(b1, b2)


def rel_err(got, ref):
    return float((got.float() - ref).abs().max() / (ref.abs().max() + 1e-6))


def main(T=int(sys.argv[1]) if len(sys.argv) > 1 else 8192):
    torch.manual_seed(0)
    xw = torch.randn(4096, 4096, device=dev).to(torch.bfloat16)
    for _ in range(300):
        k.linear_fwd(xw, xw, None, 0, 0.0, False)
    torch.cuda.synchronize()
    # numerics first (the 4-wave kernel on every layout it serves)
    ok = True
    k.gemm_set_width(256)  # small grids would otherwise take the 256x128 block (8-wave only)
    for (M, N, K) in [(1088, 768, 1088), (1280, 576, 512)]:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        b = torch.randn(N, device=dev).to(torch.bfloat16)
        k.gemm_set_waves(4)
        y = k.linear_fwd(x, w, b, 1, 0.0, False)[0]
        dx = k.linear_dgrad(dy, w)
        mg = torch.zeros(N, K, device=dev)
        k.linear_wgrad(dy, x, mg)
        k.gemm_set_waves(0)
        ry = torch.relu(x.float() @ w.float().t() + b.float())
        rdx = dy.float() @ w.float()
        rmg = dy.float().t() @ x.float()
        errs = (rel_err(y, ry), rel_err(dx, rdx), rel_err(mg, rmg))
        good = all(e < 2e-2 for e in errs)
        ok &= good
        print(f"numerics {M}x{N}x{K}: fwd {errs[0]:.2e} dgrad {errs[1]:.2e} wgrad {errs[2]:.2e} {'ok' if good else 'FAIL'}",
              flush=True)
    k.gemm_set_width(0)
    if not ok:
        sys.exit(1)
    shapes = [("qkv", T, 12288, 4096), ("out/ffn", T, 4096, 4096), ("dec", T, 28928, 4096)]
    print(f"{'case':14s} {'M':>6s} {'N':>6s} {'K':>6s} | {'8-wave us':>9s} {'TF/s':>6s} | {'4-wave us':>9s} {'TF/s':>6s} | gain")
    for name, M, N, K in shapes:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        for case, fn in ((f"{name} fwd", lambda: k.linear_fwd(x, w, None, 0, 0.0, False)),
                         (f"{name} dgrad", lambda: k.linear_dgrad(dy, w))):
            t8, t4 = ab(fn)
            print(f"{case:14s} {M:6d} {N:6d} {K:6d} | {t8*1e3:9.1f} {fl/t8/1e9:6.0f} | {t4*1e3:9.1f} {fl/t4/1e9:6.0f} |"
                  f" {100*(t8/t4-1):+5.1f} %", flush=True)
        if name != "dec":
            mg = torch.zeros(N, K, device=dev)
            t8, t4 = ab(lambda: k.linear_wgrad(dy, x, mg))
            print(f"{name+' wgrad':14s} {N:6d} {K:6d} {M:6d} | {t8*1e3:9.1f} {fl/t8/1e9:6.0f} | {t4*1e3:9.1f} {fl/t4/1e9:6.0f} |"
                  f" {100*(t8/t4-1):+5.1f} %", flush=True)


if __name__ == "__main__":
    main()
