"""Interleaved GEMM timing: mipipe MFMA kernel vs hipBLASLt (torch.matmul), one process, warm clocks,
each arm timed twice in the order ours, hipBLASLt, hipBLASLt, ours (the better of each).

    python tools/bench_gemm.py [T] [enc12|gpt2xl] > profiles/gemm_bench.txt
"""
import statistics
import sys
import time

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


def ab(fm, fh):
    """Both arms twice in the order m, h, h, m; the better of each (neither always runs first)."""
    m1, h1, h2, m2 = timeit(fm), timeit(fh), timeit(fh), timeit(fm)
    return min(m1, m2), min(h1, h2)


SHAPES = {
    "enc12": lambda T: [("qkv fwd", T, 12288, 4096), ("out fwd", T, 4096, 4096), ("ffn fwd", T, 4096, 4096),
                        ("dec fwd", T, 28928, 4096)],
    "gpt2xl": lambda T: [("qkv fwd", T, 4800, 1600), ("out fwd", T, 1600, 1600), ("fc1 fwd", T, 6400, 1600),
                         ("fc2 fwd", T, 1600, 6400)],
}


def main(T=int(sys.argv[1]) if len(sys.argv) > 1 else 4096, model=sys.argv[2] if len(sys.argv) > 2 else "enc12"):
    # clocks up before anything is timed: the first timings of a process read slow
    # (4096 x 12288 x 4096: ~357 us cold vs ~289 us warm)
    xw = torch.randn(4096, 4096, device=dev).to(torch.bfloat16)
    for _ in range(300):
        k.linear_fwd(xw, xw, None, 0, 0.0, False)
    torch.cuda.synchronize()

    shapes = SHAPES[model](T)
    print(f"{'case':12s} {'M':>6s} {'N':>6s} {'K':>6s} | {'mipipe ms':>9s} {'TF/s':>7s} | {'hipBLASLt ms':>12s} {'TF/s':>7s}")
    for name, M, N, K in shapes:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N, K, device=dev).to(torch.bfloat16)
        fl = 2.0 * M * N * K
        t_m, t_h = ab(lambda: k.linear_fwd(x, w, None, 0, 0.0, False), lambda: torch.matmul(x, w.t()))
        print(f"{name:12s} {M:6d} {N:6d} {K:6d} | {t_m:9.3f} {fl / t_m / 1e9:7.0f} | {t_h:12.3f} {fl / t_h / 1e9:7.0f}")
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        t_m, t_h = ab(lambda: k.linear_dgrad(dy, w), lambda: torch.matmul(dy, w))
        print(f"{name[:3]+' dgrad':12s} {M:6d} {K:6d} {N:6d} | {t_m:9.3f} {fl / t_m / 1e9:7.0f} | {t_h:12.3f} {fl / t_h / 1e9:7.0f}")
        mg = torch.zeros(N, K, device=dev)
        t_m, t_h = ab(lambda: k.linear_wgrad(dy, x, mg), lambda: mg.add_(torch.matmul(dy.t(), x)))
        print(f"{name[:3]+' wgrad+acc':12s} {N:6d} {K:6d} {M:6d} | {t_m:9.3f} {fl / t_m / 1e9:7.0f} | {t_h:12.3f} {fl / t_h / 1e9:7.0f}")


if __name__ == "__main__":
    main()
