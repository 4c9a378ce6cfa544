"""Weight-gradient layout probe: the flush's GEMM in its current layout (A = dY read [T, M], B = X read
[T, N]: both operands I-contiguous) against the transposed product C^T = X^T . dY with X^T stored
K-contiguous (the dgrad layout <A_KC, !B_KC>), plus what a transposition of X costs (torch copy).
One process, arms interleaved, medians; fp32 output (the main_grad store epilogue).

    python tools/wgrad_layout_probe.py [T] [gpt2xl] > profiles/wgrad_layout_probe.txt
"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
dev = "cuda"


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
    return statistics.median(ts)


def main():
    xw = torch.randn(4096, 4096, device=dev).to(torch.bfloat16)
    for _ in range(200):
        k.linear_fwd(xw, xw, None, 0, 0.0, False)
    torch.cuda.synchronize()
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    print(f"# T = {T} (K of the flush GEMM); TF/s of 2*M*N*T")
    print(f"{'case':10s} {'n_out':>6s} {'k_in':>6s} | {'II ms':>7s} {'TF/s':>6s} | {'KC^T ms':>7s} {'TF/s':>6s} | {'X^T copy ms':>11s}")
    shapes = [("qkv", 12288, 4096), ("out", 4096, 4096), ("dec", 28928, 4096), ("gpt fc1", 6400, 1600),
              ("gpt fc2", 1600, 6400)]
    if len(sys.argv) > 2 and sys.argv[2] == "gpt2xl":
        shapes = [("gpt qkv", 4800, 1600), ("gpt out", 1600, 1600), ("gpt fc1", 6400, 1600), ("gpt fc2", 1600, 6400)]
    for name, n_out, k_in in shapes:
        dy = torch.randn(T, n_out, device=dev).to(torch.bfloat16)
        x = torch.randn(T, k_in, device=dev).to(torch.bfloat16)
        xt = x.t().contiguous()
        fl = 2.0 * n_out * k_in * T
        # current: C[n_out, k_in] = dY^T X, A = dy as [K=T, M] (I-contiguous), B = x as [K=T, N]
        f_ii = lambda: k.gemm_f32(dy, x, False, False)
        # transposed: C^T[k_in, n_out] = X^T dY, A = xt [M=k_in, K=T] (K-contiguous), B = dy [K=T, N=n_out]
        f_kc = lambda: k.gemm_f32(xt, dy, True, False)
        f_tr = lambda: x.t().contiguous()
        a1, b1, c1 = timeit(f_ii), timeit(f_kc), timeit(f_tr)
        a2, b2, c2 = timeit(f_ii), timeit(f_kc), timeit(f_tr)
        a, b, c = min(a1, a2), min(b1, b2), min(c1, c2)
        ref = (dy[:256].float().t() @ x[:256].float())
        print(f"{name:10s} {n_out:6d} {k_in:6d} | {a:7.3f} {fl / a / 1e9:6.0f} | {b:7.3f} {fl / b / 1e9:6.0f} | {c:11.3f}",
              flush=True)
        del dy, x, xt, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
