"""fp32 GEMM timing on the reference config's shapes (ref_main: T = 1024 tokens per
micro-batch, E = FF = 2048, V = 28,784 padded): mipipe's v_mfma_f32_32x32x2_f32
kernel (gemm_f32.hip) vs hipBLASLt fp32 (torch.matmul), interleaved, one process.

    python tools/bench_gemm_f32.py [T] > profiles/gemm_f32_vs_hipblaslt.txt
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
dev = "cuda"
torch.backends.cuda.matmul.allow_tf32 = False


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


def main(T=int(sys.argv[1]) if len(sys.argv) > 1 else 1024):
    E = 2048
    shapes = [("qkv", T, 3 * E, E), ("out", T, E, E), ("ffn", T, E, E), ("dec", T, 28928, E)]
    cfg = os.environ.get("MIPIPE_GEMM_F32_CFG", "0 (auto)")
    print(f"# fp32 GEMM, T={T}, MIPIPE_GEMM_F32_CFG={cfg}; TF/s = 2MNK / time; fp32 MFMA peak 157 TF/s")
    print(f"{'case':12s} {'M':>6s} {'N':>6s} {'K':>6s} | {'mipipe ms':>9s} {'TF/s':>7s} | {'hipBLASLt ms':>12s} {'TF/s':>7s}")
    tot_m = tot_h = 0.0
    for name, M, N, K in shapes:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        fl = 2.0 * M * N * K
        rows = []
        rows.append((f"{name} fwd", M, N, K, timeit(lambda: k.linear_fwd(x, w, None, 0, 0.0, False)),
                     timeit(lambda: torch.matmul(x, w.t()))))
        dy = torch.randn(M, N, device=dev)
        rows.append((f"{name} dgrad", M, K, N, timeit(lambda: k.linear_dgrad(dy, w)), timeit(lambda: torch.matmul(dy, w))))
        mg = torch.zeros(N, K, device=dev)
        rows.append((f"{name} wgrad+acc", N, K, M, timeit(lambda: k.linear_wgrad(dy, x, mg)),
                     timeit(lambda: mg.add_(torch.matmul(dy.t(), x)))))
        for case, a, b, c, tm, th in rows:
            tot_m += tm
            tot_h += th
            print(f"{case:12s} {a:6d} {b:6d} {c:6d} | {tm:9.3f} {fl / tm / 1e9:7.0f} | {th:12.3f} {fl / th / 1e9:7.0f}")
    print(f"{'total':12s} {'':6s} {'':6s} {'':6s} | {tot_m:9.3f} {'':7s} | {tot_h:12.3f}")


if __name__ == "__main__":
    main()
