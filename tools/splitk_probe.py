"""Split-K factor sweep for the deferred weight-gradient flush (linear_wgrad_segments: K-segmented over the
micro-batches, fp32 main_grad) at GPT-2-XL's shapes: the automatic factor (gemm_splitk_factor) against every
forced factor.  One process, warm clocks, medians; each factor timed twice in a rotated order.

    python tools/splitk_probe.py [T_per_microbatch] [microbatches] > profiles/splitk_probe.txt
"""
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe._native_loader import kernels  # noqa: E402

k = kernels()
dev = "cuda"


def timeit(fn, iters=8):
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
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 18432
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    xw = torch.randn(4096, 4096, device=dev).to(torch.bfloat16)
    for _ in range(200):
        k.linear_fwd(xw, xw, None, 0, 0.0, False)
    torch.cuda.synchronize()
    factors = [1, 2, 3, 4, 5, 6, 7, 8]  # 1 = unsplit; "auto" = gemm_splitk_factor's pick
    print(f"# T = {mb} x {T}; ms per flush GEMM (fp32 main_grad accumulate); auto = the factor the heuristic picks")
    print(f"{'case':8s} {'n_out':>5s} {'k_in':>5s} | {'auto':>6s} | " + " ".join(f"{'s=' + str(f):>6s}" for f in factors))
    for name, n_out, k_in in [("qkv", 4800, 1600), ("out", 1600, 1600), ("fc1", 6400, 1600), ("fc2", 1600, 6400)]:
        dys = [torch.randn(T, n_out, device=dev).to(torch.bfloat16) for _ in range(mb)]
        xs = [torch.randn(T, k_in, device=dev).to(torch.bfloat16) for _ in range(mb)]
        mg = torch.zeros(n_out, k_in, device=dev)
        run = lambda: k.linear_wgrad_segments(dys, xs, mg, True)  # noqa: E731
        res = {}
        for rep in range(2):
            order = ["auto"] + factors
            order = order[rep:] + order[:rep]
            for f in order:
                k.gemm_set_splitk(1 if f == "auto" else (0 if f == 1 else f))
                t = timeit(run)
                res[f] = min(res.get(f, t), t)
        k.gemm_set_splitk(1)
        print(f"{name:8s} {n_out:5d} {k_in:5d} | {res['auto']:6.3f} | " + " ".join(f"{res[f]:6.3f}" for f in factors),
              flush=True)
        del dys, xs, mg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
