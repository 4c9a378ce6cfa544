"""Per-GEMM-class roofline of the enc12 PP=1 training step from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace -d gpurun_out/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-bubble
    python tools/gemm_roofline.py gpurun_out/prof/run_results.db --steps 6 --gfxclk 1930

The bench's default shapes (enc12_d4096, micro-batch 128 x 128 = 16,384 tokens, chunks 4, 'never'): every GEMM
class is identified by its kernel instantiation and grid (tiles = grid_x / 512 threads), its FLOPs follow from
the model, and the dgrads -- one instantiation and grid for K = 4096 / 12,288 / 28,782 -- are told apart by
duration (about 1x / 3x / 7x the K = 4096 median).  The roofline is the dense bf16 MFMA peak at the given
gfxclk: 2.5 PF/s x gfxclk / 2400 MHz (the step's mean clock from the bench JSON telemetry; the GEMM phases
themselves sit at the 1400 W cap, ~1.8 GHz, profiles/gemm_clock_r5.txt).
"""
from __future__ import annotations

import argparse
import sqlite3
import statistics
from collections import defaultdict

D, FF, V = 4096, 4096, 28782
T = 16384       # tokens per micro-batch (--tokens)
TSTEP = 4 * T   # the deferred weight-gradient GEMMs run over the step's 4 micro-batches


def classify(name: str, grid: int, dur_ns: float, dg_median: float):
    """(class, flops) of one GEMM dispatch, or None for other kernels."""
    if "gemm256_kernel" not in name:
        return None
    tpl = name[name.index("<") + 1:name.index(">")].replace(" ", "").split(",")
    a_kc, b_kc, epi, act = tpl[0] == "true", tpl[1] == "true", int(tpl[2]), int(tpl[3])
    tiles = grid // 512
    if a_kc and b_kc:  # forward
        if tiles == (T // 256) * (3 * D // 256):
            return "fwd qkv", 2.0 * T * 3 * D * D
        if tiles == (T // 256) * ((V + 255) // 256):
            return "fwd decoder", 2.0 * T * V * D
        if tiles == (T // 256) * (D // 256):
            return ("fwd fc1 (ReLU + dropout epilogue)" if act == 1 else "fwd out / fc2"), 2.0 * T * D * D
        return "fwd other", None
    if a_kc and not b_kc and epi == 0:  # dgrad: dX [T, 4096] = dY . W, K = the layer's output width
        r = dur_ns / dg_median
        if r < 1.8:
            return "dgrad out / fc1 / fc2 (K 4096)", 2.0 * T * D * D
        if r < 4.5:
            return "dgrad qkv (K 12288)", 2.0 * T * D * 3 * D
        return "dgrad decoder (K 28782)", 2.0 * T * D * V
    if not a_kc and not b_kc and epi in (1, 2):
        return "wgrad out / fc1 / fc2 (both I-contiguous)", 2.0 * D * D * TSTEP
    if a_kc and not b_kc and epi in (1, 2):  # transposed weight gradient (x^T from the flush's transpose)
        if tiles == 3 * D // 256 * D // 256:
            return "wgrad qkv (x^T, K-contiguous A)", 2.0 * 3 * D * D * TSTEP
        return "wgrad decoder (x^T, by rounds)", 2.0 * tiles * 256 * 256 * TSTEP  # per chunk: its own tiles
    return "other", None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, required=True, help="steps in the trace (warm-up included)")
    ap.add_argument("--gfxclk", type=float, required=True, help="MHz, the step's mean (bench JSON telemetry)")
    ap.add_argument("--tokens", type=int, default=16384, help="tokens per micro-batch (micro-batch x 128)")
    args = ap.parse_args()
    global T, TSTEP
    T, TSTEP = args.tokens, 4 * args.tokens
    con = sqlite3.connect(args.db)
    rows = con.execute("select name, grid_x, duration from kernels").fetchall()
    dg = [d for n, g, d in rows if "gemm256_kernel<true, false, 0, 0" in n and g // 512 == (T // 256) * (D // 256)]
    dg_med = statistics.median(dg) if dg else 1.0
    tot_ns = sum(d for _, _, d in rows)
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for n, g, d in rows:
        c = classify(n, g, d, dg_med)
        if c is None:
            continue
        cls, fl = c
        a = agg[cls]
        a[0] += 1
        a[1] += d
        a[2] += fl or 0.0
    peak = 2.5e15 * args.gfxclk / 2400.0
    s = args.steps
    print(f"# {args.db}: {s} steps, all kernels {tot_ns / 1e6 / s:.1f} ms per step; MFMA roofline at "
          f"{args.gfxclk:.0f} MHz = {peak / 1e15:.3f} PF/s dense bf16")
    print(f"{'class':<44} {'calls/step':>10} {'us/call':>9} {'ms/step':>8} {'PF/s':>6} {'% roof':>7}")
    gsum_ns = gsum_fl = 0.0
    for cls, (k, ns, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        rate = fl / (ns * 1e-9) if fl and ns else 0.0
        gsum_ns += ns
        gsum_fl += fl
        print(f"{cls:<44} {k / s:10.1f} {ns / k / 1e3:9.1f} {ns / s / 1e6:8.2f} {rate / 1e15:6.3f} "
              f"{100 * rate / peak:6.1f}%")
    print(f"{'all GEMMs':<44} {'':>10} {'':>9} {gsum_ns / s / 1e6:8.2f} {gsum_fl / gsum_ns / 1e6:6.3f} "
          f"{100 * gsum_fl / (gsum_ns * 1e-9) / peak:6.1f}%   ({100 * gsum_ns / tot_ns:.1f} % of kernel time)")


if __name__ == "__main__":
    main()
