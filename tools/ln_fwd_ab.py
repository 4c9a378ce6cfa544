"""LayerNorm forward (both kernels: one row per block above 2048 columns, one per wave up to 2048) at training shapes, for a same-box
A/B of two builds: per-call time and the outputs.

    python tools/ln_fwd_ab.py ROOT TAG                # ROOT: repo root whose mipipe/_C.so to load
    python tools/ln_fwd_ab.py --compare TAG_A TAG_B   # bitwise comparison of the saved outputs

Inputs are generated on the CPU from fixed seeds; the dropout seed comes from torch.cuda.manual_seed.
"""
import os
import statistics
import sys

import torch

CASES = [  # rows, cols, dtype, residual, p
    (8192, 4096, torch.bfloat16, True, 0.1),
    (8192, 4096, torch.bfloat16, True, 0.0),
    (8192, 4096, torch.float32, True, 0.1),
    (4096, 8192, torch.bfloat16, True, 0.1),
    # the wave-per-row kernel (<= 2048 columns): GPT-2-XL's pre-norm 1600, ref_main's fp32 2048
    (18432, 1600, torch.bfloat16, False, 0.0),
    (8192, 2048, torch.float32, True, 0.1),
]


def _path(tag):  # outside gpurun_out/: the outputs are hundreds of MB
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"ln_fwd_{tag}.pt")


def compare(a, b):
    ra = torch.load(_path(a), weights_only=True)
    rb = torch.load(_path(b), weights_only=True)
    bad = 0
    for key in ra:
        same = torch.equal(ra[key], rb[key])
        bad += not same
        if not same:
            print(f"{key}: differ, max abs {(ra[key].float() - rb[key].float()).abs().max().item():.3g}")
    print(f"{len(ra) - bad}/{len(ra)} outputs bitwise equal")
    return bad == 0


def main(root, tag):
    sys.path.insert(0, root)
    from mipipe._native_loader import kernels

    k = kernels()
    out = {}
    for rows, cols, dtype, res, p in CASES:
        g = torch.Generator().manual_seed(rows + cols)
        x = torch.randn(rows, cols, generator=g).to(dtype).cuda()
        r = torch.randn(rows, cols, generator=g).to(dtype).cuda() if res else None
        gamma = (1 + 0.1 * torch.randn(cols, generator=g)).to(dtype).cuda()
        beta = (0.1 * torch.randn(cols, generator=g)).to(dtype).cuda()

        def run():
            torch.cuda.manual_seed(3)
            return k.layernorm_fwd(x, r, gamma, beta, 1e-5, p, True)

        y = run()
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(40):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            run()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        t = statistics.median(ts)
        nbytes = rows * cols * x.element_size() * (1 + (1 if res else 0) + 2)
        name = f"{rows}x{cols} {str(dtype)[6:]} res={int(res)} p={p}"
        print(f"{tag:4s} {name:34s} {t:8.1f} us  {nbytes / t / 1e6:5.2f} TB/s (x, res in; y, z out)", flush=True)
        for i, o in enumerate(y[:4]):
            if o is not None:
                out[f"{name} out{i}"] = o.cpu()
    torch.save(out, _path(tag))


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    main(sys.argv[1], sys.argv[2])
