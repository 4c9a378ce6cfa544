"""LayerNorm backward at training shapes, for a same-box A/B of two builds: per-call time and the outputs.

    python tools/ln_bwd_ab.py ROOT TAG      # ROOT: repo root whose mipipe/_C.so to load; saves $TMPDIR/ln_bwd_TAG.pt
    python tools/ln_bwd_ab.py --compare TAG_A TAG_B   # bitwise comparison of the saved outputs

Inputs are generated on the CPU from fixed seeds, so both builds see the same bytes.
"""
import os
import statistics
import sys

import torch

CASES = [  # rows, cols, dtype, addend, p
    (8192, 4096, torch.bfloat16, True, 0.1),
    (8192, 4096, torch.bfloat16, True, 0.0),
    (8192, 4096, torch.bfloat16, False, 0.0),
    (8192, 1024, torch.bfloat16, True, 0.1),
    (4096, 4096, torch.float32, True, 0.1),
    # the wave-per-row kernel (<= 2048 columns): GPT-2-XL's 1600, ref_main's fp32 2048
    (18432, 1600, torch.bfloat16, True, 0.0),
    (18432, 1600, torch.bfloat16, False, 0.1),
    (8192, 2048, torch.float32, True, 0.1),
]


def _path(tag):  # outside gpurun_out/: the outputs are hundreds of MB
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"ln_bwd_{tag}.pt")


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
    for rows, cols, dtype, add, p in CASES:
        g = torch.Generator().manual_seed(rows + cols)
        z = torch.randn(rows, cols, generator=g).to(dtype)
        dy = torch.randn(rows, cols, generator=g).to(dtype)
        addend = torch.randn(rows, cols, generator=g).to(dtype) if add else None
        gamma = (1 + 0.1 * torch.randn(cols, generator=g)).to(dtype)
        zf = z.float()
        mean = zf.mean(-1)
        rstd = torch.rsqrt(zf.var(-1, unbiased=False) + 1e-5)
        z, dy, gamma, mean, rstd = (t.cuda() for t in (z, dy, gamma, mean, rstd))
        addend = addend.cuda() if add else None

        def run():
            return k.layernorm_bwd(dy, z, mean, rstd, gamma, p, 1234, 0, None, None, addend)

        res = run()
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
        nbytes = rows * cols * z.element_size() * (2 + (1 if add else 0) + 1 + (1 if p > 0 else 0))
        name = f"{rows}x{cols} {str(dtype)[6:]} add={int(add)} p={p}"
        print(f"{tag:4s} {name:34s} {t:8.1f} us  {nbytes / t / 1e6:5.2f} TB/s (rows in/out, excl. partials)", flush=True)
        for i, r in enumerate(res):
            if r is not None:
                out[f"{name} out{i}"] = r.cpu()
    torch.save(out, _path(tag))


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    main(sys.argv[1], sys.argv[2])
