"""Bias + activation + dropout kernels (forward and backward) at GPT-2-XL's fc1 shape, for a same-box A/B of two
builds: per-call time and the outputs.

    python tools/bias_act_ab.py ROOT TAG                 # ROOT: repo root whose mipipe/_C.so to load
    python tools/bias_act_ab.py --compare TAG_A TAG_B    # max |difference| of the saved outputs

Inputs are generated on the CPU from fixed seeds; the forward's dropout seed comes from torch.cuda.manual_seed.
"""
import os
import statistics
import sys

import torch

ROWS, COLS = 18432, 6400
CASES = [  # name, backward, act (0 none, 1 relu, 2 gelu), p
    ("gelu bwd p=0.1", True, 2, 0.1),
    ("gelu bwd p=0", True, 2, 0.0),
    ("relu bwd p=0.1", True, 1, 0.1),
    ("drop bwd p=0.1", True, 0, 0.1),
    ("gelu fwd p=0.1", False, 2, 0.1),
]


def _path(tag):  # outside gpurun_out/: the outputs are hundreds of MB
    return os.path.join(os.environ.get("TMPDIR", "/tmp"), f"bias_act_{tag}.pt")


def compare(a, b):
    ra = torch.load(_path(a), weights_only=True)
    rb = torch.load(_path(b), weights_only=True)
    for key in ra:
        d = (ra[key].float() - rb[key].float()).abs()
        scale = rb[key].float().abs().max().item()
        print(f"{key:20s} equal={torch.equal(ra[key], rb[key])}  max |diff| {d.max().item():.3g} "
              f"(max |value| {scale:.3g}), differing {(d > 0).float().mean().item() * 100:.3f} %")


def main(root, tag):
    sys.path.insert(0, root)
    from mipipe._native_loader import kernels

    k = kernels()
    g = torch.Generator().manual_seed(7)
    dy = torch.randn(ROWS, COLS, generator=g).to(torch.bfloat16).cuda()
    pre = torch.randn(ROWS, COLS, generator=g).to(torch.bfloat16).cuda()
    bias = (0.1 * torch.randn(COLS, generator=g)).to(torch.bfloat16).cuda()
    out = {}
    for name, bwd, act, p in CASES:
        if bwd:
            # relu reads the op's output as `saved`; gelu the pre-bias input
            def run():
                return k.bias_act_bwd(dy, pre, bias, act, p, 1234, 0, False)[0]
        else:
            def run():
                torch.cuda.manual_seed(11)
                return k.bias_act_fwd(pre, bias, act, p)[0]
        res = run()
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(30):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            run()
            e.record()
            e.synchronize()
            ts.append(s.elapsed_time(e) * 1e3)
        t = statistics.median(ts)
        nbytes = ROWS * COLS * 2 * (3 if bwd and act else 2)
        print(f"{tag:4s} {name:16s} {t:8.1f} us  {nbytes / t / 1e6:5.2f} TB/s", flush=True)
        out[name] = res.cpu()
    torch.save(out, _path(tag))


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        main(sys.argv[1], sys.argv[2])
