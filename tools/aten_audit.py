"""Which ATen ops still launch GPU kernels inside a training step, and from where.

Builds the bench's PP=1 stage for a config (layer count reduced: the per-layer ops repeat),
runs two warm steps through PipelineEngine + FlatAdam exactly as bench.py does, then profiles
one step with Python stacks and prints every aten op that spent device time, grouped by its
innermost mipipe / bench frame.

    python tools/aten_audit.py [--config gpt2_xl] [--num-layers 2]
"""
import argparse
import collections
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from mipipe import ops  # noqa: E402
from mipipe.models import CONFIGS  # noqa: E402
from mipipe.optim import FlatAdam  # noqa: E402
from mipipe.parallel import PipelineEngine  # noqa: E402
from mipipe.parallel.stage import build_stage, plan_stages, stage_input_shape  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="gpt2_xl")
    ap.add_argument("--num-layers", type=int, default=2)
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--chunks", type=int, default=2)
    ap.add_argument("--checkpoint", default="always")
    args = ap.parse_args()
    import dataclasses

    cfg = dataclasses.replace(CONFIGS[args.config], num_layers=args.num_layers)
    dev = torch.device("cuda", 0)
    plan = plan_stages(cfg, 1, 1, args.chunks, split_decoder=False)
    torch.manual_seed(0)
    stages = [build_stage(cfg, plan, vs, device=dev, dtype=torch.bfloat16).train() for vs in plan.vstages(0)]
    opt = FlatAdam([p for s in stages for p in s.parameters()], lr=1e-4, max_grad_norm=0.5)
    V, m, mb = cfg.vocab, args.chunks, args.micro_batch

    def loss_fn(y, t):
        return ops.cross_entropy(y.reshape(-1, V), t.reshape(-1))

    shapes = [stage_input_shape(cfg, plan, vs, mb) for vs in plan.vstages(0)]
    engine = PipelineEngine(stages, chunks=m, checkpoint=args.checkpoint, act_shape=shapes,
                            act_dtype=torch.bfloat16, loss_fn=loss_fn, device=dev)
    tokens = torch.randint(0, V, (m, mb, cfg.seq_len + 1))
    inputs = [tokens[i, :, :cfg.seq_len].to(dev) for i in range(m)]
    targets = [tokens[i, :, 1:].contiguous().to(dev) for i in range(m)]

    def step():
        opt.zero_grad()
        engine.step(inputs, targets)
        opt.step(opt.grad_sumsq())

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    kern = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    native = [e for e in kern if "mipipe" not in e.name]
    print(f"# {args.config} x{args.num_layers} layers, chunks {m} x mb {mb}, {args.checkpoint}: {len(kern)} kernels "
          f"in the step, {len(native)} not from mipipe", flush=True)
    groups = collections.Counter()
    for e in prof.events():
        if e.device_type != torch.autograd.DeviceType.CPU or not e.name.startswith("aten::"):
            continue
        if getattr(e, "self_device_time_total", 0) <= 0:
            continue
        frames = [f for f in (e.stack or []) if ("mipipe" in f or "bench" in f or "tools" in f)
                  and "aten_audit" not in f]
        where = frames[0] if frames else "(no Python frame: autograd thread)"
        shapes = str(getattr(e, "input_shapes", "") or "")[:70]
        groups[(e.name, where, shapes)] += 1
    for (name, where, shapes), n in groups.most_common(40):
        print(f"{n:4d}  {name:24s} {shapes:72s} {where}")


if __name__ == "__main__":
    main()
