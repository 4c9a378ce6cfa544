"""One pipeline rank of a PP=8 enc12_d4096 run, emulated on ONE MI355X without transport.

The rank's two looping chunks (the plan bench.py builds at PP=8: chunks=32,
micro-batch 32 x 128, except_last) run through the real PipelineEngine with a
loopback channel (sends and receives complete immediately; receive buffers
hold random activations / gradients), so the GPU executes exactly the rank's
kernels in the rank's schedule.  Reported:

* wall   -- host wall time of one step (host issue + GPU), synchronised.
Run it under ``rocprofv3 --kernel-trace --stats``: total kernel time divided by
the steps executed is the GPU busy time per step; busy / wall is the share of
the step the GPU spends in kernels (the rest is launch gaps and host waits).
(Issuing a step behind a long sleep kernel does not isolate the GPU time: the
host blocks once the queue holds a few thousand packets.)

    python tools/pp_rank_emulation.py [--rank R] [--steps N]
    python tools/pp_rank_emulation.py --config gpt2_xl --ranks all   # every rank in turn, one table

With ``--ranks all`` the table ends with the PP-step estimate these per-rank
times give: the slowest rank's wall x (1 + the planner's simulated bubble
share), and the tokens/s that implies for the whole job.
"""
import argparse
import statistics
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])

from mipipe import ops  # noqa: E402
from mipipe.models import CONFIGS  # noqa: E402
from mipipe.optim import FlatAdam  # noqa: E402
from mipipe.parallel import PipelineEngine  # noqa: E402
from mipipe.parallel.stage import build_stage, choose_virtual, stage_input_shape  # noqa: E402


from mipipe.parallel.calibrate import Loopback  # noqa: E402


# per-config defaults: BASELINE.json's PP=8 configs (#3 enc12 chunks 32 except_last, #4 GPT-2-XL chunks 8 always)
DEFAULTS = {"enc12_d4096": (32, 32, "except_last"), "gpt2_xl": (8, 18, "always")}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="enc12_d4096", choices=sorted(DEFAULTS))
    ap.add_argument("--rank", type=int, default=-1, help="pipeline rank to emulate (default: the most loaded)")
    ap.add_argument("--ranks", default=None, help="'all' or a comma list: emulate these ranks in turn")
    ap.add_argument("--pp", type=int, default=8)
    ap.add_argument("--chunks", type=int, default=None)
    ap.add_argument("--micro-batch", type=int, default=None)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--checkpoint", default=None)
    ap.add_argument("--objective", default="makespan", choices=["makespan", "balance"],
                    help="planner objective (mipipe.parallel.stage.plan_stages)")
    ap.add_argument("--plan", default="analytic", choices=["analytic", "measured"],
                    help="stage-plan unit costs: analytic FLOPs or measured unit times (mipipe.parallel.calibrate)")
    args = ap.parse_args()
    d_chunks, d_mb, d_ck = DEFAULTS[args.config]
    args.chunks = args.chunks or d_chunks
    args.micro_batch = args.micro_batch or d_mb
    args.checkpoint = args.checkpoint or d_ck

    cfg = CONFIGS[args.config]
    pp, m, mb = args.pp, args.chunks, args.micro_batch
    recompute = {"never": 0.0, "except_last": (m - 1) / m, "always": 1.0}[args.checkpoint]
    cost_fn = None
    if args.plan == "measured":
        from mipipe.parallel.calibrate import calibrated_costs, engine_unit_costs

        t0 = time.perf_counter()
        costs = calibrated_costs(cfg, mb, m, args.checkpoint, device=torch.device("cuda", 0))
        print(f"# measured engine-context unit costs (ms per micro-batch, {time.perf_counter() - t0:.1f} s): "
              + ", ".join(f"{k} {c:.3f}" for k, c in sorted(costs.items())), flush=True)
        cost_fn = lambda split: engine_unit_costs(cfg, costs, split)  # noqa: E731
    virtual, plan = choose_virtual(cfg, pp, m, bwd_ratio=2.0 + recompute, micro_batch=mb, cost_fn=cost_fn,
                                   objective=args.objective)
    print(f"# plan ({args.plan} costs, {args.objective}): v={virtual}, split head {plan.split_decoder}, "
          f"balance {plan.balance}", flush=True)
    if args.ranks:
        ranks = list(range(pp)) if args.ranks == "all" else [int(r) for r in args.ranks.split(",")]
    else:
        ranks = [args.rank if args.rank >= 0 else max(range(pp), key=plan.rank_cost)]
    walls = {}
    for rank in ranks:
        walls[rank] = run_rank(args, cfg, plan, virtual, rank)
        torch.cuda.empty_cache()
    if len(walls) > 1:
        from mipipe.parallel.stage import simulate_step
        from mipipe.pipeline import checkpoint_stop_for

        slow = max(walls, key=walls.get)
        bwd_ratio = 2.0 + recompute  # as bench.py prices the plan, recompute explicit in the simulation
        sim_t, sim_busy = simulate_step([plan.stage_cost(g) * 3.0 / (1.0 + bwd_ratio) for g in range(pp * virtual)],
                                        pp, virtual, m, 2.0, deferred_w=0.5,
                                        checkpoint_stop=checkpoint_stop_for(args.checkpoint, m))
        bub = 1.0 - max(sim_busy) / sim_t  # the slowest rank's idle share
        est = walls[slow] * (1.0 + bub)
        tokens = m * mb * cfg.seq_len
        fastest = min(walls.values())
        print(f"# per-rank wall spread: {fastest:.1f} .. {walls[slow]:.1f} ms = "
              f"{100 * (walls[slow] / fastest - 1):.1f} % ({args.plan} plan costs, {args.objective})")
        print(f"# slowest rank {slow}: {walls[slow]:.1f} ms/step; planner-simulated bubble {100 * bub:.1f} % -> "
              f"PP={pp} step ~{est:.1f} ms = {tokens / est * 1e3:,.0f} tokens/s for the job "
              f"({m} x {mb} x {cfg.seq_len} tokens per step)")
    return 0


def run_rank(args, cfg, plan, virtual, rank) -> float:
    dev = torch.device("cuda", 0)
    pp, m, mb = args.pp, args.chunks, args.micro_batch
    torch.manual_seed(0)
    stages = [build_stage(cfg, plan, vs, device=dev, dtype=torch.bfloat16).train() for vs in plan.vstages(rank)]
    shapes = [stage_input_shape(cfg, plan, vs, mb) for vs in plan.vstages(rank)]
    opt = FlatAdam([p for s in stages for p in s.parameters()], lr=1e-4, max_grad_norm=0.5)
    last = any(vs == pp * virtual - 1 for vs in plan.vstages(rank))
    V = cfg.vocab

    def loss_fn(y, t):
        return ops.cross_entropy(y.reshape(-1, V), t.reshape(-1))

    engine = PipelineEngine(stages, chunks=m, checkpoint=args.checkpoint, act_shape=shapes, act_dtype=torch.bfloat16,
                            loss_fn=loss_fn if last else None, group=Loopback(rank, pp), device=dev,
                            skip_routes={})
    g = torch.Generator(device="cpu").manual_seed(0)
    tokens = torch.randint(0, V, (m, mb, cfg.seq_len + 1), generator=g)
    inputs = [tokens[i, :, :cfg.seq_len].to(dev) for i in range(m)] if rank == 0 else None
    targets = [tokens[i, :, 1:].contiguous().to(dev) for i in range(m)]
    params = sum(p.numel() for p in opt.params)
    print(f"# PP={pp} rank {rank} of {cfg.name} (plan v={virtual}, split head {plan.split_decoder}, "
          f"vstages {plan.vstages(rank)}, units {[len(plan.slice(v)) for v in plan.vstages(rank)]}), "
          f"{params / 1e6:.1f}M params, chunks {m} x micro-batch {mb} x {cfg.seq_len}, {args.checkpoint}")

    def step():
        opt.zero_grad()
        engine.step(inputs, targets)
        opt.step(opt.grad_sumsq())

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    walls = []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        walls.append((time.perf_counter() - t0) * 1e3)
    wall = statistics.median(walls)
    total = 2 + args.steps
    print(f"wall {wall:.2f} ms/step (median of {args.steps}); {total} steps executed in all -- GPU busy per step = "
          f"rocprofv3 total kernel time / {total}", flush=True)
    del engine, opt, stages
    return wall


if __name__ == "__main__":
    sys.exit(main())
