"""Which PP=8 stage plan is fastest?  Every alternative the planner can produce,
each rank emulated on ONE MI355X.

For a BASELINE config (#3: enc12_d4096, chunks 32, micro-batch 64 -- the
bench's default until round 6, 128 since -- 'except_last'; #4: GPT-2-XL, chunks 8, micro-batch 18,
'always'),
the plans are: unit costs {analytic FLOPs, measured engine-context costs} x
objective {makespan, balance} x chunks per rank v (the decoder split chosen per
v by the same simulation the planner uses), plus the plan ``bench.py``
builds by default.  Identical plans are emulated once.

Each rank of a plan runs through the real PipelineEngine over loop-back
channels (``tools/pp_rank_emulation.run_rank``: the GPU executes exactly that
rank's kernels in its schedule, optimizer step included).  The job step is
then simulated from those MEASURED walls -- each rank's wall split over its
virtual stages in proportion to their measured unit costs, recompute explicit,
deferred weight gradients, and the stage transport's hop (IPC over xGMI:
0.15 ms + message / 100 GB/s, profiles/pp8_transport_prediction_r5.txt) --
so per-chunk boundary work the unit costs miss is in the walls.

    python tools/plan_table.py --config enc12_d4096 [--v 1,2,3,4] [--steps 4]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from mipipe.models import CONFIGS  # noqa: E402
from mipipe.parallel.calibrate import calibrated_costs, engine_unit_costs  # noqa: E402
from mipipe.parallel.stage import candidate_plans, choose_virtual, simulate_from_walls  # noqa: E402
from mipipe.pipeline import checkpoint_stop_for  # noqa: E402
from pp_rank_emulation import run_rank  # noqa: E402

# the bench's defaults per model and PP (bench.py: chunks, _default_micro_batch, checkpoint 'auto'): BASELINE
# config #2 (enc12, chunks 4 x PP, 'never'), #3 (its PP=8 run: 'except_last'), #4 (GPT-2-XL, chunks 8 at PP=8)
CONFIG = {"enc12_d4096": (32, 64, "except_last"), "gpt2_xl": (8, 18, "always")}


def bench_defaults(name: str, pp: int):
    if name == "gpt2_xl":
        return (8 if pp == 8 else 4 * pp), 18, "always"
    return 4 * pp, 128, ("except_last" if pp == 8 else "never")  # micro-batch 128 at every N since round 6
HOP_MS = 0.15
XGMI_BYTES_PER_S = 100e9


def job_step_ms(cfg, plan, walls, unit_ms, m, mb, ckpt):
    """Simulated PP step from measured rank walls (stage.simulate_from_walls, as the bench's pick)."""
    hop = HOP_MS + mb * cfg.seq_len * cfg.d_model * 2 / XGMI_BYTES_PER_S * 1e3
    return simulate_from_walls(plan, walls, engine_unit_costs(cfg, unit_ms, plan.split_decoder), m,
                               checkpoint_stop_for(ckpt, m), hop)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="enc12_d4096", choices=sorted(CONFIG))
    ap.add_argument("--pp", type=int, default=8)
    ap.add_argument("--v", default="1,2,3,4", help="chunks per rank to try")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--labels", default=None,
                    help="comma list of plan labels (e.g. DEFAULT,analytic/makespan/v=4): emulate only those plans, "
                         "--repeats times each, alternating (run-to-run noise of the comparison)")
    ap.add_argument("--repeats", type=int, default=1)
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    pp = args.pp
    m, mb, ckpt = bench_defaults(args.config, pp)
    args.chunks, args.micro_batch, args.checkpoint = m, mb, ckpt
    dev = torch.device("cuda", 0)
    bwd_ratio = 2.0 + {"never": 0.0, "except_last": (m - 1) / m, "always": 1.0}[ckpt]
    t0 = time.perf_counter()
    unit_ms = calibrated_costs(cfg, mb, m, ckpt, device=dev)
    print(f"# {cfg.name} PP={pp}, chunks {m}, micro-batch {mb} x {cfg.seq_len}, {ckpt}; measured engine-context unit "
          f"costs ({time.perf_counter() - t0:.1f} s, ms per micro-batch): "
          + ", ".join(f"{k} {c:.3f}" for k, c in sorted(unit_ms.items())), flush=True)

    def cost_fn_for(kind):
        return (lambda split: engine_unit_costs(cfg, unit_ms, split)) if kind == "measured" else None

    plans = {}  # (v, split, balance) -> (plan, [labels])

    def add(label, v, plan):
        key = (v, plan.split_decoder, tuple(plan.balance))
        plans.setdefault(key, (plan, []))[1].append(label)

    # the bench's default at PP > 1 on GPUs: the cost model's few best plans (stage.candidate_plans), the pick made
    # from their emulated rank walls (calibrate.select_plan_by_emulation) -- i.e. the best of the "candidate" rows
    for cp in candidate_plans(cfg, pp, m, bwd_ratio, mb, cost_fn_for("measured")):
        add("candidate", cp.virtual, cp)
    # the cost model alone (round 4's default, before the emulated pick)
    v0, p0 = choose_virtual(cfg, pp, m, bwd_ratio=bwd_ratio, micro_batch=mb, cost_fn=cost_fn_for("measured"),
                            objective="makespan")
    add("model-default", v0, p0)
    for kind in ("analytic", "measured"):
        for obj in ("makespan", "balance"):
            va, pa = choose_virtual(cfg, pp, m, bwd_ratio=bwd_ratio, micro_batch=mb, cost_fn=cost_fn_for(kind),
                                    objective=obj)
            add(f"{kind}/{obj}/auto", va, pa)
            for v in (int(x) for x in args.v.split(",")):
                try:
                    vv, pv = choose_virtual(cfg, pp, m, candidates=[v], bwd_ratio=bwd_ratio, micro_batch=mb,
                                            cost_fn=cost_fn_for(kind), objective=obj)
                except (TypeError, ValueError, IndexError):
                    continue
                add(f"{kind}/{obj}/v={v}", vv, pv)
    print(f"# {len(plans)} distinct plans", flush=True)
    todo = list(plans.items())
    if args.labels:
        want = set(args.labels.split(","))
        todo = [kv for kv in todo if want & set(kv[1][1])] * args.repeats
    rows = []
    for (v, split, bal), (plan, labels) in todo:
        print(f"## plan v={v} split={split} balance={list(bal)}: {', '.join(labels)}", flush=True)
        walls = []
        for r in range(pp):
            walls.append(run_rank(args, cfg, plan, v, r))
            torch.cuda.empty_cache()
        t, bub = job_step_ms(cfg, plan, walls, unit_ms, m, mb, ckpt)
        tps = m * mb * cfg.seq_len / t * 1e3
        rows.append((tps, t, bub, v, split, min(walls), max(walls), labels))
        print(f"   walls {min(walls):.1f}-{max(walls):.1f} ms ({100 * (max(walls) / min(walls) - 1):.1f} %), "
              f"job step {t:.1f} ms, bubble {100 * bub:.1f} %, {tps:,.0f} tok/s", flush=True)
    rows.sort(reverse=True)
    print(f"\n# {cfg.name} PP={pp} chunks {m} mb {mb} {ckpt}: plans by predicted job tok/s (measured rank walls, "
          f"simulated step with the IPC hop)")
    print(f"  {'job tok/s':>10s} {'step ms':>8s} {'bubble':>7s} {'v':>2s} {'split':>5s} {'rank walls ms':>15s}  plans")
    for tps, t, bub, v, split, lo, hi, labels in rows:
        print(f"  {tps:10,.0f} {t:8.1f} {100 * bub:6.1f}% {v:2d} {str(split):>5s} {lo:7.1f}-{hi:7.1f}  "
              f"{', '.join(labels)}")
    best = rows[0]
    if args.labels:
        return 0
    default = next(r for r in rows if "candidate" in r[7])  # rows are sorted: the emulated pick
    model = next(r for r in rows if "model-default" in r[7])
    print(f"# bench default (best emulated candidate): {default[0]:,.0f} tok/s = {100 * default[0] / best[0]:.1f} % "
          f"of the best ({', '.join(best[7])}); the cost model's own pick: {100 * model[0] / best[0]:.1f} %")
    return 0


if __name__ == "__main__":
    sys.exit(main())
