"""The bench's PP plan pick, then its refinement from measured walls, with every rank emulated on ONE MI355X.

Runs what bench.py does at N > 1 (stage.candidate_plans -> each rank of each candidate emulated through the real
engine over loop-back channels -> the job step simulated from the walls with the IPC hop -> the fastest), then
calibrate.refine_plan_by_walls' moves (single units off the slowest measured rank, re-emulating the two ranks a
move changes) -- here all ranks in one process, so the predicted job step before and after can be compared.

    python tools/plan_refine_probe.py --config enc12_d4096 --pp 8 [--rounds 6] [--steps 2]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mipipe.models import CONFIGS  # noqa: E402
from mipipe.parallel.calibrate import (_move_candidates, calibrated_costs, emulate_rank_ms,  # noqa: E402
                                       engine_unit_costs)
from mipipe.parallel.stage import HOP_BYTES_PER_S, HOP_LATENCY_MS, StagePlan, candidate_plans, simulate_from_walls  # noqa: E402
from mipipe.pipeline import checkpoint_stop_for  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="enc12_d4096")
    ap.add_argument("--pp", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--refine-all", action="store_true", help="refine every candidate, not only the pick")
    ap.add_argument("--replan", action="store_true", help="re-plan from wall-corrected unit costs")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    pp = args.pp
    if args.config == "gpt2_xl":
        m, mb, ckpt = (8 if pp == 8 else 4 * pp), 18, "always"
    else:  # bench.py: micro-batch 128 at every N, chunks 4 x N, 'except_last' at PP=8 (config #3)
        m, mb, ckpt = 4 * pp, 128, ("except_last" if pp == 8 else "never")
    dev = torch.device("cuda", 0)
    bwd_ratio = 2.0 + {"never": 0.0, "except_last": (m - 1) / m, "always": 1.0}[ckpt]
    t0 = time.perf_counter()
    unit_ms = calibrated_costs(cfg, mb, m, ckpt, device=dev)
    print(f"# {cfg.name} PP={pp} chunks {m} mb {mb} {ckpt}: unit costs in {time.perf_counter() - t0:.1f} s", flush=True)
    stop = checkpoint_stop_for(ckpt, m)
    hop = HOP_LATENCY_MS + mb * cfg.seq_len * cfg.d_model * 2 / HOP_BYTES_PER_S * 1e3

    def step_of(plan, walls):
        return simulate_from_walls(plan, walls, engine_unit_costs(cfg, unit_ms, plan.split_decoder), m, stop, hop)[0]

    def emu(plan, r):
        w = emulate_rank_ms(cfg, plan, r, m, mb, ckpt, device=dev, steps=args.steps)
        torch.cuda.empty_cache()
        return w

    def refine(plan, walls, t):
        t0_ = t
        for k in range(args.rounds):
            slow, moves = _move_candidates(plan, walls)
            if not moves:
                print("   no move predicted to help", flush=True)
                break
            s, nb = moves[0]
            bal = list(plan.balance)
            bal[s] -= 1
            bal[nb] += 1
            new = StagePlan(bal, plan.costs, plan.virtual, plan.split_decoder)
            nw = list(walls)
            for r in {s % pp, nb % pp}:
                nw[r] = emu(new, r)
            t2 = step_of(new, nw)
            ok = t2 < t
            print(f"   round {k}: rank {slow} slowest ({walls[slow]:.1f} ms): vstage {s} -> {nb}; walls "
                  f"{[round(w) for w in nw]}, step {t2:.1f} ms ({'kept' if ok else 'rejected'})", flush=True)
            if not ok:
                break
            plan, walls, t = new, nw, t2
        print(f"   refined: {plan.balance}, step {t0_:.1f} -> {t:.1f} ms, {m * mb * cfg.seq_len / t * 1e3:,.0f} tok/s",
              flush=True)
        return plan, walls, t

    cands = candidate_plans(cfg, pp, m, bwd_ratio, mb, lambda s: engine_unit_costs(cfg, unit_ms, s))
    results = []
    for c in cands:
        walls = [emu(c, r) for r in range(pp)]
        t = step_of(c, walls)
        print(f"candidate v={c.virtual} split={c.split_decoder} {c.balance}: walls {[round(w) for w in walls]}, "
              f"step {t:.1f} ms, {m * mb * cfg.seq_len / t * 1e3:,.0f} tok/s", flush=True)
        results.append((t, c, walls))
    pick = min(results, key=lambda x: x[0])
    print(f"bench pick (no refinement): v={pick[1].virtual} step {pick[0]:.1f} ms", flush=True)
    if args.replan:
        # wall-corrected unit costs: every unit's cost scaled by its rank's measured / modelled ratio, averaged
        # over the emulated candidates of the same decoder split; plans re-made from them and emulated
        from mipipe.parallel.stage import plan_stages

        for split in sorted({c.split_decoder for _, c, _ in results}):
            base = engine_unit_costs(cfg, unit_ms, split)
            acc = [0.0] * len(base)
            n = 0
            for t, c, walls in results:
                if c.split_decoder != split:
                    continue
                n += 1
                for r in range(pp):
                    units = [u for s_ in c.vstages(r) for u in c.slice(s_)]
                    model = sum(base[u] for u in units) * m or 1.0
                    for u in units:
                        acc[u] += base[u] * walls[r] / model
            corrected = [a / n for a in acc]
            for v in (1, 2, 3):
                try:
                    p_ = plan_stages(cfg, pp, v, m, split, bwd_ratio, costs=corrected, objective="makespan")
                except ValueError:
                    continue
                p_ = StagePlan(list(p_.balance), base, v, split)  # priced with the measured unit costs again
                walls = [emu(p_, r) for r in range(pp)]
                t = step_of(p_, walls)
                print(f"replanned v={v} split={split} {p_.balance}: walls {[round(w) for w in walls]}, step {t:.1f} ms,"
                      f" {m * mb * cfg.seq_len / t * 1e3:,.0f} tok/s", flush=True)
                results.append((t, p_, walls))
    final = []
    for t, c, walls in (results if args.refine_all else [pick]):
        print(f"refining v={c.virtual} {c.balance}", flush=True)
        final.append(refine(c, walls, t))
    best = min(final, key=lambda x: x[2])
    print(f"best after refinement: v={best[0].virtual} {best[0].balance}, step {pick[0]:.1f} -> {best[2]:.1f} ms "
          f"({100 * (pick[0] / best[2] - 1):+.1f} % tok/s)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
