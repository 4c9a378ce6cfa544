"""Stage planning: which blocks of a model each pipeline rank owns.

Costs are analytic training FLOPs per token of each block (plus a small
memory-traffic term for FLOP-free blocks such as the embedding), so ranks can
decide their slice *before* instantiating anything -- no rank ever builds the
whole 1.2B-parameter model.  The split minimises the slowest stage
(``mipipe.balance.blockpartition``), with stage boundaries allowed between the
attention and MLP halves of a layer.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
from torch import nn

from ..balance import balance_cost
from ..models.lm import LMConfig, TargetSequential, build_lm_blocks, lm_pipeline_units
from ..models.transformer import merge_units
from ..models.vocab_split import STAT_SLOTS, split_point
from ..ops.linear import mark_gemm_weight

__all__ = ["StagePlan", "plan_stages", "block_costs", "stage_input_shape", "build_stage", "simulate_step", "choose_virtual"]


@dataclass
class StagePlan:
    """Units per VIRTUAL stage (``len(balance) == ranks * virtual``); rank ``r``
    owns virtual stages ``r, r + ranks, ...`` (looping placement)."""

    balance: List[int]
    costs: List[float]
    virtual: int = 1
    split_decoder: bool = False  # decoder cut along the vocabulary into two units

    @property
    def ranks(self) -> int:
        return len(self.balance) // self.virtual

    def slice(self, vstage: int) -> range:
        start = sum(self.balance[:vstage])
        return range(start, start + self.balance[vstage])

    def vstages(self, rank: int) -> List[int]:
        return [c * self.ranks + rank for c in range(self.virtual)]

    def stage_cost(self, vstage: int) -> float:
        return sum(self.costs[i] for i in self.slice(vstage))

    def rank_cost(self, rank: int) -> float:
        return sum(self.stage_cost(s) for s in self.vstages(rank))

    def imbalance(self) -> float:
        """max rank cost / mean rank cost (1.0 = perfect)."""
        per = [self.rank_cost(r) for r in range(self.ranks)]
        return max(per) / (sum(per) / len(per))


def block_costs(cfg: LMConfig, split_decoder: bool = False) -> List[float]:
    """Training FLOPs per token of the pipeline units
    ``[Encoder, (attn core, attn out, mlp in, mlp out) x L, (final norm), Decoder]``
    (see ``mipipe.models.transformer.pipeline_units``)."""
    e, f, s, v = cfg.d_model, cfg.dim_feedforward, cfg.seq_len, cfg.vocab
    causal = 0.5 if cfg.causal else 1.0
    core = 3.0 * (2 * 3 * e * e + 4 * s * e * causal) + 3.0 * 10 * e
    out = 3.0 * (2 * e * e) + 3.0 * 10 * e  # + LN/dropout traffic
    mlp_in = 3.0 * (2 * e * f) + 3.0 * 5 * f
    mlp_out = 3.0 * (2 * e * f) + 3.0 * 10 * e
    enc = 3.0 * 40 * e  # gather + scatter-add traffic, expressed in FLOP-equivalents
    dec = 3.0 * (2 * e * v) + 3.0 * 4 * v  # GEMM + cross-entropy passes
    costs = [enc]
    for _ in range(cfg.num_layers):
        costs += [core, out, mlp_in, mlp_out]
    if cfg.norm_first:
        costs.append(3.0 * 10 * e)
    if split_decoder:
        va = split_point(v)
        costs += [dec * va / v, dec * (v - va) / v]
    else:
        costs.append(dec)
    return costs


def _rank_balanced(costs: List[float], ranks: int, virtual: int) -> List[int]:
    """Contiguous split into ranks*virtual groups minimising the largest RANK
    total (sum of its virtual stages), then the largest group: start from the
    per-group min-max split and move single boundaries while that improves."""
    groups = ranks * virtual
    bal = balance_cost(costs, groups)
    prefix = [0.0]
    for c in costs:
        prefix.append(prefix[-1] + c)

    def score(b: List[int]) -> Tuple[float, float]:
        per_rank = [0.0] * ranks
        top, pos = 0.0, 0
        for i, k in enumerate(b):
            x = prefix[pos + k] - prefix[pos]
            pos += k
            per_rank[i % ranks] += x
            top = max(top, x)
        return max(per_rank), top

    def descend(b: List[int], window: int = 0) -> Tuple[Tuple[float, float], List[int]]:
        """Coordinate descent: each boundary over its whole feasible range
        (``window`` 0) or within +-window units of where it is."""
        best = score(b)
        improved = True
        while improved:
            improved = False
            for g in range(groups - 1):
                pair = b[g] + b[g + 1]
                lo, hi = (1, pair) if not window else (max(1, b[g] - window), min(pair, b[g] + window + 1))
                for left in range(lo, hi):
                    if left == b[g]:
                        continue
                    t = list(b)
                    t[g], t[g + 1] = left, pair - left
                    sc = score(t)
                    if sc < best:
                        b, best, improved = t, sc, True
        return best, b

    # Deterministic restarts (every rank must derive the same plan): random
    # kicks of the best split, each followed by coordinate descent.
    import random

    rnd = random.Random(0)
    best, bal = descend(bal)
    # restarts: plenty for the enc12 plans (<= 24 groups), fewer for GPT-2-XL's
    # deep loops, whose 195 units make every descent long
    for _ in range(200 if groups <= 24 else 60):
        t = list(bal)
        for _ in range(3):
            g = rnd.randrange(groups - 1)
            d = rnd.choice((-2, -1, 1, 2))
            if t[g] + d >= 1 and t[g + 1] - d >= 1:
                t[g] += d
                t[g + 1] -= d
        sc, t = descend(t, window=4)  # a kick moves boundaries by <= 2: refine locally
        if sc < best:
            best, bal = sc, t
    return bal


def simulate_step(stage_costs: Sequence[float], ranks: int, virtual: int, chunks: int,
                  bwd_ratio: float = 2.0, deferred_w: float = 0.0,
                  checkpoint_stop: Optional[int] = None, transfer: float = 0.0,
                  launch: float = 0.0) -> Tuple[float, List[float]]:
    """Event simulation of one synchronous step (breadth-first looping order,
    as :class:`~mipipe.parallel.engine.PipelineEngine` runs it; transfers free).

    ``stage_costs`` are per VIRTUAL stage forward+backward costs; backward is
    ``bwd_ratio`` x forward, of which the fraction ``deferred_w`` (weight
    gradients under ``defer_wgrad``) runs after the rank's last backward.
    Returns the makespan and per-rank busy time (bubble = 1 - mean busy /
    makespan).

    With ``checkpoint_stop`` given, recompute is modelled explicitly instead
    of being folded into ``bwd_ratio``: micro-batches ``i < checkpoint_stop``
    run a recompute (one forward) right before their backward, and -- as the
    engine issues it before its gradient wait -- the recompute does not wait
    for the downstream gradient.  ``stage_costs`` then price forward +
    ``bwd_ratio`` x forward WITHOUT recompute.

    ``transfer``: latency of a stage-boundary message (activation or gradient)
    between ranks, in the units of ``stage_costs``: a dependency on another
    rank's output is ready that much after it was produced (the sender does
    not wait).  ``launch``: fixed cost of every F / B / R action (kernel-launch
    gaps of a chunk).  Both are what more virtual chunks per rank pay for their
    shorter fill and drain."""
    nv = ranks * virtual
    fwd = [c / (1.0 + bwd_ratio) for c in stage_costs]
    bwd_all = [c * bwd_ratio / (1.0 + bwd_ratio) for c in stage_costs]
    bwd = [b * (1.0 - deferred_w) for b in bwd_all]
    wgt = [b * deferred_w for b in bwd_all]
    f_done = [[None] * chunks for _ in range(nv)]
    b_done = [[None] * chunks for _ in range(nv)]
    stop = checkpoint_stop or 0

    def _bwd(s: int, i: int) -> List[Tuple[str, int, int]]:
        return ([("R", s, i)] if i < stop else []) + [("B", s, i)]

    order = {r: [("F", c * ranks + r, i) for c in range(virtual) for i in range(chunks)]
             + [a for c in reversed(range(virtual)) for i in reversed(range(chunks)) for a in _bwd(c * ranks + r, i)]
             for r in range(ranks)}
    pos = [0] * ranks
    clock = [0.0] * ranks
    busy = [0.0] * ranks
    remaining = sum(len(o) for o in order.values())
    # deferred weight gradients: after the rank's last backward, no dependencies
    for r in range(ranks):
        order[r] += [("W", c * ranks + r, i) for c in range(virtual) for i in range(chunks)] if deferred_w else []
    remaining = sum(len(o) for o in order.values())
    while remaining:
        progressed = False
        for r in range(ranks):
            while pos[r] < len(order[r]):
                kind, s, i = order[r][pos[r]]
                hop = transfer if ranks > 1 else 0.0
                if kind == "F":
                    dep = 0.0 if s == 0 else f_done[s - 1][i]
                    if dep is not None and s > 0:
                        dep += hop
                    dur = fwd[s] + launch
                elif kind == "W":
                    dep, dur = 0.0, wgt[s]
                elif kind == "R":
                    dep, dur = 0.0, fwd[s] + launch
                else:
                    dep = f_done[s][i] if s == nv - 1 else b_done[s + 1][i]
                    if dep is not None and s < nv - 1:
                        dep += hop
                    dur = bwd[s] + launch
                if dep is None:
                    break
                start = max(clock[r], dep)
                clock[r] = start + dur
                busy[r] += dur
                if kind in ("F", "B"):
                    (f_done if kind == "F" else b_done)[s][i] = clock[r]
                pos[r] += 1
                remaining -= 1
                progressed = True
        if not progressed:
            raise RuntimeError("schedule deadlock in simulation")
    return max(clock), busy


# Fraction of the backward that is weight-gradient GEMMs (deferred by the
# engine's ``defer_wgrad``): wgrad FLOPs equal dgrad FLOPs for every linear.
DEFERRED_W = 0.5


def _makespan_refined(costs: List[float], ranks: int, virtual: int, chunks: int, start: List[int],
                      bwd_ratio: float = 2.0, window: int = 3) -> List[int]:
    """Coordinate descent on the simulated step time (:func:`simulate_step`)."""
    groups = ranks * virtual

    def score(b: List[int]) -> float:
        gc, pos = [], 0
        for k in b:
            gc.append(sum(costs[pos:pos + k]))
            pos += k
        return simulate_step(gc, ranks, virtual, chunks, bwd_ratio, deferred_w=1.0 / bwd_ratio)[0]

    bal, best = list(start), score(start)
    improved = True
    while improved:
        improved = False
        for g in range(groups - 1):
            pair = bal[g] + bal[g + 1]
            # local moves: the start is already balanced, and the simulation
            # dominates planning time (GPT-2-XL has 195 units)
            for left in range(max(1, bal[g] - window), min(pair, bal[g] + window + 1)):
                if left == bal[g]:
                    continue
                t = list(bal)
                t[g], t[g + 1] = left, pair - left
                sc = score(t)
                if sc < best * (1 - 1e-9):
                    bal, best, improved = t, sc, True
    return bal


def plan_stages(cfg: LMConfig, stages: int, virtual: int = 1, chunks: int = 0, split_decoder: bool = False,
                bwd_ratio: float = 2.0, costs: Optional[List[float]] = None,
                objective: str = "makespan", seeds: Sequence[Sequence[int]] = ()) -> StagePlan:
    """Plan for ``stages`` ranks with ``virtual`` chunks each (looping placement).

    With ``virtual > 1`` the split starts from the rank-total-balanced one and
    is refined against the simulated step time for ``chunks`` micro-batches
    (default 4 x stages): a chunk far larger than its neighbours stalls the
    micro-batch flow even when rank totals are even.  ``costs``: per-unit
    costs to plan with instead of the analytic :func:`block_costs` (e.g.
    measured ones, :mod:`mipipe.parallel.calibrate`).

    ``objective="balance"``: the split with the most even RANK totals
    (``balance_by_time``'s goal), without the makespan refinement -- which
    may load ranks unevenly when that shortens the simulated fill / drain
    (profiles/pp_planning_r4.txt compares the two).

    ``seeds``: further starting splits for the makespan refinement (e.g. the
    analytic-cost plan when planning with measured costs: coordinate descent
    from the cost-balanced starts can stall in a worse local optimum,
    profiles/plan_table_r5.txt); invalid ones are ignored."""
    if costs is None:
        costs = block_costs(cfg, split_decoder)
    elif len(costs) != len(block_costs(cfg, split_decoder)):
        raise ValueError(f"{len(costs)} unit costs for {len(block_costs(cfg, split_decoder))} pipeline units")
    if stages * virtual > len(costs):
        raise ValueError(f"{stages} x {virtual} virtual stages exceed the {len(costs)} pipeline units")
    if objective not in ("makespan", "balance"):
        raise ValueError(f"objective must be 'makespan' or 'balance', got {objective!r}")
    groups = stages * virtual
    seeds = [list(b) for b in seeds
             if len(b) == groups and sum(b) == len(costs) and all(k >= 1 for k in b)]
    m = chunks or 4 * stages
    if virtual == 1:
        plan = StagePlan(balance_cost(costs, stages), costs, 1, split_decoder)
        if objective == "makespan" and seeds:
            def sim1(p: StagePlan) -> float:
                return simulate_step([p.stage_cost(g) for g in range(stages)], stages, 1, m, bwd_ratio,
                                     deferred_w=1.0 / bwd_ratio)[0]
            for b in seeds:
                cand = StagePlan(b, costs, 1, split_decoder)
                if sim1(cand) < sim1(plan):
                    plan = cand
        return plan
    if objective == "balance":
        return StagePlan(_rank_balanced(costs, stages, virtual), costs, virtual, split_decoder)
    best = None
    for start in [balance_cost(costs, stages * virtual), _rank_balanced(costs, stages, virtual)] + seeds:
        bal = _makespan_refined(costs, stages, virtual, m, start, bwd_ratio)
        plan = StagePlan(bal, costs, virtual, split_decoder)
        t = simulate_step([plan.stage_cost(g) for g in range(stages * virtual)], stages, virtual, m, bwd_ratio,
                          deferred_w=1.0 / bwd_ratio)[0]
        if best is None or t < best[0]:
            best = (t, plan)
    return _unload_busiest(best[1], costs, m, bwd_ratio, best[0])


def _unload_busiest(plan: StagePlan, costs: List[float], chunks: int, bwd_ratio: float, t0: float,
                    slack: float = 0.002) -> StagePlan:
    """Moves single units off the busiest rank while the simulated step stays
    within ``slack`` of ``t0``.  The simulation's fill/drain detail is finer
    than the cost model is accurate, and what the emulated ranks measure is the
    busiest rank's work (profiles/pp8_ranks_mb64.txt: the PP=8 vocabulary-tail
    rank ran 321 ms against 305-310 for the others).  Each accepted move
    lowers the busiest rank's cost, so the search ends."""
    ranks, virtual = plan.ranks, plan.virtual
    groups = ranks * virtual
    bal = list(plan.balance)

    def evaluate(b: List[int]) -> Tuple[float, float]:
        p = StagePlan(b, costs, virtual, plan.split_decoder)
        t = simulate_step([p.stage_cost(g) for g in range(groups)], ranks, virtual, chunks, bwd_ratio,
                          deferred_w=1.0 / bwd_ratio)[0]
        return t, max(p.rank_cost(r) for r in range(ranks))

    _, peak = evaluate(bal)
    improved = True
    while improved:
        improved = False
        for g in range(groups - 1):
            for d in (-1, 1):
                t_ = list(bal)
                t_[g] += d
                t_[g + 1] -= d
                if t_[g] < 1 or t_[g + 1] < 1:
                    continue
                t, pk = evaluate(t_)
                if pk < peak and t <= t0 * (1 + slack):
                    bal, peak, improved = t_, pk, True
    return StagePlan(bal, costs, virtual, plan.split_decoder)


UNITS_PER_LAYER = 4  # attention core, attention output, mlp in, mlp out


def unit_kind(cfg: LMConfig, index: int, split_decoder: bool = False) -> str:
    """``enc`` / ``core`` / ``out`` / ``mlp_in`` / ``mlp_out`` / ``norm`` / ``dec``
    (``dec_head`` / ``dec_tail`` when the decoder is split)."""
    if index == 0:
        return "enc"
    body = UNITS_PER_LAYER * cfg.num_layers
    if index <= body:
        return ("core", "out", "mlp_in", "mlp_out")[(index - 1) % UNITS_PER_LAYER]
    rest = index - body - 1 - (1 if cfg.norm_first else 0)
    if rest < 0:
        return "norm"
    if split_decoder:
        return "dec_head" if rest == 0 else "dec_tail"
    return "dec"


def unit_is_packed_core(cfg: LMConfig, index: int) -> bool:
    """True if pipeline unit ``index`` is an attention core (packed output)."""
    return unit_kind(cfg, index) == "core"


def stage_input_shape(cfg: LMConfig, plan: StagePlan, vstage: int, micro_batch: int) -> Tuple[int, ...]:
    """Shape of the activation virtual stage ``vstage`` receives: ``[2, mb, S, E]``
    after a packed attention core, ``[mb, S, E + F]`` after a packed MLP input
    half, else ``[mb, S, E]``."""
    base = (micro_batch, cfg.seq_len, cfg.d_model)
    if vstage == 0:
        return base
    kind = unit_kind(cfg, plan.slice(vstage).start - 1, plan.split_decoder)
    if kind == "core":
        return (2,) + base
    if kind == "mlp_in":
        return (micro_batch, cfg.seq_len, cfg.d_model + cfg.dim_feedforward)
    if kind == "dec_head":
        return (micro_batch, cfg.seq_len, cfg.d_model + STAT_SLOTS)
    return base


def build_stage(cfg: LMConfig, plan: StagePlan, vstage: int, *, device, dtype,
                skips: Sequence[Tuple[int, int]] = ()) -> TargetSequential:
    """Instantiates ONLY this virtual stage's units (on ``device``, in ``dtype``)
    and merges attention / MLP halves that ended up on the same stage.
    ``skips``: long cross-stage residuals (layer a -> layer b,
    :mod:`mipipe.models.long_skip`) whose ends fall in this stage."""
    with torch.device("meta"):
        proto = lm_pipeline_units(build_lm_blocks(cfg), split_decoder=plan.split_decoder)
    units = []
    for idx in plan.slice(vstage):
        # to_empty() builds new Parameter objects: carry the GEMM-weight tags over
        tagged = {n for n, p in proto[idx].named_parameters() if getattr(p, "_mipipe_gemm_weight", False)}
        u = proto[idx].to_empty(device=device)
        u.reset_parameters()
        for n, p in u.named_parameters():
            if n in tagged:
                mark_gemm_weight(p)
        units.append(u)
    del proto
    if skips:
        from ..models.long_skip import insert_long_skips

        units = insert_long_skips(units, skips, start=plan.slice(vstage).start)
    stage = TargetSequential(*merge_units(units))
    for p in stage.parameters():
        if p.dtype.is_floating_point:
            p.data = p.data.to(dtype)
    return stage


# Prices of the boundary terms of simulate_step, in the planner's unit
# (training FLOPs per token): a PP boundary carries d_model bf16 values per
# token over one xGMI link (~64 GB/s one direction for a single peer stream),
# against ~1.2 PF/s of achieved GEMM rate; every chunk action costs ~30 us of
# launch gaps, spread over the micro-batch's tokens.
LINK_BYTES_PER_S = 64e9
ACHIEVED_FLOP_PER_S = 1.2e15
LAUNCH_GAP_S = 30e-6


def boundary_terms(cfg: LMConfig, micro_batch: Optional[int], unit: str = "flop") -> Tuple[float, float]:
    """(transfer, launch) for :func:`simulate_step`: in per-token FLOP-equivalents
    (``unit="flop"``, the analytic costs) or in ms per micro-batch (``"ms"``,
    measured costs)."""
    tokens = (micro_batch or 8) * cfg.seq_len
    if unit == "ms":
        return 2.0 * cfg.d_model * tokens / LINK_BYTES_PER_S * 1e3, LAUNCH_GAP_S * 1e3
    transfer = 2.0 * cfg.d_model / LINK_BYTES_PER_S * ACHIEVED_FLOP_PER_S
    return transfer, LAUNCH_GAP_S * ACHIEVED_FLOP_PER_S / tokens


def choose_virtual(cfg: LMConfig, stages: int, chunks: int, candidates: Optional[Sequence[int]] = None,
                   split_options: Sequence[bool] = (False, True), bwd_ratio: float = 2.0,
                   micro_batch: Optional[int] = None, max_virtual: int = 8,
                   cost_fn=None, objective: str = "makespan") -> Tuple[int, StagePlan]:
    """Chunks per rank (and whether to split the decoder) with the shortest
    simulated step; ties (within 0.5 %) keep the simpler plan.  ``bwd_ratio``
    is backward / forward cost (2, or 3 when every micro-batch is recomputed).

    ``candidates`` default: every v from 1 to ``max_virtual`` that leaves each
    virtual stage at least one pipeline unit.  The simulation charges each
    stage-boundary message and each chunk action (:func:`boundary_terms`), so a
    deeper looping placement is chosen only when its shorter fill/drain pays
    for its extra boundaries.  ``cost_fn(split_decoder)``: per-unit costs in ms
    per micro-batch (measured, :mod:`mipipe.parallel.calibrate`) instead of
    the analytic FLOP model.  ``objective``: see :func:`plan_stages` (the
    chunk count is chosen by simulated step time either way)."""
    transfer, launch = boundary_terms(cfg, micro_batch, "ms" if cost_fn is not None else "flop")

    def sim(plan: StagePlan, v: int) -> float:
        return simulate_step([plan.stage_cost(g) for g in range(stages * v)], stages, v, chunks, bwd_ratio,
                             deferred_w=1.0 / bwd_ratio, transfer=transfer, launch=launch)[0]

    # screen every (split, v) on its rank-balanced split (cheap), then run the
    # simulation-refined planner on the few best (the refinement is the
    # expensive part: coordinate descent over the boundaries)
    screened = []
    for split in split_options:
        if split and stages == 1:
            continue
        costs = cost_fn(split) if cost_fn is not None else block_costs(cfg, split)
        units = len(costs)
        cands = candidates if candidates is not None else range(1, max(1, min(max_virtual, units // stages)) + 1)
        for v in cands:
            if stages * v > units or (v > 1 and stages == 1):
                continue
            quick = StagePlan(balance_cost(costs, stages * v), costs, v, split)
            screened.append((sim(quick, v), v, split))
    screened.sort()
    best = None
    for _, v, split in screened[:6]:
        seeds = ()
        if cost_fn is not None and objective == "makespan":
            # the analytic plan as a further start: with measured costs the refinement alone can stall
            # in a worse split (profiles/plan_table_r5.txt: config #3's analytic v=2 plan simulates 6 %
            # faster under the MEASURED costs than the split refined from them)
            seeds = (plan_stages(cfg, stages, v, chunks, split, bwd_ratio, objective="makespan").balance,)
        plan = plan_stages(cfg, stages, v, chunks, split, bwd_ratio,
                           costs=cost_fn(split) if cost_fn is not None else None, objective=objective,
                           seeds=seeds)
        t = sim(plan, v)
        # ties (within 0.5 %) keep the simpler plan: fewer chunks, no split
        key = (v, split)
        if best is None or t < best[0] * 0.995 or (t <= best[0] * 1.005 and key < best[3]):
            best = (t, v, plan, key)
    return best[1], best[2]


# Stage-transport hop used to rank plans from measured rank walls: the IPC link's cross-stream event latency plus the
# message at an assumed 100 GB/s of xGMI copy bandwidth (profiles/pp8_transport_prediction_r5.txt).
HOP_LATENCY_MS = 0.15
HOP_BYTES_PER_S = 100e9


def simulate_from_walls(plan: StagePlan, walls: Sequence[float], costs: Sequence[float], chunks: int,
                        checkpoint_stop: int, hop_ms: float) -> Tuple[float, float]:
    """(step ms, mean bubble) of ``plan`` from MEASURED per-rank step walls
    (e.g. each rank emulated over loop-back channels): each rank's wall is split
    over its virtual stages in proportion to their unit ``costs``, per
    micro-batch, recompute stripped (the simulation adds it back explicitly),
    weight gradients deferred; ``hop_ms`` per stage-boundary message.  Unlike
    the unit-cost model this carries every cost a rank really pays for its cut
    positions and chunk count (profiles/plan_table_r5.txt)."""
    pp, v = plan.ranks, plan.virtual
    rec = checkpoint_stop / chunks
    per = []
    for g in range(pp * v):
        r = g % pp
        mine = sum(costs[i] for i in plan.slice(g))
        total = sum(sum(costs[i] for i in plan.slice(s)) for s in plan.vstages(r)) or 1.0
        per.append(walls[r] * mine / total / chunks / (3.0 + rec) * 3.0)
    t, busy = simulate_step(per, pp, v, chunks, 2.0, deferred_w=1.0 / 3.0, checkpoint_stop=checkpoint_stop,
                            transfer=hop_ms)
    return t, 1.0 - sum(busy) / len(busy) / t


def candidate_plans(cfg: LMConfig, stages: int, chunks: int, bwd_ratio: float, micro_batch: Optional[int],
                    cost_fn, split_options: Sequence[bool] = (False, True), max_candidates: int = 6,
                    within: float = 0.06, max_virtual: int = 6) -> List[StagePlan]:
    """The plans worth measuring: for every v up to ``max_virtual`` the makespan
    plan from the measured costs (``cost_fn``) and from the analytic ones, kept
    when the measured-cost simulation puts them within ``within`` of the best,
    best first, at most ``max_candidates``.  The unit-cost model ranks plans only
    to ~2-3 % (the cut positions and chunk count cost what it does not see), so
    the final pick among these is made from emulated rank walls
    (:func:`mipipe.parallel.calibrate.select_plan_by_emulation`)."""
    transfer, launch = boundary_terms(cfg, micro_batch, "ms" if cost_fn is not None else "flop")
    units = len(block_costs(cfg, False))
    seen, scored = set(), []
    for v in range(1, max(1, min(max_virtual, units // stages)) + 1):
        for fn in ((cost_fn, None) if cost_fn is not None else (None,)):
            try:
                vv, plan = choose_virtual(cfg, stages, chunks, candidates=[v], split_options=split_options,
                                          bwd_ratio=bwd_ratio, micro_batch=micro_batch, cost_fn=fn)
            except (TypeError, ValueError):
                continue
            key = (vv, plan.split_decoder, tuple(plan.balance))
            if key in seen:
                continue
            seen.add(key)
            # score every candidate under the same (measured, when given) costs
            costs = cost_fn(plan.split_decoder) if cost_fn is not None else block_costs(cfg, plan.split_decoder)
            p = StagePlan(list(plan.balance), costs, vv, plan.split_decoder)
            t = simulate_step([p.stage_cost(g) for g in range(stages * vv)], stages, vv, chunks, bwd_ratio,
                              deferred_w=1.0 / bwd_ratio, transfer=transfer, launch=launch)[0]
            scored.append((t, len(scored), p))
    scored.sort(key=lambda x: (x[0], x[1]))
    best = scored[0][0]
    return [p for t, _, p in scored if t <= best * (1.0 + within)][:max_candidates]
