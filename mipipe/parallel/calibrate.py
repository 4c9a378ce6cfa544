"""Measured unit costs for the stage planner (``balance_by_time`` for the engine).

The reference points its users at profile-driven balancing: time every layer of
the model on a sample batch and split by the measured times
(``/root/reference/pipe.py:42-58``, ``torchgpipe.balance.balance_by_time``).
The engine's planner (:mod:`mipipe.parallel.stage`) prices pipeline units with
an analytic FLOP model; this module replaces that model with GPU times, in two
layers:

* :func:`measure_unit_times` -- every DISTINCT unit kind (embedding, attention
  core, attention output, MLP halves, final norm, decoder or its two
  vocabulary halves) built once, alone, with the flat optimizer's
  ``main_grad`` buffers, and run for a few micro-batches: forwards timed
  alone, then forward + backward inside ``deferred_wgrad``.  Cheap, but a unit
  run by itself is priced with the host overhead and launch gaps the engine
  hides behind longer kernels: on the PP=8 rank emulations these costs put the
  ranks' measured step times 36-38 % apart (profiles/pp_planning_r4.txt);
* :func:`measure_engine_costs` -- what the planner uses: the real
  :class:`~mipipe.parallel.engine.PipelineEngine` (one process, loop-back
  channels, as ``tools/pp_rank_emulation.py`` runs a rank) on synthetic
  stages -- two whole layers in the middle of the pipeline, the embedding +
  one layer at its head, one layer + final norm + decoder (or its vocabulary
  halves) at its tail -- with the configured micro-batch count, checkpoint
  mode and optimizer step.  Differences of the stage times give a layer, the
  embedding and the decoder end in engine context; the layer is split into
  its four units in the proportions the per-unit times give.

Costs are ms per micro-batch.  With a process group up every rank measures and
the costs are averaged (``all_reduce``), so all ranks derive one plan.  Results
are cached as JSON under ``$MIPIPE_CALIB_DIR`` (default
``~/.cache/mipipe/calibration``), keyed by model, micro-batch, chunks,
checkpoint mode, dtype and device name, and valid for the native sources they
were measured with.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..models.lm import LMConfig

__all__ = ["unit_kinds", "measure_unit_times", "unit_costs", "measure_engine_costs", "engine_unit_costs",
           "calibrated_costs", "cache_key", "CalibrationError"]


def unit_kinds(cfg: LMConfig, split_decoder: bool = False) -> List[str]:
    """Kind of every pipeline unit, in order (``mipipe.parallel.stage.unit_kind``)."""
    from .stage import block_costs, unit_kind

    return [unit_kind(cfg, i, split_decoder) for i in range(len(block_costs(cfg, split_decoder)))]


def _device_name(device: torch.device) -> str:
    if device.type == "cuda":
        return torch.cuda.get_device_name(device).replace(" ", "_").replace("/", "_")
    return "cpu"


def _digest() -> str:
    try:
        from .._native_loader import source_digest

        return source_digest()[:12]
    except Exception:  # noqa: BLE001 -- no sources next to the package
        return "na"


def cache_key(cfg: LMConfig, micro_batch: int, dtype: torch.dtype, device: torch.device, chunks: int,
              checkpoint: str = "never") -> str:
    dt = str(dtype).replace("torch.", "")
    return f"{cfg.name}-mb{micro_batch}-m{chunks}-{checkpoint}-{dt}-{_device_name(device)}"


def _single_unit_plan(cfg: LMConfig, split_decoder: bool):
    from .stage import StagePlan, block_costs

    n = len(block_costs(cfg, split_decoder))
    return StagePlan([1] * n, [0.0] * n, 1, split_decoder)


def _timer(device: torch.device):
    if device.type == "cuda":
        def start():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e

        def stop(e0) -> float:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            e1.synchronize()
            return e0.elapsed_time(e1)
    else:
        def start():
            return time.perf_counter()

        def stop(t0) -> float:
            return (time.perf_counter() - t0) * 1e3
    return start, stop


def measure_unit_times(cfg: LMConfig, micro_batch: int, *, chunks: int = 4, device: torch.device,
                       dtype: torch.dtype = torch.bfloat16, kinds: Optional[Sequence[str]] = None,
                       reps: int = 3) -> Dict[str, Tuple[float, float]]:
    """``{kind: (fwd_ms, bwd_ms)}`` per micro-batch for each unit kind of ``cfg``
    (or only ``kinds``), measured on ``device`` as described in the module
    docstring: the median of ``reps`` timed rounds of ``chunks`` micro-batches
    after one warm-up round."""
    from .. import ops
    from ..ops.linear import deferred_wgrad
    from ..optim import FlatAdam
    from .stage import build_stage, stage_input_shape

    device = torch.device(device)
    start, stop = _timer(device)
    want = None if kinds is None else set(kinds)
    out: Dict[str, Tuple[float, float]] = {}
    S, V = cfg.seq_len, cfg.vocab
    for split in (False, True):
        plan = _single_unit_plan(cfg, split)
        kinds_here = unit_kinds(cfg, split)
        for idx, kind in enumerate(kinds_here):
            if kind in out or (want is not None and kind not in want):
                continue
            if kind in ("dec_head", "dec_tail") and not split:
                continue
            torch.manual_seed(idx)
            unit = build_stage(cfg, plan, idx, device=device, dtype=dtype).train()
            opt = FlatAdam(list(unit.parameters()), lr=0.0)  # main_grad buffers, as the engine's ranks have
            shape = stage_input_shape(cfg, plan, idx, micro_batch)
            last = idx == len(kinds_here) - 1
            gen = torch.Generator(device="cpu").manual_seed(idx)
            tgt = torch.randint(0, V, (micro_batch, S), generator=gen).to(device)
            if idx == 0:
                xs = [torch.randint(0, V, (micro_batch, S), generator=gen).to(device) for _ in range(chunks)]
            else:
                xs = [(torch.randn(shape, generator=gen) * 0.5).to(device=device, dtype=dtype).requires_grad_()
                      for _ in range(chunks)]

            def fwd(x):
                y = unit(x, tgt) if unit.wants_target else unit(x)
                if last and not unit.fused_loss:
                    y = ops.cross_entropy(y.reshape(-1, V), tgt.reshape(-1))
                return y

            def fwd_bwd(x):
                y = fwd(x)
                if y.dim() == 0:
                    y.backward()
                else:
                    y.backward(torch.ones_like(y) * 1e-3)

            def round_(backward: bool) -> float:
                opt.zero_grad()
                t0 = start()
                if backward:
                    with deferred_wgrad():
                        for x in xs:
                            fwd_bwd(x)
                else:
                    with torch.no_grad():
                        for x in xs:
                            fwd(x)
                return stop(t0)

            round_(False)
            round_(True)  # warm-up (allocator, kernel first launches)
            tf = sorted(round_(False) for _ in range(reps))[reps // 2]
            tfb = sorted(round_(True) for _ in range(reps))[reps // 2]
            out[kind] = (tf / chunks, max(tfb - tf, 0.0) / chunks)
            del unit, opt, xs
            if device.type == "cuda":
                torch.cuda.empty_cache()
    return out


def unit_costs(cfg: LMConfig, times: Dict[str, Tuple[float, float]], split_decoder: bool = False,
               recompute: float = 0.0) -> List[float]:
    """Per-unit cost list for the planner, in ms per micro-batch:
    ``fwd x (1 + recompute) + bwd`` (``recompute``: the share of micro-batches
    whose forward runs twice under activation checkpointing)."""
    return [times[k][0] * (1.0 + recompute) + times[k][1] for k in unit_kinds(cfg, split_decoder)]


class _Done:
    def wait(self):
        return True

    def is_completed(self):
        return True


class Loopback:
    """Channels stand-in for one rank run alone: every transfer completes at
    once, no bytes move (receive buffers keep whatever they hold)."""

    host_staged = False

    def __init__(self, rank: int, world: int) -> None:
        self.rank, self.world, self.ranks = rank, world, list(range(world))

    def warmup(self, device) -> None:
        pass

    def send_act(self, t):
        return _Done()

    recv_act = send_grad = recv_grad = send_act


def _range_stage(cfg: LMConfig, a: int, b: int, split_decoder: bool, *, device, dtype):
    """The stage of pipeline units [a, b) and its input shape (per micro-batch: filled in by the caller)."""
    from .stage import StagePlan, block_costs, build_stage

    n = len(block_costs(cfg, split_decoder))
    bal = ([a] if a else []) + [b - a] + ([n - b] if b < n else [])
    plan = StagePlan(bal, [0.0] * n, 1, split_decoder)
    vs = 1 if a else 0
    return build_stage(cfg, plan, vs, device=device, dtype=dtype).train(), plan, vs, n


def _engine_step_ms(cfg: LMConfig, a: int, b: int, split_decoder: bool, micro_batch: int, chunks: int,
                    checkpoint: str, *, device, dtype, steps: int = 3) -> float:
    """Median wall time (ms) of one engine step + optimizer step of the stage
    made of units [a, b), run as the head / middle / tail rank of a pipeline."""
    from .. import ops
    from ..optim import FlatAdam
    from .engine import PipelineEngine
    from .stage import stage_input_shape

    stage, plan, vs, n = _range_stage(cfg, a, b, split_decoder, device=device, dtype=dtype)
    first, last = a == 0, b == n
    rank, world = (0, 1) if first and last else ((0, 2) if first else ((1, 2) if last else (1, 3)))
    S, V = cfg.seq_len, cfg.vocab
    opt = FlatAdam(list(stage.parameters()), lr=1e-6, max_grad_norm=1.0)

    def loss_fn(y, t):
        return ops.cross_entropy(y.reshape(-1, V), t.reshape(-1))

    engine = PipelineEngine([stage], chunks=chunks, checkpoint=checkpoint,
                            act_shape=[stage_input_shape(cfg, plan, vs, micro_batch)], act_dtype=dtype,
                            loss_fn=loss_fn if last else None, group=Loopback(rank, world), device=device,
                            skip_routes={})
    g = torch.Generator(device="cpu").manual_seed(a)
    tokens = torch.randint(0, V, (chunks, micro_batch, S + 1), generator=g)
    inputs = [tokens[i, :, :S].to(device) for i in range(chunks)] if first else None
    targets = [tokens[i, :, 1:].contiguous().to(device) for i in range(chunks)]

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    def step():
        opt.zero_grad()
        engine.step(inputs, targets)
        opt.step(opt.grad_sumsq())

    step()
    walls = []
    for _ in range(steps):
        sync()
        t0 = time.perf_counter()
        step()
        sync()
        walls.append((time.perf_counter() - t0) * 1e3)
    del engine, opt, stage
    if device.type == "cuda":
        torch.cuda.empty_cache()
    return sorted(walls)[len(walls) // 2]


LAYER_KINDS = ("core", "out", "mlp_in", "mlp_out")


def measure_engine_costs(cfg: LMConfig, micro_batch: int, chunks: int, checkpoint: str = "never", *,
                         device: torch.device, dtype: torch.dtype = torch.bfloat16,
                         steps: int = 3) -> Dict[str, float]:
    """``{kind: ms per micro-batch}`` in engine context (module docstring):
    checkpoint recompute, the deferred weight-gradient flush, the optimizer
    step and the host's issue overhead included as a pipeline rank pays them."""
    from .stage import UNITS_PER_LAYER, block_costs

    device = torch.device(device)
    if cfg.num_layers < 3:
        raise ValueError("engine-context calibration needs >= 3 layers")
    iso = measure_unit_times(cfg, micro_batch, chunks=min(chunks, 4), device=device, dtype=dtype,
                             kinds=LAYER_KINDS + ("norm", "dec", "dec_head", "dec_tail"))
    rec = {"never": 0.0, "except_last": (chunks - 1) / chunks, "always": 1.0}[checkpoint]
    iso_cost = {k: f * (1.0 + rec) + b for k, (f, b) in iso.items()}
    per = lambda ms: ms / chunks  # noqa: E731  -- per micro-batch
    run = lambda a, b, split=False: per(_engine_step_ms(cfg, a, b, split, micro_batch, chunks, checkpoint,  # noqa: E731
                                                        device=device, dtype=dtype, steps=steps))
    L = UNITS_PER_LAYER
    layer = run(1, 1 + 2 * L) / 2.0
    out = {"enc": max(run(0, 1 + L) - layer, 0.0)}
    tot = sum(iso_cost[k] for k in LAYER_KINDS)
    for k in LAYER_KINDS:
        out[k] = layer * iso_cost[k] / tot
    norm = 1 if cfg.norm_first else 0
    n = len(block_costs(cfg, False))
    end = max(run(n - 1 - norm - L, n) - layer, 0.0)  # norm + decoder
    if norm:
        share = iso_cost["norm"] / (iso_cost["norm"] + iso_cost["dec"])
        out["norm"], out["dec"] = end * share, end * (1 - share)
    else:
        out["dec"] = end
    ns = len(block_costs(cfg, True))
    tail = run(ns - 1, ns, True)
    head = max(run(ns - 2 - norm - L, ns - 1, True) - layer - out.get("norm", 0.0), 0.0)
    out["dec_head"], out["dec_tail"] = head, tail
    return out


def engine_unit_costs(cfg: LMConfig, costs: Dict[str, float], split_decoder: bool = False) -> List[float]:
    """Per-unit cost list for the planner from :func:`measure_engine_costs`."""
    return [costs[k] for k in unit_kinds(cfg, split_decoder)]


class CalibrationError(RuntimeError):
    """Raised on EVERY rank when any rank's calibration failed (callers fall back to analytic costs together)."""


def _load(path: str) -> Optional[dict]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def calibrated_costs(cfg: LMConfig, micro_batch: int, chunks: int, checkpoint: str = "never", *,
                     device: torch.device, dtype: torch.dtype = torch.bfloat16, refresh: bool = False,
                     group=None, measure=None) -> Dict[str, float]:
    """Engine-context unit costs (:func:`measure_engine_costs`, or ``measure()``)
    from the cache or measured -- and then identical on every rank of
    ``group`` (default: the world, when initialised): each rank measures on its
    own GPU and the costs are averaged with one ``all_reduce``; a cached table
    is used only if every rank has one (an all-reduced flag), so plans never
    diverge."""
    device = torch.device(device)
    key = cache_key(cfg, micro_batch, dtype, device, chunks, checkpoint)
    cache_dir = os.environ.get("MIPIPE_CALIB_DIR", os.path.join(os.path.expanduser("~"), ".cache", "mipipe",
                                                                "calibration"))
    found = None
    if not refresh:
        rec = _load(os.path.join(cache_dir, key + ".json"))
        if rec is not None and rec.get("digest") == _digest():
            found = rec
    distributed = dist.is_available() and dist.is_initialized()
    nccl = distributed and dist.get_backend(group) == "nccl"
    if distributed:
        # every rank takes the same branch: measure unless ALL ranks found a table
        flag = torch.tensor([0.0 if found is not None else 1.0], device=device if nccl else "cpu")
        dist.all_reduce(flag, group=group)
        if flag.item() > 0:
            found = None
    kinds = sorted(set(unit_kinds(cfg, False)) | set(unit_kinds(cfg, True)))
    ok, err = 1.0, None
    try:
        if found is not None:
            costs = {k: float(v) for k, v in found["costs"].items()}
        elif measure is not None:
            costs = measure()
        else:
            costs = measure_engine_costs(cfg, micro_batch, chunks, checkpoint, device=device, dtype=dtype)
        costs = {k: float(costs[k]) for k in kinds}
    except Exception as exc:  # noqa: BLE001 -- reported on every rank below, identically
        ok, err, costs = 0.0, repr(exc), {k: 0.0 for k in kinds}  # the text: no traceback keeps tensors alive
    if distributed:
        # ONE collective whatever happened locally: a rank whose measurement
        # failed must not leave the others waiting in a different collective
        vec = torch.tensor([ok] + [costs[k] for k in kinds], dtype=torch.float64, device=device if nccl else "cpu")
        dist.all_reduce(vec, group=group)
        vec = vec.cpu().tolist()
        n = dist.get_world_size(group)
        if vec[0] < n:
            raise CalibrationError(f"calibration failed on {n - int(vec[0])} of {n} ranks"
                                   + (f" (here: {err})" if err is not None else ""))
        costs = {k: v / n for k, v in zip(kinds, vec[1:])}
    elif err is not None:
        raise CalibrationError(f"calibration failed: {err}")
    if found is None and (not distributed or dist.get_rank() == 0):
        try:
            os.makedirs(cache_dir, exist_ok=True)
            with open(os.path.join(cache_dir, key + ".json"), "w") as f:
                json.dump({"key": key, "digest": _digest(), "costs": costs}, f, indent=1, sort_keys=True)
        except OSError:
            pass
    return costs


def emulate_rank_ms(cfg: LMConfig, plan, rank: int, chunks: int, micro_batch: int, checkpoint: str, *,
                    device: torch.device, dtype: torch.dtype = torch.bfloat16, steps: int = 2) -> float:
    """Median wall (ms) of one training step of pipeline rank ``rank`` of
    ``plan`` run alone: its virtual stages through the real PipelineEngine over
    :class:`Loopback` channels, deferred weight gradients, grad-norm and Adam
    included -- the GPU runs exactly that rank's kernels in its schedule."""
    from .. import ops
    from ..optim import FlatAdam
    from .engine import PipelineEngine
    from .stage import build_stage, stage_input_shape

    device = torch.device(device)
    pp = plan.ranks
    vss = plan.vstages(rank)
    stages = [build_stage(cfg, plan, vs, device=device, dtype=dtype).train() for vs in vss]
    opt = FlatAdam([p for s in stages for p in s.parameters()], lr=1e-6, max_grad_norm=1.0)
    last = any(vs == pp * plan.virtual - 1 for vs in vss)
    S, V = cfg.seq_len, cfg.vocab

    def loss_fn(y, t):
        return ops.cross_entropy(y.reshape(-1, V), t.reshape(-1))

    engine = PipelineEngine(stages, chunks=chunks, checkpoint=checkpoint,
                            act_shape=[stage_input_shape(cfg, plan, vs, micro_batch) for vs in vss], act_dtype=dtype,
                            loss_fn=loss_fn if last else None, group=Loopback(rank, pp), device=device,
                            skip_routes={})
    g = torch.Generator(device="cpu").manual_seed(rank)
    tokens = torch.randint(0, V, (chunks, micro_batch, S + 1), generator=g)
    inputs = [tokens[i, :, :S].to(device) for i in range(chunks)] if rank == 0 else None
    targets = [tokens[i, :, 1:].contiguous().to(device) for i in range(chunks)]

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    def step():
        opt.zero_grad()
        engine.step(inputs, targets)
        opt.step(opt.grad_sumsq())

    step()
    walls = []
    for _ in range(steps):
        sync()
        t0 = time.perf_counter()
        step()
        sync()
        walls.append((time.perf_counter() - t0) * 1e3)
    del engine, opt, stages
    if device.type == "cuda":
        torch.cuda.empty_cache()
    return sorted(walls)[len(walls) // 2]


def select_plan_by_emulation(cfg: LMConfig, candidates, prank: int, chunks: int, micro_batch: int,
                             checkpoint: str, unit_ms: Dict[str, float], *, device: torch.device,
                             dtype: torch.dtype = torch.bfloat16, replica: int = 0, group=None,
                             steps: int = 2, emulate=None, refine_rounds: int = 6):
    """Picks the fastest of ``candidates`` (:func:`~mipipe.parallel.stage.candidate_plans`)
    from MEASURED walls: every pipeline rank emulates its own rank of every
    candidate at once (:func:`emulate_rank_ms`, replica 0 only under data
    parallelism), ONE all-reduce gathers the [candidate x rank] wall matrix,
    and each candidate's job step is simulated from its walls
    (:func:`~mipipe.parallel.stage.simulate_from_walls`, IPC hop).  Identical
    on every rank.  Returns ``(plan, report)``; if any rank's emulation fails,
    every rank returns the model's first candidate (report says why).  The
    candidates are then refined from their measured walls, best first
    (:func:`refine_plan_by_walls`; ``refine_rounds`` emulated moves in all,
    0: off) and the fastest refined plan is returned.
    ``emulate(plan, prank) -> ms``: test hook."""
    from ..pipeline import checkpoint_stop_for
    from .stage import HOP_BYTES_PER_S, HOP_LATENCY_MS, simulate_from_walls

    device = torch.device(device)
    k = len(candidates)
    pp = candidates[0].ranks
    emulate = emulate or (lambda plan, r: emulate_rank_ms(cfg, plan, r, chunks, micro_batch, checkpoint,
                                                          device=device, dtype=dtype, steps=steps))
    walls = torch.zeros(k * pp + 1, dtype=torch.float64)
    err = None
    if replica == 0:
        try:
            for i, plan in enumerate(candidates):
                walls[i * pp + prank] = float(emulate(plan, prank))
        except Exception as exc:  # noqa: BLE001 -- reported on every rank below, identically
            # the text only: the exception's traceback holds the emulation's frames (stages, optimizer, engine
            # GPU tensors) alive in a cycle
            err = repr(exc)
            del exc
            import gc

            gc.collect()
            if device.type == "cuda":
                torch.cuda.empty_cache()
            walls[-1] = 1.0
    distributed = dist.is_available() and dist.is_initialized()
    if distributed:
        nccl = dist.get_backend(group) == "nccl"
        w = walls.to(device) if nccl else walls
        dist.all_reduce(w, group=group)  # ONE collective whatever happened locally
        walls = w.cpu()
    report = {"method": "emulated rank walls (loop-back engine), IPC hop", "candidates": []}
    if walls[-1] > 0:
        report["method"] = "model (emulation failed" + (f": {err}" if err is not None else " on another rank") + ")"
        return candidates[0], report
    stop = checkpoint_stop_for(checkpoint, chunks)
    hop = HOP_LATENCY_MS + micro_batch * cfg.seq_len * cfg.d_model * 2 / HOP_BYTES_PER_S * 1e3
    best = None
    for i, plan in enumerate(candidates):
        w = walls[i * pp:(i + 1) * pp].tolist()
        costs = engine_unit_costs(cfg, unit_ms, plan.split_decoder)
        t, bub = simulate_from_walls(plan, w, costs, chunks, stop, hop)
        report["candidates"].append({"v": plan.virtual, "split_decoder": plan.split_decoder,
                                     "balance": list(plan.balance), "rank_walls_ms": [round(x, 1) for x in w],
                                     "step_ms": round(t, 1), "bubble": round(bub, 3)})
        if best is None or t < best[0]:
            best = (t, i)
    report["chosen"] = best[1]
    plan = candidates[best[1]]
    report["chosen_balance"] = list(plan.balance)
    if refine_rounds > 0:
        # every candidate, best simulated first, within a shared budget of emulation rounds: a plan the cost
        # model got wrong can beat the pick once its slowest rank is unloaded (PP=8: +2.5 %,
        # profiles/plan_refine_r6.txt)
        def step_of(p, w):
            return simulate_from_walls(p, w, engine_unit_costs(cfg, unit_ms, p.split_decoder), chunks, stop, hop)[0]

        order = sorted(range(k), key=lambda i: (report["candidates"][i]["step_ms"], i))
        budget, refined = refine_rounds, []
        pick = (best, plan)
        try:
            plan = _refine_all(order, budget, refined, candidates, walls, report, pp, prank, emulate, replica,
                               group, device, step_of, best, plan)
        except Exception as exc:  # noqa: BLE001 -- deterministic code on identical walls: every rank is here
            refined.append({"error": repr(exc)})
            best, plan = pick
            report["chosen"] = best[1]
        report["refinement"] = refined
        report["chosen_balance"] = list(plan.balance)
    return plan, report


def _refine_all(order, budget, refined, candidates, walls, report, pp, prank, emulate, replica, group, device,
                step_of, best, plan):
    """The refinement loop of :func:`select_plan_by_emulation`: candidates best first, one shared budget of
    emulated moves; returns the fastest refined plan (``report["chosen"]``: its candidate index)."""
    for i in order:
        if budget <= 0:
            break
        p_i, hist = refine_plan_by_walls(candidates[i], walls[i * pp:(i + 1) * pp].tolist(),
                                         report["candidates"][i]["step_ms"], prank=prank, emulate=emulate,
                                         replica=replica, group=group, device=device, rounds=min(3, budget),
                                         step_of=step_of)
        budget -= sum(1 for h in hist if "move" in h)
        t_i = min([report["candidates"][i]["step_ms"]] + [h["step_ms"] for h in hist if h.get("accepted")])
        refined.append({"candidate": i, "balance": list(p_i.balance), "step_ms": t_i, "moves": hist})
        if t_i < best[0]:
            best, plan = (t_i, i), p_i
        if any("stopped" in h for h in hist):
            break
    report["chosen"] = best[1]
    return plan


def _move_candidates(plan, walls: Sequence[float]):
    """Single-unit boundary moves off the slowest measured rank, best first: each virtual stage of that rank
    (keeping >= 1 unit) gives its boundary unit to an adjacent virtual stage owned by another rank.  The unit's
    share of the slow rank's wall is priced by its unit cost (``plan.costs``) and only moves predicted to lower
    the larger of the two walls are kept, the lowest predicted maximum first (ties: lower virtual stage)."""
    pp, n = plan.ranks, len(plan.balance)
    slow = max(range(pp), key=lambda r: (walls[r], -r))
    mine = sum(plan.costs[i] for s in plan.vstages(slow) for i in plan.slice(s)) or 1.0
    moves = []
    for s in plan.vstages(slow):
        if plan.balance[s] <= 1:
            continue
        sl = plan.slice(s)
        for nb in (s - 1, s + 1):
            if not (0 <= nb < n) or nb % pp == slow:
                continue
            unit = sl.start if nb < s else sl.stop - 1
            c = walls[slow] * plan.costs[unit] / mine
            peak = max(walls[nb % pp] + c, walls[slow] - c)
            if peak < walls[slow]:
                moves.append((peak, s, nb))
    moves.sort()
    return slow, [(s, nb) for _, s, nb in moves]


def refine_plan_by_walls(plan, walls: Sequence[float], step_ms: float, *, prank: int, emulate,
                         replica: int = 0, group=None, device=None, rounds: int = 4, step_of=None):
    """Moves single units off the slowest MEASURED rank of the chosen plan.

    The unit-cost model balances what it prices; the emulated walls also carry what it does not (the loss and
    decoder's optimizer share on the last rank, the embedding gradient on the first, the recompute of
    ``except_last``): at PP=8, micro-batch 128 the chosen plan's walls spread 476-584 ms
    (profiles/plan_table_r5.txt).  Each round takes the best move of :func:`_move_candidates`, re-emulates ONLY
    the two ranks whose virtual stages changed (a rank's wall depends on its own stages alone), gathers the walls
    with one all-reduce, and keeps the move if the simulated job step (``step_of(plan, walls)``) is shorter;
    the first move that does not help ends the search.  Identical decisions on every rank (same walls); a rank
    whose emulation raises ends the search for all.  Returns ``(plan, history)``."""
    from .stage import StagePlan

    pp = plan.ranks
    walls = list(walls)
    history = []
    distributed = dist.is_available() and dist.is_initialized()
    for _ in range(rounds):
        slow, moves = _move_candidates(plan, walls)
        if not moves:
            break
        s, nb = moves[0]
        bal = list(plan.balance)
        bal[s] -= 1
        bal[nb] += 1
        new = StagePlan(bal, plan.costs, plan.virtual, plan.split_decoder)
        changed = {s % pp, nb % pp}
        buf = torch.zeros(pp + 1, dtype=torch.float64)
        if replica == 0 and prank in changed:
            try:
                buf[prank] = float(emulate(new, prank))
            except Exception as exc:  # noqa: BLE001 -- every rank stops below, identically
                history.append({"error": repr(exc)})
                del exc
                buf[-1] = 1.0
        if distributed:
            w = buf.to(device) if dist.get_backend(group) == "nccl" else buf
            dist.all_reduce(w, group=group)
            buf = w.cpu()
        if buf[-1] > 0:
            history.append({"stopped": "emulation failed"})
            break
        new_walls = [float(buf[r]) if r in changed else walls[r] for r in range(pp)]
        t = step_of(new, new_walls)
        ok = t < step_ms
        history.append({"slowest_rank": slow, "move": [s, nb], "rank_walls_ms": [round(x, 1) for x in new_walls],
                        "step_ms": round(t, 1), "accepted": ok})
        if not ok:
            break
        plan, walls, step_ms = new, new_walls, t
    return plan, history
