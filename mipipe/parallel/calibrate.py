"""Measured unit costs for the stage planner (``balance_by_time`` for the engine).

The reference points its users at profile-driven balancing: time every layer of
the model on a sample batch and split by the measured times
(``/root/reference/pipe.py:42-58``, ``torchgpipe.balance.balance_by_time``).
The engine's planner (:mod:`mipipe.parallel.stage`) prices pipeline units with
an analytic FLOP model; this module replaces that model with GPU times:

* every DISTINCT unit kind of the model (embedding, attention core, attention
  output, MLP halves, final norm, decoder or its two vocabulary halves) is
  built once -- one unit, never the model -- with the flat optimizer's
  ``main_grad`` buffers, and run for ``chunks`` micro-batches of the real
  shape: forwards timed alone, then forward + backward inside
  ``deferred_wgrad`` (the weight gradients as ONE K-segmented GEMM per weight,
  as the engine flushes them), so ``bwd = (fwd+bwd) - fwd`` includes the
  batched weight-gradient cost;
* a unit's cost is ``fwd x (1 + recompute share) + bwd`` in ms per
  micro-batch, the recomputed forward of checkpointed micro-batches included;
* with a process group up, the times are averaged over the ranks
  (``all_reduce``) so every rank derives the same plan from the same numbers;
* results are cached as JSON under ``$MIPIPE_CALIB_DIR`` (default
  ``~/.cache/mipipe/calibration``), keyed by model, micro-batch, dtype, device
  name and the native-source digest, and the tables measured on MI355X for the
  BASELINE configs ship in ``mipipe/parallel/calibration/``.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..models.lm import LMConfig

__all__ = ["unit_kinds", "measure_unit_times", "unit_costs", "calibrated_times", "cache_key"]

SHIPPED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "calibration")


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


def cache_key(cfg: LMConfig, micro_batch: int, dtype: torch.dtype, device: torch.device, chunks: int) -> str:
    dt = str(dtype).replace("torch.", "")
    return f"{cfg.name}-mb{micro_batch}-m{chunks}-{dt}-{_device_name(device)}"


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


def _load(path: str) -> Optional[dict]:
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def calibrated_times(cfg: LMConfig, micro_batch: int, *, device: torch.device, dtype: torch.dtype = torch.bfloat16,
                     chunks: int = 4, refresh: bool = False, use_shipped: bool = True,
                     group=None) -> Dict[str, Tuple[float, float]]:
    """Unit times from the cache (or the shipped table for this device), else
    measured -- and then identical on every rank of ``group`` (default: the
    world, when initialised): each rank measures, the times are averaged with
    one ``all_reduce``; a cache hit on one rank is used only if every rank hit
    the same table (an all-reduced flag), so plans never diverge."""
    device = torch.device(device)
    key = cache_key(cfg, micro_batch, dtype, device, chunks)
    cache_dir = os.environ.get("MIPIPE_CALIB_DIR", os.path.join(os.path.expanduser("~"), ".cache", "mipipe",
                                                                "calibration"))
    found = None
    if not refresh:
        for d in ([cache_dir] + ([SHIPPED] if use_shipped else [])):
            rec = _load(os.path.join(d, key + ".json"))
            if rec is not None and rec.get("digest") in (_digest(), "any"):
                found = rec
                break
    kinds = sorted(set(unit_kinds(cfg, False)) | set(unit_kinds(cfg, True)))
    distributed = dist.is_available() and dist.is_initialized()
    if distributed:
        # every rank must take the same branch: measure unless ALL found a table
        # (tables could still differ between ranks: averaged below like measurements)
        flag = torch.tensor([0.0 if found is not None else 1.0])
        if dist.get_backend(group) == "nccl":
            flag = flag.to(device)
        dist.all_reduce(flag, group=group)
        if flag.item() > 0:
            found = None
    if found is not None:
        times = {k: tuple(v) for k, v in found["times"].items()}
    else:
        times = measure_unit_times(cfg, micro_batch, chunks=chunks, device=device, dtype=dtype, kinds=kinds)
    if distributed:
        vec = torch.tensor([times[k][j] for k in kinds for j in (0, 1)], dtype=torch.float64)
        if dist.get_backend(group) == "nccl":
            vec = vec.to(device)
        dist.all_reduce(vec, group=group)
        vec = (vec / dist.get_world_size(group)).cpu().tolist()
        times = {k: (vec[2 * i], vec[2 * i + 1]) for i, k in enumerate(kinds)}
    if found is None and (not distributed or dist.get_rank() == 0):
        try:
            os.makedirs(cache_dir, exist_ok=True)
            with open(os.path.join(cache_dir, key + ".json"), "w") as f:
                json.dump({"key": key, "digest": _digest(), "chunks": chunks,
                           "times": {k: list(v) for k, v in times.items()}}, f, indent=1, sort_keys=True)
        except OSError:
            pass
    return times
