"""Tracing, memory and pipeline-timeline instrumentation.

* :func:`torch_profiler` -- the reference driver's ``torch.profiler`` setup
  (``/root/reference/main.py:196-202``): schedule(wait=1, warmup=1, active=2),
  TensorBoard trace handler, shapes/memory/stacks.  On ROCm it records HIP
  kernels through roctracer; the per-cell ``chunk{i}-part{j}`` roctx ranges
  emitted by :mod:`mipipe.worker` show up in it and in rocprofv3 traces.
* :func:`memory_report` -- peak allocated/reserved per device (the numbers the
  reference read off its TensorBoard memory view).
* :func:`record_memory_history` / :func:`dump_memory_snapshot` -- the commented
  memory-snapshot path of ``main.py:263-271`` (viewable at pytorch.org/memory_viz);
  the snapshot is written with ``torch.save`` (not pickle by hand).
* :class:`StageTimer` -- per-stage busy time from HIP events, for bubble %.
"""
from __future__ import annotations

import contextlib
import json
from typing import Dict, Iterable, List, Optional

import torch

__all__ = [
    "torch_profiler",
    "memory_report",
    "reset_peak_memory",
    "record_memory_history",
    "dump_memory_snapshot",
    "StageTimer",
    "bubble_fraction",
    "range",
]


def torch_profiler(log_dir: str, *, wait: int = 1, warmup: int = 1, active: int = 2, repeat: int = 1,
                   record_shapes: bool = True, profile_memory: bool = True, with_stack: bool = True):
    """A ``torch.profiler.profile`` context like the reference's (call ``.step()`` per iteration)."""
    return torch.profiler.profile(
        schedule=torch.profiler.schedule(wait=wait, warmup=warmup, active=active, repeat=repeat),
        on_trace_ready=torch.profiler.tensorboard_trace_handler(log_dir),
        record_shapes=record_shapes,
        profile_memory=profile_memory,
        with_stack=with_stack,
    )


def reset_peak_memory(devices: Iterable[torch.device]) -> None:
    for d in devices:
        d = torch.device(d)
        if d.type == "cuda":
            torch.cuda.reset_peak_memory_stats(d)


def memory_report(devices: Iterable[torch.device]) -> Dict[str, Dict[str, float]]:
    """MB allocated / peak allocated / reserved / peak reserved per device."""
    out: Dict[str, Dict[str, float]] = {}
    for d in devices:
        d = torch.device(d)
        if d.type != "cuda":
            continue
        s = torch.cuda.memory_stats(d)
        mb = 1024.0 * 1024.0
        out[str(d)] = {
            "allocated_mb": s.get("allocated_bytes.all.current", 0) / mb,
            "peak_allocated_mb": s.get("allocated_bytes.all.peak", 0) / mb,
            "reserved_mb": s.get("reserved_bytes.all.current", 0) / mb,
            "peak_reserved_mb": s.get("reserved_bytes.all.peak", 0) / mb,
        }
    return out


def record_memory_history(enabled: bool = True, max_entries: int = 100000) -> None:
    torch.cuda.memory._record_memory_history(enabled="all" if enabled else None, max_entries=max_entries)


def dump_memory_snapshot(path: str) -> None:
    torch.save(torch.cuda.memory._snapshot(), path)


@contextlib.contextmanager
def range(label: str):  # noqa: A001 - mirrors roctx naming
    """roctx range (visible in rocprofv3 --marker-trace) when the extension is loaded."""
    from ..worker import label_range

    with label_range(label):
        yield


class StageTimer:
    """Accumulates GPU busy intervals of one device with HIP events."""

    def __init__(self, device: torch.device) -> None:
        self.device = torch.device(device)
        self.pairs: List = []

    @contextlib.contextmanager
    def span(self):
        if self.device.type != "cuda":
            yield
            return
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        try:
            yield
        finally:
            b.record()
            self.pairs.append((a, b))

    def busy_ms(self) -> float:
        if not self.pairs:
            return 0.0
        torch.cuda.synchronize(self.device)
        return sum(a.elapsed_time(b) for a, b in self.pairs)

    def reset(self) -> None:
        self.pairs.clear()


def bubble_fraction(busy_ms: Iterable[float], step_ms: float) -> float:
    """1 - mean(stage busy) / step time."""
    busy = list(busy_ms)
    if not busy or step_ms <= 0:
        return 0.0
    return 1.0 - (sum(busy) / len(busy)) / step_ms
