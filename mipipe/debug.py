"""Stream-race checking ("a debug mode that synchronises after every
cell and compares results").

The reference has no race detection: memory safety across its copy and compute
streams rests on ``record_stream``, the ``Wait`` events and the phony edges
(/root/reference/README.md:203-208, 341-346; /root/reference/pipeline.py:43-48).
A missing wait there -- or here, in :class:`~mipipe.pipe.Pipe`'s copy streams
or the engine's RCCL receives -- lets a kernel read a buffer before its
producer finished, which shows up as a silently wrong (and usually
run-to-run different) result.

:func:`check_pipe` / :func:`check_engine` run one training step twice from the
same parameters, gradients and RNG state:

1. as scheduled -- copies, computation and transfers overlap on their streams;
2. serialised -- ``Pipe``: every copy on its device's compute stream and every
   device synchronised after each clock tick (``MIPIPE_SYNC_DEBUG=1`` does the
   latter alone); engine: the device synchronised after every action
   (``PipelineEngine(sync_debug=True)`` / ``MIPIPE_SYNC_DEBUG=1``),

and compare the outputs / loss and every parameter gradient.  The serialised
run cannot race, so a difference beyond the rounding of atomics (the
embedding backward and a few reductions accumulate in a run-dependent order:
relative differences ~1e-6) points at a missing stream dependency.  The
gradients are left as the serialised run produced them.

    report = check_pipe(pipe, x, loss_fn=lambda y: y.float().pow(2).mean())
    report.raise_if_failed()
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence, Tuple

import torch
from torch import Tensor, nn

__all__ = ["RaceReport", "check_pipe", "check_engine", "serialized_pipe"]


@dataclass
class RaceReport:
    """Largest relative difference per compared tensor (scheduled vs serialised)."""

    max_rel: Dict[str, float] = field(default_factory=dict)
    tol: float = 1e-3

    @property
    def ok(self) -> bool:
        return all(v <= self.tol for v in self.max_rel.values())

    def worst(self) -> Tuple[str, float]:
        if not self.max_rel:
            return ("", 0.0)
        k = max(self.max_rel, key=self.max_rel.get)
        return k, self.max_rel[k]

    def raise_if_failed(self) -> None:
        if not self.ok:
            bad = sorted(((v, k) for k, v in self.max_rel.items() if v > self.tol), reverse=True)[:8]
            raise RuntimeError("stream race suspected: scheduled and serialised runs differ -- " +
                               ", ".join(f"{k}: {v:.3g}" for v, k in bad))


def _named_params(modules: Sequence[nn.Module]) -> List[Tuple[str, nn.Parameter]]:
    out, seen = [], set()
    for mi, m in enumerate(modules):
        for name, p in m.named_parameters():
            if id(p) not in seen:
                seen.add(id(p))
                out.append((f"{mi}.{name}", p))
    return out


def _reset_grads(params: List[Tuple[str, nn.Parameter]]) -> None:
    with torch.no_grad():
        for _, p in params:
            p.grad = None
            mg = getattr(p, "main_grad", None)
            if mg is not None:
                mg.zero_()
                p._mg_fresh = False  # type: ignore[attr-defined]  # accumulate onto the zeros


def _capture(params: List[Tuple[str, nn.Parameter]]) -> Dict[str, Tensor]:
    out = {}
    for name, p in params:
        g = getattr(p, "main_grad", None)
        if g is not None and p.grad is not None:
            g = g + p.grad.float()
        elif g is None:
            g = p.grad
        if g is not None:
            out[name] = g.detach().float().clone()
    return out


def _rel(a: Tensor, b: Tensor) -> float:
    a, b = a.float(), b.float()
    scale = b.abs().max().item()
    diff = (a - b).abs().max().item()
    if diff != diff:  # NaN in one run only
        return float("inf")
    return diff / scale if scale > 0 else diff


class _RNG:
    def __init__(self, devices: Sequence[torch.device]) -> None:
        self.devices = [d for d in devices if d.type == "cuda"]
        self.cpu = torch.get_rng_state()
        self.dev = [torch.cuda.get_rng_state(d) for d in self.devices]

    def restore(self) -> None:
        torch.set_rng_state(self.cpu)
        for d, s in zip(self.devices, self.dev):
            torch.cuda.set_rng_state(s, d)


def _synchronize(devices: Sequence[torch.device]) -> None:
    for d in devices:
        if d.type == "cuda":
            torch.cuda.synchronize(d)


@contextlib.contextmanager
def serialized_pipe(pipe) -> Iterator[None]:
    """Runs ``pipe`` with its copies on the compute streams and a device-wide
    synchronisation after every clock tick (no overlap anywhere)."""
    from .stream import current_stream

    pl = pipe.pipeline
    saved = (pl.copy_streams, pl.sync_debug, pl.dedicated_streams)
    pl.copy_streams = [[current_stream(d)] * len(s) for d, s in zip(pl.devices, pl.copy_streams)]
    pl.dedicated_streams = [None] * len(pl.devices)  # every partition of a GPU on its current stream
    pl.sync_debug = True
    try:
        yield
    finally:
        pl.copy_streams, pl.sync_debug, pl.dedicated_streams = saved


def check_pipe(pipe, *inputs: Any, loss_fn: Optional[Callable[[Tensor], Tensor]] = None,
               tol: float = 1e-3) -> RaceReport:
    """Scheduled vs serialised :class:`~mipipe.pipe.Pipe` forward + backward."""
    devices = list(pipe.devices)
    params = _named_params([pipe])

    def run() -> Tensor:
        out = pipe(*inputs)
        if hasattr(out, "local_value"):
            out = out.local_value()
        loss = loss_fn(out) if loss_fn is not None else out.float().pow(2).mean()
        loss.backward()
        _synchronize(devices)
        return out.detach().float().clone()

    rng = _RNG(devices)
    _reset_grads(params)
    out1 = run()
    g1 = _capture(params)
    rng.restore()
    _reset_grads(params)
    with serialized_pipe(pipe):
        out2 = run()
    g2 = _capture(params)
    report = RaceReport(tol=tol)
    report.max_rel["output"] = _rel(out1, out2)
    for k in g2:
        report.max_rel[f"grad {k}"] = _rel(g1[k], g2[k]) if k in g1 else float("inf")
    return report


def check_engine(engine, inputs: Optional[Sequence[Tensor]] = None, targets: Optional[Sequence[Tensor]] = None,
                 tol: float = 1e-3) -> RaceReport:
    """Scheduled vs serialised :class:`~mipipe.parallel.PipelineEngine` step on
    this rank (every rank of the pipeline must call it: both runs are full
    pipeline steps).  Compares the loss (last stage) and this rank's gradients."""
    devices = [engine.device]
    params = _named_params(engine.modules)
    rng = _RNG(devices)
    _reset_grads(params)
    st1 = engine.step(inputs, targets)
    _synchronize(devices)
    g1 = _capture(params)
    rng.restore()
    _reset_grads(params)
    saved = engine.sync_debug
    engine.sync_debug = True
    try:
        st2 = engine.step(inputs, targets)
    finally:
        engine.sync_debug = saved
    _synchronize(devices)
    g2 = _capture(params)
    report = RaceReport(tol=tol)
    if st1.loss is not None and st2.loss is not None:
        report.max_rel["loss"] = _rel(st1.loss.reshape(1), st2.loss.reshape(1))
    for k in g2:
        report.max_rel[f"grad {k}"] = _rel(g1[k], g2[k]) if k in g1 else float("inf")
    return report
