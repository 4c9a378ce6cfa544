"""Multi-process synchronous pipeline (GPipe) over RCCL -- one rank per MI355X.

This is the scale-out form of :class:`mipipe.Pipe` (SURVEY §5.8 (b), §7.2 step
5): instead of one process driving every GPU from worker threads with peer
copies, each GPU is one process (``torchrun --nproc-per-node N``) that owns a
contiguous slice of the model, and activations / gradients move between
neighbouring ranks with RCCL send/recv over xGMI.  It keeps the reference's
semantics:

* micro-batching of the mini-batch on dim 0 into ``chunks`` micro-batches;
* the GPipe fill-drain schedule: all forwards (clock cycles ``i + j = k``), then
  all backwards in reverse micro-batch order -- exactly the order the
  reference's fork/join phonies force (``/root/reference/pipeline.py:128-132``);
* ``checkpoint`` in {``always``, ``except_last``, ``never``}: checkpointed
  micro-batches run forward under ``no_grad`` keeping only the stage input and
  the RNG state, and are recomputed (bit-identical dropout) right before their
  backward (``/root/reference/pipe.py:255-260,354``);
* eval mode never checkpoints (``pipeline.py:153-155``).

Optionally ``schedule="1f1b"`` (PipeDream-flush): same bubble, activation
memory bounded by the number of stages instead of ``chunks``.

Overlap: all receives of a phase are posted before the first compute so each
transfer lands while the previous micro-batch computes; sends are asynchronous.
Per-stage busy time is measured with HIP events to report the pipeline bubble.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import Tensor, nn

from ..checkpoint import enable_checkpointing, enable_recomputing
from ..pipeline import checkpoint_stop_for
from .p2p import P2P

__all__ = ["PipelineEngine", "StepStats", "schedule_actions"]


@dataclass
class StepStats:
    loss: Optional[Tensor] = None
    busy_ms: float = 0.0          # GPU time of this stage's compute (events)
    step_ms: float = 0.0          # wall time of the step on this rank
    forward_ms: List[float] = field(default_factory=list)
    backward_ms: List[float] = field(default_factory=list)


def schedule_actions(kind: str, m: int, n: int, j: int) -> List[Tuple[str, int]]:
    """Ordered (F|B, micro-batch) actions of stage ``j`` of ``n`` for ``m`` micro-batches."""
    if kind == "gpipe":
        return [("F", i) for i in range(m)] + [("B", i) for i in reversed(range(m))]
    if kind == "1f1b":
        warm = min(n - j - 1, m)
        acts: List[Tuple[str, int]] = [("F", i) for i in range(warm)]
        f, b = warm, 0
        while f < m:
            acts.append(("F", f))
            f += 1
            acts.append(("B", b))
            b += 1
        while b < m:
            acts.append(("B", b))
            b += 1
        return acts
    raise ValueError(f"unknown schedule {kind!r}")


class _RNGState:
    __slots__ = ("cpu", "dev")

    def __init__(self, device: torch.device) -> None:
        self.cpu = torch.get_rng_state()
        self.dev = torch.cuda.get_rng_state(device) if device.type == "cuda" else None


class PipelineEngine:
    """Runs one training (or eval) step of a pipeline stage.

    Args:
        module: this rank's stage (single tensor in, single tensor out).
        chunks: micro-batches per mini-batch.
        checkpoint: ``always`` / ``except_last`` / ``never``.
        act_shape: shape of the activation this stage RECEIVES per micro-batch
            (gradient buffers take the shape of this stage's outputs).
        act_dtype: its dtype.
        loss_fn: ``loss_fn(output, target) -> scalar`` on the last stage.
        group: process group of the pipeline (default: WORLD).
        schedule: ``gpipe`` (reference order) or ``1f1b``.
    """

    def __init__(
        self,
        module: nn.Module,
        *,
        chunks: int,
        checkpoint: str = "never",
        act_shape: Sequence[int],
        act_dtype: torch.dtype,
        loss_fn: Optional[Callable[[Tensor, Tensor], Tensor]] = None,
        group: Optional[dist.ProcessGroup] = None,
        device: Optional[torch.device] = None,
        schedule: str = "gpipe",
        measure: bool = False,
    ) -> None:
        if checkpoint not in ("always", "except_last", "never"):
            raise ValueError("checkpoint is not one of 'always', 'except_last', or 'never'")
        self.module = module
        self.chunks = int(chunks)
        self.checkpoint = checkpoint
        self.act_shape = tuple(act_shape)
        self.act_dtype = act_dtype
        self.loss_fn = loss_fn
        self.schedule = schedule
        self.measure = measure
        if dist.is_available() and dist.is_initialized():
            self.p2p: Optional[P2P] = P2P(group)
            self.rank, self.world = self.p2p.rank, self.p2p.world
        else:
            self.p2p = None
            self.rank, self.world = 0, 1
        if schedule != "gpipe" and self.world > 1:
            # 1F1B interleaves activation sends with gradient receives on the same
            # link; without grouped send/recv that deadlocks on RCCL rendezvous.
            raise NotImplementedError("multi-rank schedule '1f1b' is not supported yet; use 'gpipe'")
        self.device = device or next(module.parameters()).device
        self.is_first = self.rank == 0
        self.is_last = self.rank == self.world - 1

    # ------------------------------------------------------------------ helpers
    def _new_act(self, like: Optional[Tensor] = None) -> Tensor:
        if like is not None:
            return torch.empty(like.shape, dtype=like.dtype, device=self.device)
        return torch.empty(self.act_shape, dtype=self.act_dtype, device=self.device)

    def _timer(self):
        if not self.measure or self.device.type != "cuda":
            return None
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    # ------------------------------------------------------------------ step
    def step(self, inputs: Optional[Sequence[Tensor]] = None, targets: Optional[Sequence[Tensor]] = None) -> StepStats:
        """Forward + backward of one mini-batch given as per-micro-batch lists.

        ``inputs`` (first stage) and ``targets`` (last stage) have ``chunks``
        entries.  Gradients accumulate into the parameters (or their
        ``main_grad``); the caller runs the optimizer.  Returns the mean loss on
        the last stage.
        """
        m, n, j = self.chunks, self.world, self.rank
        training = self.module.training and torch.is_grad_enabled()
        stop = checkpoint_stop_for(self.checkpoint, m) if self.module.training else 0
        stats = StepStats()
        t0 = time.perf_counter()

        # Post every activation receive of the forward phase up front.
        recv_x: List[Optional[Tensor]] = [None] * m
        recv_w: List[Optional[dist.Work]] = [None] * m
        if not self.is_first:
            for i in range(m):
                recv_x[i] = self._new_act()
                recv_w[i] = self.p2p.irecv(recv_x[i], j - 1)

        stage_in: List[Optional[Tensor]] = [None] * m
        stage_out: List[Optional[Tensor]] = [None] * m
        rng: List[Optional[_RNGState]] = [None] * m
        losses: List[Tensor] = []
        sends: List[dist.Work] = []
        grad_w: List[Optional[dist.Work]] = [None] * m
        grad_buf: List[Optional[Tensor]] = [None] * m
        events = []

        def forward(i: int) -> None:
            if self.is_first:
                x = inputs[i]
            else:
                recv_w[i].wait()
                x = recv_x[i]
                recv_x[i] = None
                if training:
                    x.requires_grad_(True)
            tm = self._timer()
            if tm:
                tm[0].record()
            if training and i < stop:
                rng[i] = _RNGState(self.device)
                with torch.no_grad(), enable_checkpointing():
                    y = self.module(x)
            else:
                y = self.module(x)
            if self.is_last and self.loss_fn is not None:
                loss = self.loss_fn(y, targets[i])
                losses.append(loss.detach())
                y = loss / m  # backward seeds from the scaled loss
            if tm:
                tm[1].record()
                events.append(("F", tm))
            stage_in[i] = x
            stage_out[i] = y if (training and i >= stop) else None
            out_meta[i] = torch.empty(y.shape, dtype=y.dtype, device="meta")
            if not self.is_last:
                sends.append(self.p2p.isend(y.detach(), j + 1))

        out_meta: List[Optional[Tensor]] = [None] * m

        def post_grad_recv(i: int) -> None:
            if not self.is_last and grad_w[i] is None:
                grad_buf[i] = self._new_act(out_meta[i])
                grad_w[i] = self.p2p.irecv(grad_buf[i], j + 1)

        def backward(i: int) -> None:
            x = stage_in[i]
            tm = self._timer()
            if not self.is_last:
                grad_w[i].wait()
            if tm:
                tm[0].record()
            if stage_out[i] is None:
                # Recompute with the RNG state of the original forward.
                st = rng[i]
                devices = [self.device] if self.device.type == "cuda" else []
                with torch.random.fork_rng(devices=devices):
                    torch.set_rng_state(st.cpu)
                    if st.dev is not None:
                        torch.cuda.set_rng_state(st.dev, self.device)
                    with torch.enable_grad(), enable_recomputing():
                        y = self.module(x)
                        if self.is_last and self.loss_fn is not None:
                            y = self.loss_fn(y, targets[i]) / m
            else:
                y = stage_out[i]
            if self.is_last:
                y.backward()
            else:
                torch.autograd.backward(y, grad_buf[i])
            if tm:
                tm[1].record()
                events.append(("B", tm))
            stage_out[i] = None
            grad_buf[i] = None
            if not self.is_first:
                sends.append(self.p2p.isend(x.grad, j - 1))
            stage_in[i] = None
            rng[i] = None

        actions = schedule_actions(self.schedule, m, n, j) if training else [("F", i) for i in range(m)]
        started_backward = False
        for kind, i in actions:
            if kind == "F":
                with torch.set_grad_enabled(training):
                    forward(i)
            else:
                if not started_backward:
                    started_backward = True
                    # Post all gradient receives of the drain phase at once.
                    if self.schedule == "gpipe":
                        for k in reversed(range(m)):
                            post_grad_recv(k)
                post_grad_recv(i)
                backward(i)

        for w in sends:
            w.wait()

        if losses:
            stats.loss = torch.stack(losses).float().mean()
        if events:
            torch.cuda.synchronize(self.device)
            for kind, (a, b) in events:
                ms = a.elapsed_time(b)
                (stats.forward_ms if kind == "F" else stats.backward_ms).append(ms)
            stats.busy_ms = sum(stats.forward_ms) + sum(stats.backward_ms)
        stats.step_ms = (time.perf_counter() - t0) * 1e3
        return stats
