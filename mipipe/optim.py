"""Flat-buffer Adam with fused gradient clipping.

MI355X-first memory layout: at construction every parameter of a device is
re-pointed into ONE contiguous model buffer (bf16 for bf16 models), with an
fp32 master copy, an fp32 ``main_grad`` buffer and the two Adam moments laid
out identically.  Consequences:

* ops (``mipipe.ops.linear``, ``embedding``, ``layer_norm``) accumulate weight
  gradients straight into ``param.main_grad`` in fp32 -- no bf16 rounding
  across micro-batches and no per-parameter ``.grad`` tensors;
* ``clip_grad_norm_`` is one sum-of-squares kernel per stage, one 4-byte
  all-reduce across pipeline stages (the reference's cross-device norm stack,
  ``/root/reference/main.py:219``), and the clip coefficient is consumed on the
  device by the Adam kernel -- no host synchronisation;
* the Adam step is one kernel launch per (device, dtype) group.

Semantics match ``torch.optim.Adam`` (L2 weight decay) or ``AdamW``
(``adamw=True``) with ``clip_grad_norm_(max_norm)`` applied first.

``overlap_modules`` (optional): the step runs on a side stream of its own, in
chunks laid out in forward order (the non-GEMM parameters -- embedding,
LayerNorm, biases -- first, then the GEMM weights in the order given), with an
event after each chunk; a forward pre-hook on every module that owns
parameters makes the compute stream wait for the chunk holding that module's
last parameter, once per step.  The next step's forward then starts while the
update of later layers is still streaming through HBM: the memory-bound update
fills the CUs the GEMMs leave idle instead of running alone at the end of the
step.  The step also zero-fills the non-GEMM gradients on that stream (the
GEMM weights' gradients are overwritten by their first write), so under
``overlap_modules`` ``step()`` consumes the gradients.
"""
from __future__ import annotations

import math
import os
from typing import Dict, Iterable, List, Optional, Tuple

import torch
from torch import Tensor, nn

from . import _native_loader

__all__ = ["FlatAdam"]


class _Group:
    def __init__(self, params: List[nn.Parameter], device: torch.device, dtype: torch.dtype) -> None:
        # GEMM-only weights (ops.linear.mark_gemm_weight) first: their main_grad
        # is never zero-filled -- the step's first weight-gradient GEMM
        # overwrites it -- so zero_grad fills only the tail [n_lazy:).
        lazy = [p for p in params if getattr(p, "_mipipe_gemm_weight", False)]
        params = lazy + [p for p in params if not getattr(p, "_mipipe_gemm_weight", False)]
        self.lazy = lazy
        self.n_lazy = sum(p.numel() for p in lazy)
        self.params = params
        self.device = device
        self.dtype = dtype
        n = sum(p.numel() for p in params)
        self.numel = n
        self.model = torch.empty(n, dtype=dtype, device=device)
        off = 0
        with torch.no_grad():
            for p in params:
                k = p.numel()
                self.model[off : off + k].copy_(p.detach().reshape(-1))
                off += k
        self.master = self.model if dtype == torch.float32 else self.model.float()
        self.main_grad = torch.zeros(n, dtype=torch.float32, device=device)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=device)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=device)
        off = 0
        for p in params:
            k = p.numel()
            p.data = self.model[off : off + k].view_as(p)
            p.main_grad = self.main_grad[off : off + k].view_as(p)  # type: ignore[attr-defined]
            off += k


class FlatAdam:
    def __init__(
        self,
        params: Iterable[nn.Parameter],
        lr: float = 1e-3,
        betas: Tuple[float, float] = (0.9, 0.999),
        eps: float = 1e-8,
        weight_decay: float = 0.0,
        *,
        adamw: bool = False,
        max_grad_norm: Optional[float] = None,
        defer_wgrad: bool = False,
        overlap_modules: Optional[Iterable[nn.Module]] = None,
    ) -> None:
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.adamw = adamw
        self.max_grad_norm = max_grad_norm
        # defer_wgrad: zero_grad() starts queueing the weight-gradient GEMMs of
        # the coming backward (mipipe.ops.linear deferral) and fold_grads() --
        # called by grad_sumsq() and step() -- runs them as ONE K-segmented GEMM
        # per weight over all micro-batches: main_grad is written once per step
        # instead of read-modified-written per micro-batch, and a multi-GPU Pipe
        # sends its input gradients upstream without waiting for weight
        # gradients.  Read main_grad only after fold_grads().  Not for use
        # inside the multi-process engine, which defers on its own.
        self.defer_wgrad = defer_wgrad
        self._deferring = False
        self.step_count = 0
        buckets: Dict[Tuple[torch.device, torch.dtype], List[nn.Parameter]] = {}
        seen = set()
        for p in params:
            if not p.requires_grad or id(p) in seen:
                continue
            seen.add(id(p))
            buckets.setdefault((p.device, p.dtype), []).append(p)
        self.groups = [_Group(ps, d, t) for (d, t), ps in buckets.items()]
        self._overlap = None
        # chunk starts must keep the kernel's 16-byte vectors aligned: the non-GEMM range starts at n_lazy
        if (overlap_modules is not None and all(g.device.type == "cuda" for g in self.groups)
                and all(g.n_lazy % 64 == 0 for g in self.groups)):
            self._overlap = _Overlap(self, list(overlap_modules))

    @property
    def params(self) -> List[nn.Parameter]:
        return [p for g in self.groups for p in g.params]

    def zero_grad(self, set_to_none: bool = True, lazy: Optional[bool] = None) -> None:
        """Zeroes the gradients.  ``lazy``: GEMM-only weights are marked fresh
        instead of filled (their first gradient write overwrites; any still
        fresh at the optimizer step are zeroed then).  Default: on, unless
        MIPIPE_LAZY_ZERO=0."""
        if lazy is None:
            lazy = os.environ.get("MIPIPE_LAZY_ZERO", "1") != "0"
        # A backward whose gradients were never read: discard what it queued
        # for this optimizer's parameters (without running the GEMMs).
        from .ops.linear import deferred_param_ids, drop_deferred_wgrad

        mine = self._param_ids()
        if mine & deferred_param_ids():
            drop_deferred_wgrad(mine)
        if self._overlap is not None and self._overlap.zeroed:
            # the overlapped step zero-filled the non-GEMM gradients on its stream
            # and marked the GEMM weights fresh; nothing to queue here
            self._overlap.zeroed = False
            for g in self.groups:
                for p in g.params:
                    p.grad = None
            if self.defer_wgrad and not self._deferring:
                from .ops.linear import begin_deferred_wgrad

                self._deferring = begin_deferred_wgrad()
            return
        self.wait_step()
        for g in self.groups:
            if lazy and g.n_lazy:
                g.main_grad[g.n_lazy:].zero_()
                for p in g.lazy:
                    p._mg_fresh = True  # type: ignore[attr-defined]
            else:
                g.main_grad.zero_()
                for p in g.lazy:
                    p._mg_fresh = False  # type: ignore[attr-defined]
            for p in g.params:
                p.grad = None
        if self.defer_wgrad and not self._deferring:
            from .ops.linear import begin_deferred_wgrad

            # False when another optimizer's deferral is active: the queue is
            # shared, and fold_grads() flushes it when it holds our weights.
            self._deferring = begin_deferred_wgrad()

    def _param_ids(self) -> set:
        return {id(p) for g in self.groups for p in g.params}

    def fold_grads(self) -> None:
        """Adds any autograd ``.grad`` (ops without main_grad support) into
        main_grad and zeroes lazily-zeroed gradients nothing wrote this step
        (after running deferred weight-gradient GEMMs, with ``defer_wgrad``).

        The deferral queue is process-wide: the optimizer that opened it ends
        it here; any other optimizer whose weights sit in it flushes the queue
        (running every queued GEMM) and leaves the deferral open."""
        from .ops.linear import deferred_param_ids, end_deferred_wgrad, flush_wgrad

        if self._overlap is not None:
            self._overlap.wait_pending()  # modules that never ran forward this step
        if self._deferring:
            self._deferring = False
            end_deferred_wgrad()
        elif self._param_ids() & deferred_param_ids():
            flush_wgrad()
        with torch.no_grad():
            for g in self.groups:
                for p in g.params:
                    fresh = getattr(p, "_mg_fresh", False)
                    if p.grad is not None:
                        if fresh:
                            p.main_grad.copy_(p.grad)  # type: ignore[attr-defined]
                        else:
                            p.main_grad.add_(p.grad.float())  # type: ignore[attr-defined]
                        p.grad = None
                    elif fresh:
                        p.main_grad.zero_()  # type: ignore[attr-defined]
                    p._mg_fresh = False  # type: ignore[attr-defined]

    def grad_sumsq(self) -> Optional[Tensor]:
        """fp32 [1] tensor: sum of squared gradients of all local groups (on the
        first group's device).  Folds pending autograd ``.grad`` first."""
        self.fold_grads()
        total = None
        for g in self.groups:
            if g.device.type == "cuda":
                sq = _native_loader.kernels().sumsq(g.main_grad)
            else:
                sq = g.main_grad.double().pow(2).sum().float().reshape(1)
            total = sq if total is None else total + sq.to(total.device)
        return total

    @torch.no_grad()
    def step(self, grad_sumsq: Optional[Tensor] = None) -> None:
        """One Adam step.  ``grad_sumsq`` (global, e.g. all-reduced over pipeline
        stages) enables clipping to ``max_grad_norm``; None computes it locally."""
        self.fold_grads()
        if self.max_grad_norm is not None and grad_sumsq is None:
            grad_sumsq = self.grad_sumsq()
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        max_norm = float(self.max_grad_norm) if self.max_grad_norm is not None else 0.0
        if self._overlap is not None:
            self._overlap.step(grad_sumsq, b1, b2, bc1, bc2, max_norm)
            return
        for g in self.groups:
            sq = grad_sumsq.to(g.device) if grad_sumsq is not None else None
            if g.device.type == "cuda":
                k = _native_loader.kernels()
                model = g.model if g.dtype != torch.float32 else None
                k.adam_step(g.master, model, g.main_grad, g.exp_avg, g.exp_avg_sq, self.lr, b1, b2, self.eps,
                            self.weight_decay, bc1, bc2, sq, max_norm, self.adamw)
            else:
                self._step_eager(g, b1, b2, bc1, bc2, sq, max_norm)

    def _step_eager(self, g: _Group, b1, b2, bc1, bc2, sq, max_norm) -> None:
        grad = g.main_grad
        if sq is not None and max_norm > 0:
            coef = torch.clamp(max_norm / (sq.sqrt() + 1e-6), max=1.0)
            grad = grad * coef
        p = g.master
        if self.weight_decay:
            if self.adamw:
                p.mul_(1 - self.lr * self.weight_decay)
            else:
                grad = grad + self.weight_decay * p
        g.exp_avg.mul_(b1).add_(grad, alpha=1 - b1)
        g.exp_avg_sq.mul_(b2).addcmul_(grad, grad, value=1 - b2)
        denom = (g.exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(self.eps)
        p.addcdiv_(g.exp_avg, denom, value=-self.lr / bc1)
        if g.master is not g.model:
            g.model.copy_(p)

    def wait_step(self) -> None:
        """Makes the current stream wait for an overlapped step still in flight
        (no-op otherwise).  Needed only by code that reads the parameters or the
        optimizer state outside the hooked modules' forwards."""
        if self._overlap is not None:
            self._overlap.wait_all()

    def state_dict(self) -> dict:
        self.wait_step()
        return {
            "step": self.step_count,
            "groups": [
                {"master": g.master, "exp_avg": g.exp_avg, "exp_avg_sq": g.exp_avg_sq} for g in self.groups
            ],
        }

    def load_state_dict(self, state: dict) -> None:
        self.wait_step()
        self.step_count = int(state["step"])
        with torch.no_grad():
            for g, s in zip(self.groups, state["groups"]):
                g.master.copy_(s["master"])
                g.exp_avg.copy_(s["exp_avg"])
                g.exp_avg_sq.copy_(s["exp_avg_sq"])
                if g.master is not g.model:
                    g.model.copy_(g.master)


def overlap_chunks(sizes: List[int], n_lazy_params: int, min_chunk: int) -> Tuple[List[Tuple[int, int]], List[int]]:
    """Chunks of a group's flat buffer for the overlapped step, in issue order,
    and each parameter's chunk (the one that updates its LAST element).

    ``sizes``: parameter numels in buffer order, the first ``n_lazy_params``
    being the GEMM weights.  Chunk 0 is the non-GEMM range ``[n_lazy, n)`` (if
    any); the GEMM range follows, cut at parameter ends rounded down to 64
    elements once a chunk holds ``min_chunk`` elements."""
    n_lazy = sum(sizes[:n_lazy_params])
    n = sum(sizes)
    chunks: List[Tuple[int, int]] = [(n_lazy, n)] if n > n_lazy else []
    owner = [0] * len(sizes)
    start = off = 0
    pending: List[Tuple[int, int]] = []  # (parameter index, its end offset) not yet in a closed chunk
    for i in range(n_lazy_params):
        off += sizes[i]
        pending.append((i, off))
        end = off if off == n_lazy else (off // 64) * 64
        if end - start >= min_chunk or off == n_lazy:
            chunks.append((start, end))
            for j, j_end in pending:
                if j_end <= end:
                    owner[j] = len(chunks) - 1
            pending = [(j, j_end) for j, j_end in pending if j_end > end]
            start = end
    return chunks, owner


class _Overlap:
    """The side-stream step of :class:`FlatAdam` (``overlap_modules``).

    Chunks per group, in forward order: ``[n_lazy, n)`` (every non-GEMM
    parameter: embedding, LayerNorm, biases; its zero-fill rides with it), then
    the GEMM weights ``[0, n_lazy)`` cut at parameter ends into chunks of at
    least ``MIN_CHUNK`` elements.  Boundaries stay multiples of 64 elements (the
    Adam kernel's 16-byte vectors)."""

    MIN_CHUNK = 1 << 23

    def __init__(self, opt: "FlatAdam", modules: List[nn.Module]) -> None:
        self.opt = opt
        self.zeroed = False
        self.streams = {}
        self.chunks: List[List[Tuple[int, int]]] = []  # per group: [(start, end)] in issue order
        chunk_of: Dict[int, Tuple[int, int]] = {}  # id(param) -> (group, chunk index)
        for gi, g in enumerate(opt.groups):
            if g.device not in self.streams:
                # the least priority HIP offers: when a CU frees, the compute queue's next block goes first
                least = torch.cuda.Stream.priority_range()[0]
                prio = int(os.environ.get("MIPIPE_OPT_STREAM_PRIORITY", least))
                self.streams[g.device] = torch.cuda.Stream(device=g.device, priority=prio)
            chunks, owner = overlap_chunks([p.numel() for p in g.params], len(g.lazy), self.MIN_CHUNK)
            for p, ci in zip(g.params, owner):
                chunk_of[id(p)] = (gi, ci)
            self.chunks.append(chunks)
        # module -> the (group, chunk) its forward must wait for: the latest chunk holding a parameter of its
        # SUBTREE (a block may run a child through another method than __call__ -- e.g. forward_fanout -- so
        # the child's own hook would not fire); for the given root modules only their direct parameters (a
        # root's subtree is the whole stage: its children's hooks give the per-unit granularity)
        self.need: Dict[int, Dict[int, int]] = {}
        self.hooks = []

        def need_of(params) -> Dict[int, int]:
            need: Dict[int, int] = {}
            for p in params:
                if id(p) in chunk_of:
                    gi, ci = chunk_of[id(p)]
                    need[gi] = max(need.get(gi, -1), ci)
            return need

        for top in modules:
            for mod in top.modules():
                if id(mod) in self.need:
                    continue
                need = need_of(mod.parameters(recurse=mod is not top))
                if need:
                    self.need[id(mod)] = need
                    self.hooks.append(mod.register_forward_pre_hook(self._hook))
        # one event per chunk, re-recorded every step (a wait binds to the record before it)
        self.events = [[torch.cuda.Event() for _ in chunks] for chunks in self.chunks]
        self.pending: Dict[int, Dict[int, int]] = {}  # modules still to wait this step

    def _hook(self, mod: nn.Module, args) -> None:
        need = self.pending.pop(id(mod), None)
        if need:
            for gi, ci in need.items():
                g = self.opt.groups[gi]
                torch.cuda.current_stream(g.device).wait_event(self.events[gi][ci])

    def step(self, grad_sumsq: Optional[Tensor], b1, b2, bc1, bc2, max_norm) -> None:
        self.wait_pending()  # a step without a forward in between
        k = _native_loader.kernels()
        opt = self.opt
        for gi, g in enumerate(opt.groups):
            cur = torch.cuda.current_stream(g.device)
            side = self.streams[g.device]
            sq = grad_sumsq.to(g.device) if grad_sumsq is not None else None
            side.wait_stream(cur)  # gradients, the global norm
            if sq is not None:
                sq.record_stream(side)
            with torch.cuda.stream(side):
                for ci, (a, b) in enumerate(self.chunks[gi]):
                    model = g.model[a:b] if g.dtype != torch.float32 else None
                    k.adam_step(g.master[a:b], model, g.main_grad[a:b], g.exp_avg[a:b], g.exp_avg_sq[a:b],
                                opt.lr, b1, b2, opt.eps, opt.weight_decay, bc1, bc2, sq, max_norm, opt.adamw)
                    if ci == 0 and a == g.n_lazy:
                        g.main_grad[a:b].zero_()  # the non-GEMM gradients of the next step
                    self.events[gi][ci].record(side)
            for p in g.lazy:
                p._mg_fresh = True  # type: ignore[attr-defined]  # the next backward's first write overwrites
        self.zeroed = True
        self.pending = {mid: dict(need) for mid, need in self.need.items()}

    def wait_pending(self) -> None:
        """The current streams wait for every chunk a module has not waited for yet."""
        if self.pending:
            self.pending = {}
            self.wait_all()

    def wait_all(self) -> None:
        for g in self.opt.groups:
            torch.cuda.current_stream(g.device).wait_stream(self.streams[g.device])
        self.pending = {}
