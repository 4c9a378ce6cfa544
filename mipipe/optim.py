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

    def state_dict(self) -> dict:
        return {
            "step": self.step_count,
            "groups": [
                {"master": g.master, "exp_avg": g.exp_avg, "exp_avg_sq": g.exp_avg_sq} for g in self.groups
            ],
        }

    def load_state_dict(self, state: dict) -> None:
        self.step_count = int(state["step"])
        with torch.no_grad():
            for g, s in zip(self.groups, state["groups"]):
                g.master.copy_(s["master"])
                g.exp_avg.copy_(s["exp_avg"])
                g.exp_avg_sq.copy_(s["exp_avg_sq"])
                if g.master is not g.model:
                    g.model.copy_(g.master)
