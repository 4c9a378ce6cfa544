"""Fork / Join: artificial autograd edges between micro-batches.

``fork(x) -> (x', phony)`` and ``join(y, phony) -> y'`` are identity functions in
both directions; the only thing they add is a graph edge ``x' -> phony -> y'``.
The scheduler uses them to force micro-batch ``i-1`` to run backward through a
partition only after micro-batch ``i`` has (``/root/reference/pipeline.py:43-48``),
to hang recomputation off the graph (checkpoint.py) and to route skip tensors
through portals (skip/portal.py).  Semantics: ``/root/reference/README.md:122-183``.
"""
from __future__ import annotations

from typing import Tuple

import torch

from .phony import get_phony

__all__ = ["fork", "Fork", "join", "Join"]


class Fork(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor):  # type: ignore[override]
        phony = get_phony(x.device, requires_grad=False)
        return x.detach(), phony.detach()

    @staticmethod
    def backward(ctx, grad_x: torch.Tensor, grad_phony: torch.Tensor):  # type: ignore[override]
        # The phony gradient carries no information; its *arrival* is what
        # releases this node.
        return grad_x


class Join(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, phony: torch.Tensor):  # type: ignore[override]
        return x.detach()

    @staticmethod
    def backward(ctx, grad_x: torch.Tensor):  # type: ignore[override]
        return grad_x, None


def fork(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Branches a phony off ``x``.  Only adds an edge when autograd tracks ``x``."""
    if torch.is_grad_enabled() and x.requires_grad:
        return Fork.apply(x)
    return x, get_phony(x.device, requires_grad=False)


def join(x: torch.Tensor, phony: torch.Tensor) -> torch.Tensor:
    """Merges ``phony`` into ``x`` so that ``x``'s backward waits for the phony's."""
    if torch.is_grad_enabled() and (x.requires_grad or phony.requires_grad):
        return Join.apply(x, phony)
    return x
