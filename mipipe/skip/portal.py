"""Portals: carry a skip tensor across partitions outside the batch.

A portal holds one stashed tensor and exposes three autograd functions, each
of which only emits or consumes a *phony* on the batch's own graph:

* :class:`PortalBlue`   -- at the stash site; backward hands the gradient that
  came through the portal back to the stashed tensor.
* :class:`PortalCopy`   -- at the pop partition's fence; moves the tensor (and in
  backward its gradient) between devices on the copy streams, like ``Copy``.
* :class:`PortalOrange` -- at the pop site; forward re-emits the tensor, backward
  parks its gradient in the portal.

Because every function is threaded onto the batch's phony chain the autograd
engine runs their backwards in the order Orange -> Copy -> Blue.

Tensor life: a portal drops its tensor as soon as the last forward user has
taken it, to keep activation memory at the reference's level.  The number of
forward users depends on checkpointing (see ``SkipTrackerThroughPortals.save``).

Attribution: the portal design (three autograd functions on the phony chain,
the 3-vs-2 forward-user tensor life, PortalCopy reusing Copy's forward /
backward) follows upstream PyTorch's torch.distributed.pipeline.sync.skip
(BSD-3-Clause, originally from torchgpipe); this file re-implements that
behaviour, which SURVEY.md C14 requires bit-for-bit.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from ..copy import Copy
from ..phony import get_phony
from ..stream import AbstractStream, get_device

__all__ = ["Portal", "PortalBlue", "PortalOrange", "PortalCopy"]


class Portal:
    """Holds one skip tensor (with a use budget) and its gradient."""

    def __init__(self, tensor: Optional[Tensor], tensor_life: int) -> None:
        self.tensor: Optional[Tensor] = None
        self.tensor_life = 0
        self.put_tensor(tensor, tensor_life)
        self.grad: Optional[Tensor] = None

    # -- forward-side uses ------------------------------------------------------
    def blue(self) -> Tensor:
        """Stash site: returns a phony that carries the portal's backward edge."""
        tensor = self.use_tensor()
        if tensor is None:
            return get_phony(torch.device("cpu"), requires_grad=False)
        return PortalBlue.apply(self, tensor)

    def orange(self, phony: Tensor) -> Optional[Tensor]:
        """Pop site: re-emits the tensor, attached after ``phony``."""
        self.check_tensor_life()
        if self.tensor is None:
            return self.use_tensor()
        return PortalOrange.apply(self, phony)

    def copy(self, prev_stream: AbstractStream, next_stream: AbstractStream, phony: Tensor) -> Tensor:
        """Fence of the pop partition: moves the tensor to the next device."""
        if self.tensor is None:
            return get_phony(torch.device("cpu"), requires_grad=False)
        return PortalCopy.apply(self, prev_stream, next_stream, phony)

    # -- bookkeeping -----------------------------------------------------------
    def check_tensor_life(self) -> None:
        if self.tensor_life <= 0:
            raise RuntimeError("tensor in portal has been removed")

    def put_tensor(self, tensor: Optional[Tensor], tensor_life: int) -> None:
        self.tensor_life = tensor_life
        self.tensor = tensor if tensor_life > 0 else None

    def use_tensor(self) -> Optional[Tensor]:
        self.check_tensor_life()
        tensor = self.tensor
        self.tensor_life -= 1
        if self.tensor_life <= 0:
            self.tensor = None
        return tensor

    def put_grad(self, grad: Optional[Tensor]) -> None:
        self.grad = grad

    def use_grad(self) -> Optional[Tensor]:
        grad, self.grad = self.grad, None
        return grad


class PortalBlue(torch.autograd.Function):
    @staticmethod
    def forward(ctx, portal: Portal, tensor: Tensor):  # type: ignore[override]
        ctx.portal = portal
        return get_phony(tensor.device, requires_grad=False).detach()

    @staticmethod
    def backward(ctx, grad_phony: Tensor) -> Tuple[None, Optional[Tensor]]:  # type: ignore[override]
        return None, ctx.portal.use_grad()


class PortalOrange(torch.autograd.Function):
    @staticmethod
    def forward(ctx, portal: Portal, phony: Tensor):  # type: ignore[override]
        ctx.portal = portal
        tensor = portal.use_tensor()
        assert tensor is not None
        return tensor.detach()

    @staticmethod
    def backward(ctx, grad: Tensor) -> Tuple[None, None]:  # type: ignore[override]
        ctx.portal.put_grad(grad)
        return None, None


class PortalCopy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, portal: Portal, prev_stream, next_stream, phony):  # type: ignore[override]
        ctx.portal = portal
        assert portal.tensor is not None
        # Reuse Copy's stream discipline (record_stream on both ends).
        (portal.tensor,) = Copy.forward(ctx, prev_stream, next_stream, portal.tensor)
        return get_phony(get_device(next_stream), requires_grad=False).detach()

    @staticmethod
    def backward(ctx, grad_phony):  # type: ignore[override]
        portal = ctx.portal
        assert portal.grad is not None
        _, _, portal.grad = Copy.backward(ctx, portal.grad)
        return None, None, None, None
