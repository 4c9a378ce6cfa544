"""DeferredBatchNorm: mini-batch running statistics under micro-batching.

With ``Pipe(..., deferred_batch_norm=True)`` (``/root/reference/pipe.py:261-265,
341-342``) each ``_BatchNorm`` that tracks running statistics is replaced by this
module.  Normalisation still uses the *micro-batch* statistics (that is what
the forward of a micro-batch can see), but the running mean/variance are
updated once per mini-batch from sums accumulated over all ``chunks``
micro-batches, so they equal what a single BatchNorm over the whole mini-batch
would record (unbiased variance, like ``nn.BatchNorm``).  Recomputation
(``is_recomputing()``) does not count twice.
"""
from __future__ import annotations

from typing import Optional, TypeVar, cast

import torch
import torch.nn.functional as F
from torch import Tensor, nn
from torch.nn.modules.batchnorm import _BatchNorm

from .checkpoint import is_recomputing

__all__ = ["DeferredBatchNorm"]

TModule = TypeVar("TModule", bound=nn.Module)


class DeferredBatchNorm(_BatchNorm):
    sum: Tensor
    sum_squares: Tensor
    running_mean: Tensor
    running_var: Tensor
    num_batches_tracked: Tensor

    def __init__(
        self,
        num_features: int,
        eps: float = 1e-5,
        momentum: Optional[float] = 0.1,
        affine: bool = True,
        chunks: int = 1,
    ) -> None:
        super().__init__(num_features, eps, momentum, affine, track_running_stats=True)
        self.register_buffer("sum", torch.zeros_like(self.running_mean))
        self.register_buffer("sum_squares", torch.zeros_like(self.running_var))
        self.counter = 0
        self.tracked = 0
        self.chunks = chunks

    def _check_input_dim(self, input: Tensor) -> None:
        # Per-channel statistics need at least (N, C, L).
        if input.dim() <= 2:
            raise ValueError(f"expected at least 3D input (got {input.dim()}D input)")

    def _track(self, input: Tensor) -> bool:
        """Accumulates sums of one micro-batch; True once all chunks are in."""
        dims = [0, *range(2, input.dim())]
        with torch.no_grad():
            x = input.detach().float()
            self.sum += x.sum(dims).to(self.sum.dtype)
            self.sum_squares += (x * x).sum(dims).to(self.sum_squares.dtype)
        self.counter += input.numel() // input.size(1)
        self.tracked += 1
        return self.tracked == self.chunks

    def _commit(self) -> None:
        """Folds the mini-batch statistics into the running averages."""
        self.num_batches_tracked += 1
        if self.momentum is None:
            factor = 1.0 / float(self.num_batches_tracked)
        else:
            factor = float(self.momentum)
        n = self.counter
        mean = self.sum / n
        var = self.sum_squares / n - mean * mean
        if n > 1:
            var = var * (n / (n - 1))  # unbiased, as nn.BatchNorm records
        with torch.no_grad():
            self.running_mean.mul_(1 - factor).add_(mean, alpha=factor)
            self.running_var.mul_(1 - factor).add_(var, alpha=factor)
            self.sum.zero_()
            self.sum_squares.zero_()
        self.counter = 0
        self.tracked = 0

    def forward(self, input: Tensor) -> Tensor:  # type: ignore[override]
        self._check_input_dim(input)
        if not self.training:
            return F.batch_norm(
                input, self.running_mean, self.running_var, self.weight, self.bias,
                training=False, momentum=0.0, eps=self.eps,
            )
        if not is_recomputing():
            if self._track(input):
                self._commit()
        return F.batch_norm(
            input, None, None, self.weight, self.bias, training=True, momentum=0.0, eps=self.eps
        )

    @classmethod
    def convert_deferred_batch_norm(cls, module: TModule, chunks: int = 1) -> TModule:
        """Returns ``module`` with every tracking ``_BatchNorm`` replaced in place
        (parameters and buffers are shared, not copied)."""
        if isinstance(module, DeferredBatchNorm) and module.chunks is chunks:
            return cast(TModule, module)

        out: nn.Module = module
        if isinstance(module, _BatchNorm) and module.track_running_stats:
            out = DeferredBatchNorm(module.num_features, module.eps, module.momentum, module.affine, chunks)
            if module.affine:
                out.register_parameter("weight", module.weight)
                out.register_parameter("bias", module.bias)
            out.register_buffer("running_mean", module.running_mean)
            out.register_buffer("running_var", module.running_var)
            out.register_buffer("num_batches_tracked", module.num_batches_tracked)
            device = module.running_mean.device
            out.sum = out.sum.to(device=device, dtype=module.running_mean.dtype)
            out.sum_squares = out.sum_squares.to(device=device, dtype=module.running_var.dtype)

        for name, child in module.named_children():
            out.add_module(name, cls.convert_deferred_batch_norm(child, chunks))
        return cast(TModule, out)
