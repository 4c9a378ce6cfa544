"""Fused ``LayerNorm(residual + dropout(x))`` (kernel: csrc/kernels/layernorm.hip).

GPU tensors always go to the HIP kernel (a missing extension raises); CPU
tensors use the eager reference so CPU-only tests exercise the same module
code.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor

from ._util import kernels_for
from .linear import accumulable

__all__ = ["add_dropout_layer_norm", "layer_norm_fanout", "layer_norm_reference"]


def layer_norm_reference(
    x: Tensor, residual: Optional[Tensor], weight: Tensor, bias: Tensor, eps: float, p: float, training: bool
) -> Tensor:
    h = F.dropout(x, p, training) if p > 0 else x
    if residual is not None:
        h = residual + h
    return F.layer_norm(h, (h.shape[-1],), weight, bias, eps)


class _AddDropoutLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, p, fanout=False, save=True):  # type: ignore[override]
        ctx.set_materialize_grads(False)
        k = kernels_for(x)
        xc = x.contiguous()
        rc = residual.contiguous() if residual is not None else None
        # z (the normalised sum) is written only for a backward, and only when it
        # is not the input itself: a pre-norm LayerNorm (no residual, no dropout)
        # saves x, and a forward under no_grad (a checkpointed stage) saves nothing
        z_is_x = residual is None and p == 0.0
        y, z, mean, rstd, seed, offset = k.layernorm_fwd(xc, rc, weight, bias, eps, p, save and not z_is_x)
        if save and z_is_x:
            z = xc
        ctx.save_for_backward(z, mean, rstd, weight)
        ctx.p = p
        ctx.seed = seed
        ctx.offset = offset
        ctx.has_residual = residual is not None
        ctx.bias = bias
        if fanout:
            # x again for its other consumer (pre-norm residual); its gradient
            # is added to dx inside the LayerNorm backward kernel
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dfan=None):  # type: ignore[override]
        z, mean, rstd, weight = ctx.saved_tensors
        if dy is None:  # only the fan-out branch carries a gradient
            return dfan, None, None, None, None, None, None, None
        k = kernels_for(dy)
        mg = accumulable(weight)
        mb = accumulable(ctx.bias) if ctx.bias is not None else None
        add = dfan.contiguous() if dfan is not None and dfan.dtype == dy.dtype else None
        if mg is not None and mb is not None:
            # dgamma/dbeta accumulate straight into the fp32 main_grad buffers
            dz, dx, dgamma, dbeta = k.layernorm_bwd(dy.contiguous(), z, mean, rstd, weight, ctx.p, ctx.seed,
                                                    ctx.offset, mg, mb, add)
        else:
            dz, dx, dgamma, dbeta = k.layernorm_bwd(dy.contiguous(), z, mean, rstd, weight, ctx.p, ctx.seed,
                                                    ctx.offset, None, None, add)
        if dx is None:
            dx = dz
        if dfan is not None and add is None:
            dx = dx + dfan
        dres = dz if ctx.has_residual else None
        return dx, dres, dgamma, dbeta, None, None, None, None


def add_dropout_layer_norm(
    x: Tensor,
    residual: Optional[Tensor],
    weight: Tensor,
    bias: Tensor,
    eps: float = 1e-5,
    p: float = 0.0,
    training: bool = True,
) -> Tensor:
    """``LayerNorm(residual + dropout(x, p))`` with affine ``weight``/``bias``."""
    p = float(p) if training else 0.0
    if not x.is_cuda:
        return layer_norm_reference(x, residual, weight, bias, eps, p, True)
    return _AddDropoutLayerNorm.apply(x, residual, weight, bias, float(eps), p, False, torch.is_grad_enabled())


def layer_norm_fanout(x: Tensor, weight: Tensor, bias: Tensor, eps: float = 1e-5):
    """``(LayerNorm(x), x')``: ``x'`` is ``x`` for its other consumer (the
    pre-norm residual ``x' + f(LN(x))``); the gradient reaching ``x'`` is added
    inside the LayerNorm backward kernel instead of by an autograd add kernel."""
    if not x.is_cuda or not torch.is_grad_enabled() or not x.requires_grad:
        return add_dropout_layer_norm(x, None, weight, bias, eps, 0.0, True), x
    return _AddDropoutLayerNorm.apply(x, None, weight, bias, float(eps), 0.0, True)
