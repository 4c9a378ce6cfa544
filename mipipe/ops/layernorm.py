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

from ._util import native_or_none

__all__ = ["add_dropout_layer_norm", "layer_norm_reference"]


def layer_norm_reference(
    x: Tensor, residual: Optional[Tensor], weight: Tensor, bias: Tensor, eps: float, p: float, training: bool
) -> Tensor:
    h = F.dropout(x, p, training) if p > 0 else x
    if residual is not None:
        h = residual + h
    return F.layer_norm(h, (h.shape[-1],), weight, bias, eps)


class _AddDropoutLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, eps, p):  # type: ignore[override]
        k = native_or_none(x)
        xc = x.contiguous()
        rc = residual.contiguous() if residual is not None else None
        y, z, mean, rstd, seed, offset = k.layernorm_fwd(xc, rc, weight, bias, eps, p, True)
        ctx.save_for_backward(z, mean, rstd, weight)
        ctx.p = p
        ctx.seed = seed
        ctx.offset = offset
        ctx.has_residual = residual is not None
        ctx.bias_main_grad = getattr(bias, "main_grad", None)
        return y

    @staticmethod
    def backward(ctx, dy):  # type: ignore[override]
        z, mean, rstd, weight = ctx.saved_tensors
        k = native_or_none(dy)
        mg = getattr(weight, "main_grad", None)
        mb = ctx.bias_main_grad
        if mg is not None and mb is not None:
            # dgamma/dbeta accumulate straight into the fp32 main_grad buffers
            dz, dx, dgamma, dbeta = k.layernorm_bwd(dy.contiguous(), z, mean, rstd, weight, ctx.p, ctx.seed,
                                                    ctx.offset, mg, mb)
        else:
            dz, dx, dgamma, dbeta = k.layernorm_bwd(dy.contiguous(), z, mean, rstd, weight, ctx.p, ctx.seed,
                                                    ctx.offset)
        if dx is None:
            dx = dz
        dres = dz if ctx.has_residual else None
        return dx, dres, dgamma, dbeta, None, None


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
    return _AddDropoutLayerNorm.apply(x, residual, weight, bias, float(eps), p)
