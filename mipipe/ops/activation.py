"""Fused bias + activation + dropout (kernel: csrc/kernels/elementwise.hip)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor

from ._util import kernels_for

__all__ = ["bias_act_dropout", "ACTIVATIONS", "bias_act_reference"]

ACTIVATIONS = {None: 0, "none": 0, "relu": 1, "gelu": 2}


def bias_act_reference(x: Tensor, bias: Optional[Tensor], activation: Optional[str], p: float, training: bool) -> Tensor:
    y = x + bias if bias is not None else x
    if activation == "relu":
        y = F.relu(y)
    elif activation == "gelu":
        y = F.gelu(y)
    return F.dropout(y, p, training) if p > 0 else y


class _BiasActDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act, p):  # type: ignore[override]
        k = kernels_for(x)
        xc = x.contiguous()
        y, seed, offset = k.bias_act_fwd(xc, bias, act, p)
        # ReLU/identity backward needs only the output; GELU the pre-activation.
        ctx.save_for_backward(xc if act == 2 else y, bias)
        ctx.act, ctx.p, ctx.seed, ctx.offset = act, p, seed, offset
        return y

    @staticmethod
    def backward(ctx, dy):  # type: ignore[override]
        saved, bias = ctx.saved_tensors
        k = kernels_for(dy)
        dx, db = k.bias_act_bwd(
            dy.contiguous(), saved, bias, ctx.act, ctx.p, ctx.seed, ctx.offset, bias is not None and ctx.needs_input_grad[1]
        )
        return dx, db, None, None


def bias_act_dropout(
    x: Tensor, bias: Optional[Tensor], activation: Optional[str], p: float = 0.0, training: bool = True
) -> Tensor:
    """``dropout(act(x + bias), p)``."""
    p = float(p) if training else 0.0
    if not x.is_cuda:
        return bias_act_reference(x, bias, activation, p, True)
    return _BiasActDropout.apply(x, bias, ACTIVATIONS[activation], p)
