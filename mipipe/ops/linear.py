"""Linear layers: GEMM + fused bias / activation / dropout epilogue.

Forward:  ``y = dropout(act(x @ W^T + b))``.
Backward: the epilogue's backward is one fused elementwise pass
(csrc/kernels/elementwise.hip) that also yields ``db``; then
``dx = dpre @ W`` and ``dW = dpre^T @ x``.  When the weight carries a
``main_grad`` fp32 buffer (flat-buffer optimizer, :mod:`mipipe.optim`) ``dW``
is accumulated there in fp32 and autograd receives no weight gradient, so
micro-batch gradient accumulation never rounds through bf16.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor

from ._util import native_or_none
from .activation import ACTIVATIONS, bias_act_reference

__all__ = ["linear", "accumulate_wgrad"]

_MIXED_ADDMM: Optional[bool] = None


def accumulate_wgrad(main_grad: Tensor, dy2d: Tensor, x2d: Tensor) -> None:
    """``main_grad (fp32) += dy2d^T @ x2d`` with bf16 operands."""
    global _MIXED_ADDMM
    if _MIXED_ADDMM is None or _MIXED_ADDMM:
        try:
            torch.addmm(main_grad, dy2d.t(), x2d, out_dtype=torch.float32, out=main_grad)
            _MIXED_ADDMM = True
            return
        except (RuntimeError, TypeError):
            _MIXED_ADDMM = False
    main_grad.add_(torch.matmul(dy2d.t(), x2d).float())


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act, p):  # type: ignore[override]
        k = native_or_none(x)
        y = torch.matmul(x, weight.t())
        fused = act != 0 or p > 0.0
        seed = offset = 0
        if fused:
            pre = y
            y, seed, offset = k.bias_act_fwd(pre, bias, act, p)
            saved = pre if act == 2 else y
        else:
            if bias is not None:
                y = y + bias
            saved = None
        ctx.save_for_backward(x, weight, bias, saved)
        ctx.act, ctx.p, ctx.seed, ctx.offset, ctx.fused = act, p, seed, offset, fused
        return y

    @staticmethod
    def backward(ctx, dy):  # type: ignore[override]
        x, weight, bias, saved = ctx.saved_tensors
        k = native_or_none(dy)
        dy = dy.contiguous()
        need_db = bias is not None and ctx.needs_input_grad[2]
        if ctx.fused:
            dpre, db = k.bias_act_bwd(dy, saved, bias, ctx.act, ctx.p, ctx.seed, ctx.offset, need_db)
        else:
            dpre = dy
            db = k.column_sum(dy.view(-1, dy.shape[-1])) if need_db else None
        dx = torch.matmul(dpre, weight) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            d2 = dpre.reshape(-1, dpre.shape[-1])
            x2 = x.reshape(-1, x.shape[-1])
            main = getattr(weight, "main_grad", None)
            if main is not None:
                accumulate_wgrad(main, d2, x2)
            else:
                dw = torch.matmul(d2.t(), x2)
        if db is not None and bias is not None:
            main_b = getattr(bias, "main_grad", None)
            if main_b is not None:
                main_b.add_(db)
                db = None
        return dx, dw, db, None, None


def linear(
    x: Tensor,
    weight: Tensor,
    bias: Optional[Tensor] = None,
    activation: Optional[str] = None,
    dropout_p: float = 0.0,
    training: bool = True,
) -> Tensor:
    """``dropout(act(x @ weight.T + bias))``."""
    p = float(dropout_p) if training else 0.0
    if not x.is_cuda:
        y = F.linear(x, weight)
        return bias_act_reference(y, bias, activation, p, True)
    return _Linear.apply(x, weight, bias, ACTIVATIONS[activation], p)
