"""Token embedding x scale + positional encoding + dropout (kernel: csrc/kernels/embedding.hip).

The backward accumulates straight into ``weight.main_grad`` (fp32) when the
parameter has one (flat-buffer optimizer, :mod:`mipipe.optim`) and returns no
dense gradient; otherwise it builds a dense fp32 gradient and casts it.

A positional table that requires a gradient (GPT-2's learned positions, fp32)
rides through the same kernels: the forward adds it in the gather, the
backward's scatter-add also accumulates each masked row at its position (into
the table's ``main_grad`` when it has one) -- no separate add, dropout or
batch reduction.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor

from ._util import kernels_for
from .linear import accumulable

__all__ = ["embed_scale_posenc_dropout"]


class _Embed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens, weight, pe, scale, p):  # type: ignore[override]
        k = kernels_for(weight)
        out, seed, offset = k.embedding_fwd(tokens.contiguous(), weight, pe, scale, p)
        ctx.save_for_backward(tokens.contiguous())
        ctx.weight, ctx.pe = weight, (pe if ctx.needs_input_grad[2] else None)
        ctx.scale, ctx.p, ctx.seed, ctx.offset = scale, p, seed, offset
        return out

    @staticmethod
    def backward(ctx, dout):  # type: ignore[override]
        (tokens,) = ctx.saved_tensors
        weight, pe = ctx.weight, ctx.pe
        k = kernels_for(dout)
        main = accumulable(weight)
        acc = main if main is not None else torch.zeros(weight.shape, dtype=torch.float32, device=weight.device)
        dpe = dpe_main = None
        if pe is not None:
            dpe_main = accumulable(pe)
            dpe = dpe_main if dpe_main is not None else torch.zeros(pe.shape, dtype=torch.float32, device=pe.device)
        k.embedding_bwd(tokens, dout.contiguous(), acc, ctx.scale, ctx.p, ctx.seed, ctx.offset, dpe)
        dw = None if main is not None else acc.to(weight.dtype)
        dp = None if (pe is None or dpe_main is not None) else dpe.to(pe.dtype)
        return None, dw, dp, None, None


def embed_scale_posenc_dropout(
    tokens: Tensor, weight: Tensor, pe: Optional[Tensor], scale: float, p: float, training: bool = True
) -> Tensor:
    """``dropout(weight[tokens] * scale + pe[:S])`` for ``tokens [B, S]`` -> ``[B, S, E]``."""
    p = float(p) if training else 0.0
    if not weight.is_cuda:
        x = F.embedding(tokens, weight) * scale
        if pe is not None:
            x = x + pe[: tokens.shape[1]].to(x.dtype)
        return F.dropout(x, p, True) if p > 0 else x
    if pe is not None and pe.dtype not in (torch.float32, weight.dtype):
        pe = pe.float()
    if pe is not None and not pe.is_contiguous():
        pe = pe.contiguous()
    # a table in the model dtype is read as stored: its gradient goes straight to
    # its fp32 main_grad (no cast node, no dense gradient)
    return _Embed.apply(tokens, weight, pe, float(scale), p)
