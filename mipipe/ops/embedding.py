"""Token embedding x scale + positional encoding + dropout (kernel: csrc/kernels/embedding.hip).

The backward accumulates straight into ``weight.main_grad`` (fp32) when the
parameter has one (flat-buffer optimizer, :mod:`mipipe.optim`) and returns no
dense gradient; otherwise it builds a dense fp32 gradient and casts it.
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
        ctx.save_for_backward(tokens)
        ctx.weight = weight
        ctx.scale, ctx.p, ctx.seed, ctx.offset = scale, p, seed, offset
        return out

    @staticmethod
    def backward(ctx, dout):  # type: ignore[override]
        (tokens,) = ctx.saved_tensors
        weight = ctx.weight
        k = kernels_for(dout)
        main = accumulable(weight)
        if main is not None:
            k.embedding_bwd(tokens, dout.contiguous(), main, ctx.scale, ctx.p, ctx.seed, ctx.offset)
            return None, None, None, None, None
        acc = torch.zeros(weight.shape, dtype=torch.float32, device=weight.device)
        k.embedding_bwd(tokens, dout.contiguous(), acc, ctx.scale, ctx.p, ctx.seed, ctx.offset)
        return None, acc.to(weight.dtype), None, None, None


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
    if pe is not None and pe.dtype != torch.float32:
        pe = pe.float()
    return _Embed.apply(tokens, weight, pe, float(scale), p)
