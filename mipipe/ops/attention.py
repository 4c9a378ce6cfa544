"""Scaled dot-product attention (kernel: csrc/kernels/attention.hip).

Layout: ``q, k, v`` are ``[B, H, S, D]`` (any strides with unit stride on D
are made contiguous).  Supports causal masking and attention-probability
dropout whose mask is regenerated from the Philox (seed, offset) in backward.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor

from ._util import native_or_none

__all__ = ["attention", "attention_reference"]


def attention_reference(q: Tensor, k: Tensor, v: Tensor, causal: bool, p: float, scale: Optional[float] = None) -> Tensor:
    """Eager fp32 math (CPU path and test oracle)."""
    d = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(d)
    s = torch.matmul(q.float(), k.float().transpose(-1, -2)) * scale
    if causal:
        n, m = s.shape[-2], s.shape[-1]
        mask = torch.ones(n, m, dtype=torch.bool, device=s.device).triu(1 + m - n)
        s = s.masked_fill(mask, float("-inf"))
    pr = torch.softmax(s, dim=-1)
    if p > 0:
        pr = F.dropout(pr, p, True)
    return torch.matmul(pr, v.float()).to(q.dtype)


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, p, scale):  # type: ignore[override]
        kern = native_or_none(q)
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        o, lse, seed, offset = kern.attention_fwd(q, k, v, causal, p, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.p, ctx.scale, ctx.seed, ctx.offset = causal, p, scale, seed, offset
        return o

    @staticmethod
    def backward(ctx, do):  # type: ignore[override]
        q, k, v, o, lse = ctx.saved_tensors
        kern = native_or_none(do)
        dq, dk, dv = kern.attention_bwd(
            do.contiguous(), q, k, v, o, lse, ctx.causal, ctx.p, ctx.scale, ctx.seed, ctx.offset
        )
        return dq, dk, dv, None, None, None


def attention(
    q: Tensor, k: Tensor, v: Tensor, causal: bool = False, dropout_p: float = 0.0, training: bool = True,
    scale: Optional[float] = None,
) -> Tensor:
    p = float(dropout_p) if training else 0.0
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if not q.is_cuda:
        return attention_reference(q, k, v, causal, p, scale)
    kern = native_or_none(q)
    if not hasattr(kern, "attention_fwd"):
        # Bring-up only: the HIP flash kernel is not in this build yet.
        return F.scaled_dot_product_attention(q, k, v, dropout_p=p, is_causal=causal, scale=scale)
    return _FlashAttention.apply(q, k, v, bool(causal), p, scale)
