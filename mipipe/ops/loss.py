"""Fused cross-entropy (kernel: csrc/kernels/loss.hip).

``cross_entropy(logits [N, V], target [N])`` with mean reduction over
non-ignored targets, like ``nn.CrossEntropyLoss()``.  No log-probabilities are
materialised; the backward scale ``dL / n_valid`` stays on the device.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import Tensor

from ._util import native_or_none

__all__ = ["cross_entropy"]


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):  # type: ignore[override]
        k = native_or_none(logits)
        lc = logits if (logits.dim() == 2 and logits.stride(1) == 1) else logits.contiguous()
        loss_rows, lse = k.cross_entropy_fwd(lc, target.contiguous(), ignore_index)
        count = (target != ignore_index).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(lc, target, lse, count)
        ctx.ignore_index = ignore_index
        return loss_rows.sum() / count

    @staticmethod
    def backward(ctx, dloss):  # type: ignore[override]
        logits, target, lse, count = ctx.saved_tensors
        k = native_or_none(logits)
        scale = (dloss.to(torch.float32) / count).reshape(1).contiguous()
        return k.cross_entropy_bwd(logits, target, lse, scale, ctx.ignore_index), None, None


def _rows_uniform(t: Tensor) -> bool:
    """True if all leading dims collapse to one row stride (e.g. a [B, S, :V] slice of [B, S, Vpad])."""
    stride = t.stride(-2)
    expect = stride
    for size, st in zip(reversed(t.shape[:-1]), reversed(t.stride()[:-1])):
        if size != 1 and st != expect:
            return False
        expect = st * size
    return True


def cross_entropy(logits: Tensor, target: Tensor, ignore_index: int = -100) -> Tensor:
    if logits.dim() != 2:
        # keeps a padded-vocabulary view strided (no copy)
        lead = logits.shape[:-1].numel()
        logits = logits.as_strided((lead, logits.shape[-1]), (logits.stride(-2), 1)) \
            if logits.stride(-1) == 1 and _rows_uniform(logits) else logits.reshape(-1, logits.shape[-1])
    target = target.reshape(-1)
    if not logits.is_cuda:
        return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)
    return _CrossEntropy.apply(logits, target, int(ignore_index))
