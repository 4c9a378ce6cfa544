"""Fused cross-entropy (kernel: csrc/kernels/loss.hip).

``cross_entropy(logits [N, V], target [N])`` with mean reduction over
non-ignored targets, like ``nn.CrossEntropyLoss()``.  No log-probabilities are
materialised; the backward scale ``dL / n_valid`` stays on the device.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import Tensor

from ._util import kernels_for

__all__ = ["cross_entropy", "mark_zero_padded", "take_zero_padded"]

# data_ptr -> padded width of gradient buffers whose pad columns are zero,
# written by the cross-entropy backward and consumed (once) by the Decoder's
# vocabulary-slice backward.  Entries are ints, never tensors.
_ZERO_PADDED = {}


def mark_zero_padded(buf: Tensor) -> None:
    if len(_ZERO_PADDED) > 64:  # stale entries (a graph that never reached the slice)
        _ZERO_PADDED.clear()
    _ZERO_PADDED[buf.data_ptr()] = (buf.shape[-1], buf.untyped_storage().nbytes())


def take_zero_padded(g: Tensor, width: int) -> bool:
    """True if ``g`` is the ``[..., :V]`` view of a zero-padded gradient buffer
    of row width ``width`` (and forgets the buffer)."""
    ent = _ZERO_PADDED.get(g.data_ptr())
    if ent is None or ent[0] != width or g.stride(-1) != 1 or g.storage_offset() != 0:
        return False
    rows = g.numel() // g.shape[-1] if g.shape[-1] else 0
    if g.stride(-2) != width or ent[1] < rows * width * g.element_size():
        return False
    del _ZERO_PADDED[g.data_ptr()]
    return True


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):  # type: ignore[override]
        _ZERO_PADDED.clear()  # marks live from a CE backward to the slice backward of the same pass
        k = kernels_for(logits)
        lc = logits if (logits.dim() == 2 and logits.stride(1) == 1) else logits.contiguous()
        target = target.contiguous()
        # row losses, then a one-block masked mean: loss and the per-row weights
        # valid / count (the backward's row scale) with no ATen reductions
        loss, lse, weight = k.cross_entropy_mean_fwd(lc, target, ignore_index)
        ctx.save_for_backward(lc, target, lse, weight)
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, dloss):  # type: ignore[override]
        logits, target, lse, weight = ctx.saved_tensors
        k = kernels_for(logits)
        scale = dloss.to(torch.float32).reshape(1)  # x weight[row] in the kernel
        n, v = logits.shape
        ld = logits.stride(0)
        if ld > v:
            # Rows of a padded-vocabulary buffer (the Decoder's [..., :V] view):
            # the gradient gets the same padded geometry, zeros in the pad, so
            # its rows are 16-byte aligned (vector path) and the Decoder's
            # slice backward can hand the padded buffer on without a copy.
            buf = torch.empty((n, ld), dtype=logits.dtype, device=logits.device)
            k.cross_entropy_bwd(logits, target, lse, scale, ctx.ignore_index, weight, buf, True)
            mark_zero_padded(buf)
            return buf[:, :v], None, None
        return k.cross_entropy_bwd(logits, target, lse, scale, ctx.ignore_index, weight), None, None


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
