"""Vocabulary-split LM head: the decoder GEMM + cross-entropy as TWO pipeline units.

The reference LM's decoder (``main.py:42-55``; E x V = 4096 x 28,782 in the
benchmark config) is one indivisible block worth ~1.2 transformer layers, so
with 8 pipeline stages -- and especially with two model chunks per rank -- the
stage holding it sets the pace.  Here it is cut along the vocabulary:

* :class:`DecoderHead` (virtual stage k) computes logits for vocabulary rows
  ``[0, va)``, their log-sum-exp ``lse_a`` and, where a token's target falls in
  that range, the target logit, and forwards ``[h | lse_a, t_a]`` (the two
  fp32 statistics ride in 8 extra activation slots, bit-cast);
* :class:`DecoderTail` (virtual stage k+1) computes logits for ``[va, V)``,
  combines ``lse = logaddexp(lse_a, lse_b)`` and returns the mean
  cross-entropy -- exactly the unsplit loss.

Backward is exact as well: the tail's gradient message back to the head
carries, in the same 8 slots, the global ``lse`` and the per-row loss
gradient, from which the head forms ``dlogits_a = (exp(l_a - lse) - onehot)
* g`` -- the same rows of the full softmax gradient.  No logits cross the link:
per token the boundary carries E + 8 values instead of E.

Both units need the targets (``wants_target``); the tail computes the loss
itself (``fused_loss``) -- see :class:`mipipe.parallel.engine.PipelineEngine`.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor, nn

from ..ops._util import kernels_for
from ..ops.linear import accumulable, accumulate_wgrad, mark_gemm_weight

__all__ = ["DecoderHead", "DecoderTail", "split_point", "split_decoder", "STAT_SLOTS"]

STAT_SLOTS = 8  # extra activation elements per token carrying fp32 (lse, target-logit) / (lse, grad)


def split_point(ntoken: int, pad_to: int = 256) -> int:
    """Head vocabulary size: half the vocabulary rounded up to the GEMM tile."""
    return min(ntoken, (ntoken // 2 + pad_to - 1) // pad_to * pad_to)


def _tile_linear(k, x2: Tensor, w: Tensor, b: Tensor) -> Tuple[Tensor, bool]:
    tile = (k is not None and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and k.gemm_supported(x2.shape[0], w.shape[0], w.shape[1])
            and k.gemm_supported(x2.shape[0], w.shape[1], w.shape[0]))
    if tile:
        return k.linear_fwd(x2, w, b, 0, 0.0, False)[0], True
    return torch.addmm(b, x2, w.t()), False


def _dgrad(k, tile: bool, d: Tensor, w: Tensor) -> Tensor:
    return k.linear_dgrad(d, w) if tile else torch.matmul(d, w)


def _bias_grad(k, d: Tensor, b: Tensor) -> Optional[Tensor]:
    main = accumulable(b)
    if main is not None:
        if k is not None:
            k.column_sum(d, main, True)
        else:
            main.add_(d.float().sum(0))
        return None
    return d.sum(0).to(b.dtype)


def _lse_and_target(k, logits: Tensor, tgt: Tensor) -> Tuple[Tensor, Tensor]:
    """Row log-sum-exp and the logit at ``tgt`` (rows with tgt < 0: undefined)."""
    if k is not None:
        loss_rows, lse = k.cross_entropy_fwd(logits, tgt, -1)
        return lse, lse - loss_rows
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    return lse, lf.gather(1, tgt.clamp(min=0)[:, None])[:, 0]


def _softmax_grad(k, logits: Tensor, tgt: Tensor, lse: Tensor, g_row: Tensor, out: Tensor) -> Tensor:
    """out[:, :V] = (exp(logits - lse) - onehot(tgt)) * g_row (tgt < 0: no one-hot)."""
    if k is not None:
        return k.cross_entropy_bwd(logits, tgt, lse, None, -1, row_scale=g_row, out=out)
    p = torch.exp(logits.float() - lse[:, None])
    rows = torch.nonzero(tgt >= 0)[:, 0]
    p[rows, tgt[rows]] -= 1.0
    out[:, : logits.shape[1]] = (p * g_row[:, None]).to(out.dtype)
    return out


def _stats_to_slots(a: Tensor, b: Tensor, dtype: torch.dtype) -> Tensor:
    buf = torch.zeros(a.shape[0], STAT_SLOTS, dtype=dtype, device=a.device)
    f = buf.view(torch.float32)
    f[:, 0] = a
    f[:, 1] = b
    return buf


def _slots_to_stats(slots: Tensor) -> Tuple[Tensor, Tensor]:
    f = slots.contiguous().view(torch.float32)
    return f[:, 0].contiguous(), f[:, 1].contiguous()


class _HeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, target):  # type: ignore[override]
        k = kernels_for(x) if x.is_cuda else None
        e = x.shape[-1]
        x2 = x.reshape(-1, e).contiguous()
        logits, tile = _tile_linear(k, x2, w, b)
        t = target.reshape(-1).to(x2.device)
        va = w.shape[0]
        ta = torch.where((t >= 0) & (t < va), t, torch.full_like(t, -1)).contiguous()
        lse, tlog = _lse_and_target(k, logits, ta)
        out = torch.cat((x2, _stats_to_slots(lse, tlog, x2.dtype)), dim=-1)
        ctx.save_for_backward(x2, w, b, logits, ta)
        ctx.tile, ctx.shape = tile, x.shape
        return out.view(*x.shape[:-1], e + STAT_SLOTS)

    @staticmethod
    def backward(ctx, dout):  # type: ignore[override]
        x2, w, b, logits, ta = ctx.saved_tensors
        k = kernels_for(x2) if x2.is_cuda else None
        e = x2.shape[1]
        d2 = dout.reshape(-1, e + STAT_SLOTS)
        lse, g_row = _slots_to_stats(d2[:, e:])
        dlog = torch.empty_like(logits)
        _softmax_grad(k, logits, ta, lse, g_row, dlog)
        dx = d2[:, :e] + _dgrad(k, ctx.tile, dlog, w)
        dw = accumulate_wgrad(dlog, x2, w)
        db = _bias_grad(k, dlog, b)
        return dx.view(ctx.shape), dw, db, None


class _TailFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, packed, w, b, target, va, vb, ignore_index):  # type: ignore[override]
        k = kernels_for(packed) if packed.is_cuda else None
        e = packed.shape[-1] - STAT_SLOTS
        p2 = packed.reshape(-1, e + STAT_SLOTS)
        x2 = p2[:, :e].contiguous()
        lse_a, t_a = _slots_to_stats(p2[:, e:])
        logits, tile = _tile_linear(k, x2, w, b)
        lv = logits[:, :vb]
        t = target.reshape(-1).to(x2.device)
        in_b = (t >= va) & (t < va + vb)
        tb = torch.where(in_b, t - va, torch.full_like(t, -1)).contiguous()
        lse_b, t_b = _lse_and_target(k, lv, tb)
        lse = torch.logaddexp(lse_a, lse_b)
        tl = torch.where(in_b, t_b, t_a)
        valid = (t != ignore_index) & (t >= 0) & (t < va + vb)
        count = valid.sum().clamp_min(1).to(torch.float32)
        loss = ((lse - tl) * valid).sum() / count
        ctx.save_for_backward(x2, w, b, logits, tb, lse, valid, count)
        ctx.tile, ctx.vb, ctx.shape = tile, vb, packed.shape
        return loss

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        x2, w, b, logits, tb, lse, valid, count = ctx.saved_tensors
        k = kernels_for(x2) if x2.is_cuda else None
        g_row = (valid.to(torch.float32) * (g.to(torch.float32) / count)).contiguous()
        dlog = torch.zeros_like(logits)  # padded vocabulary columns stay zero
        _softmax_grad(k, logits[:, : ctx.vb], tb, lse, g_row, dlog)
        dx = _dgrad(k, ctx.tile, dlog, w)
        dw = accumulate_wgrad(dlog, x2, w)
        db = _bias_grad(k, dlog, b)
        dpacked = torch.cat((dx.to(x2.dtype), _stats_to_slots(lse, g_row, x2.dtype)), dim=-1)
        return dpacked.view(ctx.shape), dw, db, None, None, None, None


class DecoderHead(nn.Module):
    """Vocabulary rows ``[0, va)`` of the decoder; forwards ``[h | lse_a, t_a]``."""

    wants_target = True

    def __init__(self, ntoken: int, d_model: int, va: int, *, device=None, dtype=None) -> None:
        super().__init__()
        self.ntoken, self.va = ntoken, va
        self.weight = mark_gemm_weight(nn.Parameter(torch.empty(va, d_model, device=device, dtype=dtype)))
        self.bias = nn.Parameter(torch.zeros(va, device=device, dtype=dtype))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        with torch.no_grad():
            nn.init.uniform_(self.weight, -0.1, 0.1)  # main.py:47-50
            nn.init.zeros_(self.bias)

    def forward(self, x: Tensor, target: Tensor) -> Tensor:
        return _HeadFn.apply(x, self.weight, self.bias, target)

    def flops_per_token(self, seq_len: int) -> float:
        return 2.0 * self.weight.shape[0] * self.weight.shape[1]


class DecoderTail(nn.Module):
    """Vocabulary rows ``[va, V)`` (padded to the GEMM tile); returns the mean loss."""

    wants_target = True
    fused_loss = True

    def __init__(self, ntoken: int, d_model: int, va: int, *, pad_to: int = 256, ignore_index: int = -100,
                 device=None, dtype=None) -> None:
        super().__init__()
        self.ntoken, self.va, self.vb = ntoken, va, ntoken - va
        self.padded = (self.vb + pad_to - 1) // pad_to * pad_to
        self.ignore_index = ignore_index
        self.weight = mark_gemm_weight(nn.Parameter(torch.empty(self.padded, d_model, device=device, dtype=dtype)))
        self.bias = nn.Parameter(torch.zeros(self.padded, device=device, dtype=dtype))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        with torch.no_grad():
            nn.init.uniform_(self.weight, -0.1, 0.1)
            self.weight[self.vb:].zero_()
            nn.init.zeros_(self.bias)

    def forward(self, packed: Tensor, target: Tensor) -> Tensor:
        return _TailFn.apply(packed, self.weight, self.bias, target, self.va, self.vb, self.ignore_index)

    def flops_per_token(self, seq_len: int) -> float:
        return 2.0 * self.weight.shape[0] * self.weight.shape[1]


def split_decoder(dec: nn.Module) -> Tuple[DecoderHead, DecoderTail]:
    """Head/tail holding copies of a :class:`~mipipe.models.lm.Decoder`'s rows."""
    v, e = dec.ntoken, dec.weight.shape[1]
    va = split_point(v)
    fk = {"device": dec.weight.device, "dtype": dec.weight.dtype}
    head = DecoderHead(v, e, va, **fk)
    tail = DecoderTail(v, e, va, **fk)
    if dec.weight.device.type != "meta":
        with torch.no_grad():
            head.weight.copy_(dec.weight[:va])
            head.bias.copy_(dec.bias[:va])
            tail.weight.zero_()
            tail.bias.zero_()
            tail.weight[: v - va].copy_(dec.weight[va:v])
            tail.bias[: v - va].copy_(dec.bias[va:v])
    return head, tail
