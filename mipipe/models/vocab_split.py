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
from ..ops.linear import accumulable, accumulate_wgrad, gemm_operand, mark_gemm_weight

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


def _dgrad_into(k, tile: bool, d: Tensor, w: Tensor, res: Optional[Tensor], out: Tensor) -> None:
    """out = d . w (+ res), written in place (out may be a column slice)."""
    if tile:
        k.linear_dgrad(d, w, res, out)
    elif res is not None:
        out.copy_(torch.addmm(res, d, w))
    else:
        out.copy_(torch.mm(d, w))


def _bias_grad(k, d: Tensor, b: Tensor) -> Optional[Tensor]:
    main = accumulable(b)
    if main is not None:
        if k is not None:
            k.column_sum(d, main, True)
        else:
            main.add_(d.float().sum(0))
        return None
    if k is not None:
        return k.column_sum(d).to(b.dtype)
    return d.sum(0).to(b.dtype)


def _slot_words(t2: Tensor, e: int) -> Tensor:
    """The statistic slots of packed rows ``t2 = [h (e values) | slots]`` as a
    [rows, words] fp32 view -- no copy."""
    if t2.dtype == torch.float32:
        return t2[:, e:]
    return t2.view(torch.float32)[:, e * t2.element_size() // 4:]


def _targets(target: Tensor, device) -> Tensor:
    return target.reshape(-1).to(device=device, dtype=torch.int64).contiguous()


def _native(k, x2: Tensor) -> bool:
    """The HIP path: pack / statistics kernels move 16-byte row chunks."""
    es = x2.element_size()
    return k is not None and (x2.shape[1] * es) % 16 == 0 and (STAT_SLOTS * es) % 16 == 0


# ---------------------------------------------------------------- CPU (reference) path
def _stats_to_slots(a: Tensor, b: Tensor, dtype: torch.dtype) -> Tensor:
    buf = torch.zeros(a.shape[0], STAT_SLOTS, dtype=dtype, device=a.device)
    f = buf.view(torch.float32)
    f[:, 0] = a
    f[:, 1] = b
    return buf


def _softmax_grad(logits: Tensor, tgt: Tensor, lse: Tensor, g_row: Tensor, out: Tensor) -> None:
    """out[:, :V] = (exp(logits - lse) - onehot(tgt)) * g_row (tgt outside [0, V): no one-hot)."""
    p = torch.exp(logits.float() - lse[:, None])
    rows = torch.nonzero((tgt >= 0) & (tgt < logits.shape[1]))[:, 0]
    p[rows, tgt[rows]] -= 1.0
    out[:, : logits.shape[1]] = (p * g_row[:, None]).to(out.dtype)


class _HeadFn(torch.autograd.Function):
    """Forward: logits_a = x . w^T + b; out = [x | lse_a, logit_a[target]].
    On the GPU: the tile GEMM, then ONE kernel packing x and the statistics
    (``vsplit_head_fwd``).  Backward: one softmax-gradient kernel reading lse and
    dL/dloss_row straight from the message slots, the dgrad GEMM adding the
    incoming dx in its epilogue (residual read from the message in place)."""

    @staticmethod
    def forward(ctx, x, w, b, target):  # type: ignore[override]
        e = x.shape[-1]
        x2 = x.reshape(-1, e)
        k = kernels_for(x2) if x2.is_cuda else None
        t = _targets(target, x2.device)
        va = w.shape[0]
        ctx.native = _native(k, x2)
        if ctx.native:
            x2 = gemm_operand(x2)
            logits, tile = _tile_linear(k, x2, w, b)
            out = torch.empty(x2.shape[0], e + STAT_SLOTS, dtype=x2.dtype, device=x2.device)
            k.vsplit_head_fwd(logits, t, x2, out)
        else:
            logits, tile = _tile_linear(k, x2, w, b)
            lf = logits.float()
            lse = torch.logsumexp(lf, dim=-1)
            ta = torch.where((t >= 0) & (t < va), t, torch.zeros_like(t))
            tlog = torch.where((t >= 0) & (t < va), lf.gather(1, ta[:, None])[:, 0], torch.zeros_like(lse))
            out = torch.cat((x2, _stats_to_slots(lse, tlog, x2.dtype)), dim=-1)
        ctx.save_for_backward(x2, w, b, logits, t)
        ctx.tile, ctx.shape = tile, x.shape
        return out.view(*x.shape[:-1], e + STAT_SLOTS)

    @staticmethod
    def backward(ctx, dout):  # type: ignore[override]
        x2, w, b, logits, t = ctx.saved_tensors
        k = kernels_for(x2) if x2.is_cuda else None
        e = x2.shape[1]
        d2 = dout.reshape(-1, e + STAT_SLOTS)
        dlog = torch.empty_like(logits)
        dx = torch.empty(x2.shape, dtype=x2.dtype, device=x2.device)
        if ctx.native:
            d2 = gemm_operand(d2)
            words = _slot_words(d2, e)
            k.cross_entropy_bwd(logits, t, words[:, 0], None, -1, row_scale=words[:, 1], out=dlog)
        else:
            words = _slot_words(d2.contiguous(), e)
            _softmax_grad(logits, t, words[:, 0], words[:, 1], dlog)
        _dgrad_into(k, ctx.tile, dlog, w, d2[:, :e], dx)
        dw = accumulate_wgrad(dlog, x2, w)
        db = _bias_grad(k, dlog, b)
        return dx.view(ctx.shape), dw, db, None


class _TailFn(torch.autograd.Function):
    """Forward: logits_b over the padded tail rows, then ``vsplit_tail_fwd``:
    merged lse, row losses, the mean (a fixed-order one-block reduction) and the
    per-row weights valid / count.  Backward: one softmax-gradient kernel
    (scale = dL x weight, zeroed pad columns) that also writes (lse, dL/dloss_row)
    into the gradient message's slots; the dgrad GEMM writes dx into the same
    message -- no concatenation."""

    @staticmethod
    def forward(ctx, packed, w, b, target, va, vb, ignore_index):  # type: ignore[override]
        e = packed.shape[-1] - STAT_SLOTS
        p2 = packed.reshape(-1, e + STAT_SLOTS)
        k = kernels_for(p2) if p2.is_cuda else None
        t = _targets(target, p2.device)
        ctx.native = _native(k, p2[:, :e])
        if ctx.native:
            p2 = gemm_operand(p2)
            x2 = p2[:, :e]
            logits, tile = _tile_linear(k, x2, w, b)
            loss, lse, weight = k.vsplit_tail_fwd(logits[:, :vb], t, va, ignore_index, _slot_words(p2, e))
        else:
            x2 = p2[:, :e].contiguous()
            words = _slot_words(p2.contiguous(), e)
            lse_a, t_a = words[:, 0], words[:, 1]
            logits, tile = _tile_linear(k, x2, w, b)
            lf = logits[:, :vb].float()
            lse = torch.logaddexp(lse_a, torch.logsumexp(lf, dim=-1))
            in_b = (t >= va) & (t < va + vb)
            tb = torch.where(in_b, t - va, torch.zeros_like(t))
            tl = torch.where(in_b, lf.gather(1, tb[:, None])[:, 0], t_a)
            valid = ((t != ignore_index) & (t >= 0) & (t < va + vb)).to(torch.float32)
            count = valid.sum().clamp_min(1.0)
            loss = ((lse - tl) * valid).sum() / count
            weight = valid / count
        ctx.save_for_backward(x2, w, b, logits, t, lse, weight)
        ctx.tile, ctx.va, ctx.vb, ctx.ignore, ctx.shape = tile, va, vb, ignore_index, packed.shape
        return loss

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        x2, w, b, logits, t, lse, weight = ctx.saved_tensors
        k = kernels_for(x2) if x2.is_cuda else None
        e, vb = x2.shape[1], ctx.vb
        dpacked = torch.empty(x2.shape[0], e + STAT_SLOTS, dtype=x2.dtype, device=x2.device)
        dlog = torch.empty_like(logits)
        if ctx.native:
            gs = g.to(torch.float32).reshape(1)
            k.cross_entropy_bwd(logits[:, :vb], t, lse, gs, ctx.ignore, row_scale=weight, out=dlog, zero_pad=True,
                                t_offset=ctx.va, stat_out=dpacked[:, e:])
        else:
            g_row = weight * g.to(torch.float32)
            dlog[:, vb:] = 0  # padded vocabulary rows of the weight get no gradient
            _softmax_grad(logits[:, :vb], t - ctx.va, lse, g_row, dlog)
            dpacked[:, e:] = _stats_to_slots(lse, g_row, x2.dtype)
        _dgrad_into(k, ctx.tile, dlog, w, None, dpacked[:, :e])
        dw = accumulate_wgrad(dlog, x2, w)
        db = _bias_grad(k, dlog, b)
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
