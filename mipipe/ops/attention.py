"""Scaled dot-product attention on the HIP flash-attention kernels
(csrc/kernels/attention.hip).

Two entry points:

* :func:`attention_packed` -- ``qkv [B, S, 3, H, D]`` (the QKV projection output
  viewed in place) -> ``o [B, S, H, D]``.  No transposes: the kernels read Q, K
  and V with strides and the backward writes one packed ``dqkv`` gradient.
* :func:`attention` -- the usual ``q, k, v [B, H, S, D]`` API (views are
  permuted, not copied).

Causal masking and attention dropout are supported; the dropout mask is
regenerated from Philox (seed, offset) in backward, so checkpoint recompute
replays it exactly.  Supported on the GPU path: bf16 with ``S % 64 == 0`` and
``D in {64, 128, 256}`` (attention.hip), fp32 with ``S % 32 == 0`` and
``D in {64, 128}`` (attention_f32.hip, the reference's own precision); the
CPU path is eager math.  Any smaller head dim (e.g. 32, 80, 96, 160) runs on
the kernels zero-padded to the next supported one (the scale stays that of the
real head dim; the padded columns are sliced off), and a non-causal sequence of
an unsupported length runs padded too when its head dim leaves a spare padded
feature to mask the padded keys with (bf16), or with the kernels' own key bound
(fp32: ``kv_len``, so the reference's fp32 D=64 tail window runs on the kernels;
``_run_shape``).  A CAUSAL sequence of any other length (the
reference's ``get_batch`` tail window, /root/reference/main.py:108-113) is
zero-padded at the end to the next supported length: under the causal mask
no real query sees a padded key, so the real rows are exact; the padded rows
are sliced off (and get no gradient).
"""
from __future__ import annotations

import math
import os
import threading
from collections import OrderedDict
from typing import Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor

from ..checkpoint import is_recomputing, recompute_expected
from ._util import kernels_for

__all__ = ["attention", "attention_packed", "attention_reference", "clear_keep_words"]


def attention_reference(q: Tensor, k: Tensor, v: Tensor, causal: bool, p: float, scale: Optional[float] = None) -> Tensor:
    """Eager fp32 math on ``[B, H, S, D]`` (CPU path and test oracle)."""
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


# Keep words across a checkpoint: the long-sequence forward (attention_long.hip) makes its dropout keep words
# inside the kernel (Philox in the loop: ~1.6x the forward's VALU work) and returns them for the backward.  A
# checkpoint's first, no-grad forward throws them away and its recompute makes the same words again from the
# same restored Philox draw.  Instead the first forward leaves them here, keyed by (device, seed, offset), and
# the recompute -- whose draw is that key again -- reads them (the kernel variant that loads the words).  The
# words are bit-identical either way (tests/test_gpu_kernels.py::test_attention_keep_words_reused_bit_exact).
# Bounded: at most MIPIPE_ATTN_KEEP_REUSE_GB (default 16) are held, oldest dropped first (a dropped entry is just
# made again), and only when that recompute will run (checkpoint.recompute_expected(): not for a training-mode
# forward under no_grad); MIPIPE_ATTN_KEEP_REUSE=0 turns it off.
_KEEP_REUSE = os.environ.get("MIPIPE_ATTN_KEEP_REUSE", "1") != "0"
_KEEP_LIMIT = int(float(os.environ.get("MIPIPE_ATTN_KEEP_REUSE_GB", "16")) * (1 << 30))
_keep_words: "OrderedDict[tuple, Tensor]" = OrderedDict()
_keep_bytes = 0
_keep_lock = threading.Lock()
keep_stats = {"stored": 0, "reused": 0}  # counters, for the tests


def _i64(x: int) -> int:
    return x - (1 << 64) if x >= (1 << 63) else x


def _next_draw(device: torch.device) -> tuple:
    """(device, seed, offset) the next Philox draw on ``device`` will return (the binding's int64 view)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    g = torch.cuda.default_generators[idx]
    return (idx, _i64(g.initial_seed()), g.get_offset())


def clear_keep_words() -> None:
    """Drops every held keep-word set (the engine calls it at the end of a step)."""
    global _keep_bytes
    with _keep_lock:
        _keep_words.clear()
        _keep_bytes = 0


def _attention_fwd(kern, q, k, v, causal, p, scale, kv_len):
    global _keep_bytes
    reuse = _KEEP_REUSE and p > 0 and q.is_cuda and q.dtype == torch.bfloat16 and kv_len == 0
    words = key = None
    if reuse and is_recomputing():
        key = _next_draw(q.device)
        with _keep_lock:
            words = _keep_words.pop(key, None)
            if words is not None:
                _keep_bytes -= words.numel() * 4
                keep_stats["reused"] += 1
    if words is not None:
        out = kern.attention_fwd(q, k, v, causal, p, scale, kv_len, words, key[1], key[2])
    else:
        out = kern.attention_fwd(q, k, v, causal, p, scale, kv_len)
    bits = out[4]
    if reuse and bits.numel() and recompute_expected() and not torch.is_grad_enabled():
        idx = q.device.index if q.device.index is not None else torch.cuda.current_device()
        with _keep_lock:
            _keep_words[(idx, out[2], out[3])] = bits
            _keep_bytes += bits.numel() * 4
            keep_stats["stored"] += 1
            while _keep_bytes > _KEEP_LIMIT and _keep_words:
                _, old = _keep_words.popitem(last=False)
                _keep_bytes -= old.numel() * 4
    return out


class _AttentionPacked(torch.autograd.Function):
    """``qkv [B, S, 3, H, D]`` (contiguous) in, ``o [B, S, H, D]`` out; the
    backward produces the packed ``dqkv`` in one buffer."""

    @staticmethod
    def forward(ctx, qkv, causal, p, scale, kv_len=0):  # type: ignore[override]
        kern = kernels_for(qkv)
        q, k, v = qkv.select(2, 0), qkv.select(2, 1), qkv.select(2, 2)
        o, lse, seed, offset, bits = _attention_fwd(kern, q, k, v, causal, p, scale, kv_len)
        ctx.save_for_backward(qkv, o, lse, bits)
        ctx.causal, ctx.p, ctx.scale, ctx.seed, ctx.offset, ctx.kv_len = causal, p, scale, seed, offset, kv_len
        return o

    @staticmethod
    def backward(ctx, do):  # type: ignore[override]
        qkv, o, lse, bits = ctx.saved_tensors
        kern = kernels_for(do)
        if do.stride() != o.stride():
            do = do.contiguous()
        dqkv = torch.empty_like(qkv)
        kern.attention_bwd(do, qkv.select(2, 0), qkv.select(2, 1), qkv.select(2, 2), o, lse, ctx.causal, ctx.p,
                           ctx.scale, ctx.seed, ctx.offset, dqkv.select(2, 0), dqkv.select(2, 1), dqkv.select(2, 2),
                           bits if bits.numel() else None, ctx.kv_len)
        return dqkv, None, None, None, None


class _Attention(torch.autograd.Function):
    """Separate q, k, v as [B, S, H, D] views sharing one layout."""

    @staticmethod
    def forward(ctx, q, k, v, causal, p, scale, kv_len=0):  # type: ignore[override]
        kern = kernels_for(q)
        o, lse, seed, offset, bits = _attention_fwd(kern, q, k, v, causal, p, scale, kv_len)
        ctx.save_for_backward(q, k, v, o, lse, bits)
        ctx.causal, ctx.p, ctx.scale, ctx.seed, ctx.offset, ctx.kv_len = causal, p, scale, seed, offset, kv_len
        return o

    @staticmethod
    def backward(ctx, do):  # type: ignore[override]
        q, k, v, o, lse, bits = ctx.saved_tensors
        kern = kernels_for(do)
        if do.stride() != o.stride():
            do = do.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        kern.attention_bwd(do, q, k, v, o, lse, ctx.causal, ctx.p, ctx.scale, ctx.seed, ctx.offset, dq, dk, dv,
                           bits if bits.numel() else None, ctx.kv_len)
        return dq, dk, dv, None, None, None, None


_noted = set()


def _note_math_path(S: int, D: int, dtype) -> None:
    """Shapes outside the kernels' tiling use the eager math path; say so once per shape."""
    key = (S, D, dtype)
    if key not in _noted:
        _noted.add(key)
        import warnings

        warnings.warn(f"mipipe attention: S={S} D={D} {dtype} runs the eager math path (HIP kernels: bf16 with "
                      "S % 64 == 0, D in {64, 128, 256}; fp32 with S % 32 == 0, D in {64, 128})", stacklevel=3)


def _gpu_ok(t: Tensor, S: int, D: int) -> bool:
    if t.dtype == torch.bfloat16:
        return kernels_for(t).attention_supported(S, D)
    if t.dtype == torch.float32:
        return kernels_for(t).attention_f32_supported(S, D)
    return False


def _causal_pad(t: Tensor, S: int, D: int) -> Optional[int]:
    """The padded length a causal sequence of S runs at on the kernels (None: none fits)."""
    step = 64 if t.dtype == torch.bfloat16 else 32
    for sp in (-(-S // step) * step, max(128, -(-S // step) * step)):
        if sp != S and _gpu_ok(t, sp, D):
            return sp
    return None


_KEY_MASK = -32768.0  # exact in bf16; times the query's 1 and any scale >= 2^-8: exp underflows to 0


def _run_shape(t: Tensor, S: int, D: int, causal: bool, scale: float) -> Optional[Tuple[int, int, int]]:
    """(sequence length, head dim, key bound) the kernels run a (S, D) attention
    at, or None (eager path).  The key bound (``kv_len``, 0 = none) is set for a
    non-causal fp32 sequence padded at the end: the fp32 kernels mask keys past
    it themselves.

    * A head dim the kernels do not tile is zero-padded to the next one they do: the
      padded features add 0 to every score (the softmax scale stays 1/sqrt(D) of the
      real head dim) and give output / gradient columns that are sliced off.
    * A causal sequence of an unsupported length is zero-padded at the end (see the
      module doc).
    * A non-causal one too, when a padded feature is free to mask the padded keys:
      feature D is 1 in every query, 0 in every real key and -32768 in every padded
      key, so a padded key scores -32768 * scale below any real one and gets weight 0
      (its V rows are 0 as well)."""
    dims = [D] + [d for d in ((64, 128, 256) if t.dtype == torch.bfloat16 else (64, 128)) if d > D]
    for dp in dims:
        if _gpu_ok(t, S, dp):
            return S, dp, 0
        if t.dtype == torch.float32 and not causal:  # key bound inside the kernel
            sp = _causal_pad(t, S, dp)
            if sp is not None:
                return sp, dp, S
            continue
        # the spare-feature key mask needs exp(-32768 * scale) to underflow to 0
        sp = _causal_pad(t, S, dp) if (causal or (dp > D and scale >= 2.0 ** -8)) else None
        if sp is not None:
            return sp, dp, 0
    return None


def attention_packed(qkv: Tensor, causal: bool = False, dropout_p: float = 0.0, training: bool = True,
                     scale: Optional[float] = None) -> Tensor:
    """``qkv [B, S, 3, H, D]`` -> ``o [B, S, H, D]``."""
    B, S, three, H, D = qkv.shape
    assert three == 3
    p = float(dropout_p) if training else 0.0
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(D)
    if qkv.is_cuda and _gpu_ok(qkv, S, D):
        return _AttentionPacked.apply(qkv.contiguous(), bool(causal), p, scale)
    run = _run_shape(qkv, S, D, bool(causal), scale) if qkv.is_cuda else None
    if run is not None:
        sp, dp, kv_len = run
        padded = F.pad(qkv, (0, dp - D, 0, 0, 0, 0, 0, sp - S))
        if kv_len:  # the kernel masks keys >= S itself
            return _AttentionPacked.apply(padded, bool(causal), p, scale, kv_len)[:, :S, :, :D]
        if sp != S and not causal:  # mask the padded keys through the spare feature D
            # [B, S, 3, H, D]: index (b, s, which, h, d) -> q = which 0, k = which 1, sequence dim 1
            c = torch.zeros_like(padded)
            c[:, :, 0, :, D] = 1.0
            c[:, S:, 1, :, D] = _KEY_MASK
            padded = padded + c
        return _AttentionPacked.apply(padded, bool(causal), p, scale)[:, :S, :, :D]
    q, k, v = qkv.select(2, 0), qkv.select(2, 1), qkv.select(2, 2)
    if qkv.is_cuda:
        _note_math_path(S, D, qkv.dtype)
    o = attention_reference(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), causal, p, scale)
    return o.transpose(1, 2)


def attention(
    q: Tensor, k: Tensor, v: Tensor, causal: bool = False, dropout_p: float = 0.0, training: bool = True,
    scale: Optional[float] = None,
) -> Tensor:
    """``q, k, v [B, H, S, D]`` -> ``[B, H, S, D]``."""
    p = float(dropout_p) if training else 0.0
    scale = float(scale) if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    if not q.is_cuda:
        return attention_reference(q, k, v, causal, p, scale)
    S, D = q.shape[2], q.shape[3]
    if not _gpu_ok(q, S, D):
        run = _run_shape(q, S, D, bool(causal), scale)
        if run is None:
            _note_math_path(S, D, q.dtype)
            return attention_reference(q, k, v, causal, p, scale)
        sp, dp, kv_len = run
        pad = lambda t: F.pad(t, (0, dp - D, 0, sp - S))  # noqa: E731
        qp, kp = pad(q), pad(k)
        if kv_len:  # the kernel masks keys >= S itself
            qs, ks, vs = (t.transpose(1, 2) for t in (qp, kp, pad(v)))
            qs, ks, vs = (t.contiguous() for t in (qs, ks, vs))
            return _Attention.apply(qs, ks, vs, bool(causal), p, scale, kv_len).transpose(1, 2)[:, :, :S, :D]
        if sp != S and not causal:  # mask the padded keys through the spare feature D ([B, H, S, D])
            cq, ck = torch.zeros_like(qp), torch.zeros_like(kp)
            cq[..., D] = 1.0
            ck[:, :, S:, D] = _KEY_MASK
            qp, kp = qp + cq, kp + ck
        return attention(qp, kp, pad(v), causal, dropout_p, training, scale)[:, :, :S, :D]
    qs, ks, vs = (t.transpose(1, 2) for t in (q, k, v))
    if not (qs.stride() == ks.stride() == vs.stride()) or qs.stride(3) != 1:
        qs, ks, vs = (t.contiguous() for t in (qs, ks, vs))
    o = _Attention.apply(qs, ks, vs, bool(causal), p, scale)
    return o.transpose(1, 2)
