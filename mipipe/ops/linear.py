"""Linear layers on the MFMA GEMM (csrc/kernels/gemm.hip) with fused epilogues.

Forward:  ``y = dropout(act(x @ W^T + b))`` -- one GEMM launch; bias,
          activation and dropout live in the epilogue (GELU also writes its
          pre-activation for backward).
Backward: the activation/dropout backward is one elementwise pass
          (csrc/kernels/elementwise.hip, same Philox mask layout as the
          epilogue) that also yields ``db``; then ``dx = dpre @ W`` (GEMM with a
          transposing LDS read of W) and ``dW += dpre^T @ x`` accumulated in
          fp32 straight into ``weight.main_grad`` when the flat optimizer owns
          the parameter, so micro-batch accumulation never rounds to bf16.

bf16 runs the v_mfma_f32_16x16x32_bf16 kernel (gemm.hip), fp32 -- the
reference's own precision -- the v_mfma_f32_32x32x2_f32 kernel (gemm_f32.hip)
with the same epilogues and main_grad path.  Only shapes neither kernel covers
(e.g. a width that is not a multiple of 8 / 4) run the plain GEMM through
torch.matmul with the same fused elementwise kernels.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.nn.functional as F
from torch import Tensor

from ._util import kernels_for
from .activation import ACTIVATIONS, bias_act_reference

__all__ = ["linear", "linear_fanout", "deferred_wgrad", "flush_wgrad", "accumulate_wgrad", "mark_gemm_weight"]


def mark_gemm_weight(p: Tensor) -> Tensor:
    """Tags a weight whose gradient only this module's GEMMs write.  The flat
    optimizer then skips zero-filling its ``main_grad`` in ``zero_grad`` and
    the first weight-gradient GEMM of the step OVERWRITES it (plain fp32
    stores, no read-modify-write); see :func:`_claim`."""
    p._mipipe_gemm_weight = True  # type: ignore[attr-defined]
    return p


def _claim(p: Tensor) -> bool:
    """Whether the next gradient write into ``p.main_grad`` must accumulate:
    False exactly once after a lazy ``FlatAdam.zero_grad`` (the buffer holds
    stale values then, and the first writer overwrites it)."""
    if getattr(p, "_mg_fresh", False):
        p._mg_fresh = False  # type: ignore[attr-defined]
        return False
    return True


def accumulable(p: Tensor) -> Optional[Tensor]:
    """``p.main_grad`` ready for ACCUMULATING writers (atomics, += epilogues):
    a lazily-zeroed buffer is zero-filled first (a tagged weight reached by a
    writer that cannot overwrite, e.g. a tied embedding)."""
    main = getattr(p, "main_grad", None)
    if main is not None and not _claim(p):
        main.zero_()
    return main


def _add_or_copy(main: Tensor, g: Tensor, p: Tensor) -> None:
    if _claim(p):
        main.add_(g.float())
    else:
        main.copy_(g)


def _gemm_supported(k, dtype: torch.dtype, m: int, n: int, kk: int) -> bool:
    if dtype == torch.bfloat16:
        return k.gemm_supported(m, n, kk)
    if dtype == torch.float32:
        return k.gemm_f32_supported(m, n, kk)
    return False


def _aligned(t: Tensor) -> bool:
    """The GEMM moves operands, addends and outputs in 16-byte chunks."""
    return t.data_ptr() % 16 == 0


def gemm_operand(t: Tensor) -> Tensor:
    """``t`` itself when the tile GEMMs can read it in place -- 2-D, unit column
    stride, 16-byte aligned rows (a column slice of a packed message is fine) --
    else an aligned contiguous copy."""
    if (t.dim() == 2 and t.stride(1) == 1 and (t.stride(0) * t.element_size()) % 16 == 0
            and t.stride(0) >= t.shape[1] and _aligned(t)):
        return t
    t = t.contiguous()
    return t if _aligned(t) else t.clone()


def _tile_ok(k, x2: Tensor, weight: Tensor) -> bool:
    """All three GEMMs of the layer (fwd [T,N,K], dgrad [T,K,N], wgrad [N,K,T]) fit the tile kernel."""
    t, (n, kk) = x2.shape[0], weight.shape
    dt = x2.dtype
    return (
        weight.dtype == dt
        and _aligned(x2)
        and _aligned(weight)
        and _gemm_supported(k, dt, t, n, kk)
        and _gemm_supported(k, dt, t, kk, n)
        and _gemm_supported(k, dt, n, kk, t)
    )


class ActFold:
    """Hand-off between an activation layer ``h = drop(act(x W1^T + b1))`` and
    the ONE layer consuming ``h`` (an MLP's two halves): the consumer's dgrad
    GEMM applies the activation's backward (act' of the saved tensor and the
    dropout mask) in its epilogue, so the producer's backward receives the
    gradient of its pre-activation and skips its own elementwise pass -- one
    write and one read of the [tokens, d_ff] gradient fewer, and no separate
    kernel.  Only valid when ``h`` has no other consumer: the caller (e.g.
    :class:`~mipipe.models.transformer.FeedForwardBlock`) guarantees that; the
    producer checks it receives exactly the tensor the consumer produced.
    """

    __slots__ = ("act", "saved", "p", "seed", "offset", "grad", "version")

    def __init__(self) -> None:
        self.act, self.saved, self.p, self.seed, self.offset = 0, None, 0.0, 0, 0
        # the folded gradient the consumer produced, and its version: the
        # producer accepts only this tensor, unmodified (autograd accumulates a
        # second consumer's gradient in place or into a new tensor)
        self.grad: Optional[Tensor] = None
        self.version = 0

    def done(self, grad: Tensor) -> None:
        self.grad, self.version = grad, grad._version

    def take(self, d2: Tensor) -> bool:
        """True if ``d2`` is the folded gradient (then consumed); raises if a
        fold happened but the gradient reaching the producer is another tensor."""
        g, self.grad = self.grad, None
        if g is None:
            return False
        if d2.data_ptr() != g.data_ptr() or g._version != self.version:
            raise RuntimeError("mipipe: an activation's backward was folded into its consumer's dgrad, but the "
                               "gradient reaching the activation is a different tensor (the activation output "
                               "has another consumer): do not pass one ActFold to such a graph")
        return True

    def offer(self, act: int, saved: Tensor, p: float, seed: int, offset: int) -> None:
        self.act, self.saved, self.p, self.seed, self.offset = act, saved, p, seed, offset

    def release(self) -> None:
        """Drops the offered tensor (the consumer took its own reference, or none came)."""
        self.saved = None

    def ready_for(self, x2: Tensor) -> bool:
        s = self.saved
        if s is None or x2.dtype != torch.bfloat16:
            return False
        if self.act == KACT_RELU_BITS:  # the output's nonzeros as bits, [rows, cols / 8]
            return s.dtype == torch.uint8 and tuple(s.shape) == (x2.shape[0], x2.shape[1] // 8)
        return s.shape == x2.shape and s.dtype == x2.dtype


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act, p, fanout=False, res=None, fold_out=None,
                fold_in=None, save=True):  # type: ignore[override]
        ctx.set_materialize_grads(False)
        k = kernels_for(x)
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        w = weight.contiguous()
        fused_tile = _tile_ok(k, x2, w)
        seed = offset = 0
        preact = xt = None
        saved_act = act  # the activation code the backward applies to the saved tensor
        ctx.has_res = res is not None
        if fused_tile:
            r2 = None
            if res is not None:
                r2 = res.reshape(-1, w.shape[0])
                if r2.dtype != x2.dtype or not r2.is_contiguous() or not _aligned(r2):
                    r2 = r2.to(x2.dtype).contiguous()
                    if not _aligned(r2):
                        r2 = r2.clone()
            # x^T for the transposed weight-gradient GEMM, written by this GEMM
            # (GemmArgs::at): only when a backward will want this weight's
            # gradient in a flat-optimizer main_grad
            if (save and _EMIT_XT and x2.dtype == torch.bfloat16 and ctx.needs_input_grad[1]
                    and getattr(weight, "main_grad", None) is not None and k.gemm_emit_ok(act, p, act == 2)):
                xt = torch.empty((x2.shape[1], x2.shape[0]), dtype=x2.dtype, device=x2.device)
            # GELU's saved tensor is written only for a backward (not under no_grad):
            # GELU'(pre) itself on the bf16 path (aux_grad), so the backward --
            # a separate pass or the consumer's dgrad epilogue -- is one multiply
            aux_grad = _GELU_SAVE_GRAD and act == 2 and save and x2.dtype == torch.bfloat16
            # ReLU (+ dropout) folded into the consumer's dgrad: hand it the output's nonzeros as bits (1/16 of
            # the bytes its epilogue would re-read from the bf16 output; profiles/gemm_roofline_r6.txt)
            bits = None
            if (fold_out is not None and act == 1 and p > 0.0 and save and _RELU_BITS and x2.dtype == torch.bfloat16
                    and k.linear_bits_ok(x2.shape[0], w.shape[0], x2.shape[1], act, p)):
                bits = torch.empty((x2.shape[0], w.shape[0] // 8), dtype=torch.uint8, device=x2.device)
            y, preact, seed, offset = k.linear_fwd(x2, w, bias, act, p, act == 2 and save, r2, xt, aux_grad, bits)
            if aux_grad:
                saved_act = KACT_SAVED_GRAD
            res = None  # added in the epilogue
        else:
            bits = None
            y = torch.matmul(x2, w.t())
            if act != 0 or p > 0.0 or bias is not None:
                pre_bias = y
                y, seed, offset = k.bias_act_fwd(y.contiguous(), bias, act, p)
                if act == 2:
                    preact = pre_bias  # pre-BIAS; backward adds the bias back
        saved = preact if act == 2 else (y if act == 1 else None)
        # activation backward folded into the consumer's dgrad (ActFold): the
        # producer's saved tensor is ALSO saved here, through save_for_backward
        # (released after this backward, seen by saved-tensor hooks), never
        # held by the hand-off object itself
        ctx.fold_out = ctx.fold_in = None
        fold_saved = None
        if fold_out is not None and fused_tile and act != 0 and x2.dtype == torch.bfloat16 and saved is not None:
            if bits is not None:
                fold_out.offer(KACT_RELU_BITS, bits, p, seed, offset)
            else:
                fold_out.offer(saved_act, saved, p, seed, offset)
            ctx.fold_out = fold_out
        if fold_in is not None and fused_tile and fold_in.ready_for(x2) and ctx.needs_input_grad[0]:
            ctx.fold_in = fold_in
            ctx.fold_args = (fold_in.act, fold_in.p, fold_in.seed, fold_in.offset)
            fold_saved = fold_in.saved
        if fold_in is not None:
            fold_in.saved = None
        # x is kept for the weight gradient only: x^T replaces it when written
        ctx.x_is_t = xt is not None
        ctx.save_for_backward(xt if xt is not None else x2, w, bias, saved, fold_saved)
        ctx.act, ctx.p, ctx.seed, ctx.offset = saved_act, p, seed, offset
        ctx.fused_tile = fused_tile
        ctx.in_shape = shape
        y = y.view(*shape[:-1], w.shape[0])
        if res is not None:
            y = y + res
        if fanout:
            # the input again, for its other consumer: its gradient comes back
            # to this node and is added in the dgrad GEMM's epilogue
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dres=None):  # type: ignore[override]
        x2, w, bias, saved, fold_saved = ctx.saved_tensors
        dres_in = dy if ctx.has_res else None  # y = res + f(x): the residual input's gradient is dy
        if dy is None:  # only the fan-out branch carries a gradient
            return dres, None, None, None, None, None, None, None, None, None
        k = kernels_for(dy)
        d2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        if ctx.fused_tile and not _aligned(d2):
            d2 = d2.clone()  # a misaligned contiguous view: the tile GEMMs move 16-byte chunks
        need_db = bias is not None and ctx.needs_input_grad[2]
        main_b = accumulable(bias) if need_db else None
        # inside deferred_wgrad(): the bias gradient joins the step's batch too
        defer_b = main_b is not None and _DEFERRED is not None and d2.shape[-1] % 8 == 0
        act, p = ctx.act, ctx.p
        if ctx.fold_out is not None and ctx.fold_out.take(d2):
            act, p = 0, 0.0  # d2 is already the pre-activation gradient
        if act != 0 or p > 0.0:
            # GEMM-saved GELU pre-activation already includes the bias.
            bias_for_bwd = None if ctx.fused_tile else bias
            dpre, db = k.bias_act_bwd(d2, saved if saved is not None else d2, bias_for_bwd, act, p,
                                      ctx.seed, ctx.offset, need_db and not defer_b, None if defer_b else main_b)
        else:
            dpre = d2
            db = None
            if defer_b:
                pass
            elif main_b is not None:
                k.column_sum(d2, main_b, True)  # fp32 main_grad += colsum(dy)
            elif need_db:
                db = k.column_sum(d2)
        if defer_b:
            _defer_bias(bias, dpre)

        dx = None
        if ctx.needs_input_grad[0]:
            r2 = None
            if dres is not None:
                r2 = dres.reshape(-1, dres.shape[-1])
                if not (ctx.fused_tile and r2.dtype == dpre.dtype and r2.is_contiguous() and _aligned(r2)):
                    r2 = None
            fin = ctx.fold_in
            if ctx.fused_tile and fin is not None and r2 is None and dres is None:
                f_act, f_p, f_seed, f_offset = ctx.fold_args
                dx = k.linear_dgrad(dpre, w, None, None, f_act, fold_saved, f_p, f_seed, f_offset)
                fin.done(dx)
            elif ctx.fused_tile:
                dx = k.linear_dgrad(dpre, w, r2)
            else:
                dx = torch.matmul(dpre, w)
            dx = dx.view(ctx.in_shape)
            if dres is not None and r2 is None:
                dx = dx + dres

        dw = None
        if ctx.needs_input_grad[1] and ctx.x_is_t:  # x2 holds x^T [K, T]
            if _DEFERRED is not None:
                _defer(w, dpre, x2, True)
            else:
                k.linear_wgrad_xt_segments([dpre], [x2], w.main_grad, _claim(w))
        elif ctx.needs_input_grad[1]:
            main = getattr(w, "main_grad", None)
            if main is not None and ctx.fused_tile and _DEFERRED is not None:
                _defer(w, dpre, x2)
            elif main is not None and ctx.fused_tile:
                k.linear_wgrad(dpre, x2, main, _claim(w))
            elif main is not None:
                _add_or_copy(main, torch.matmul(dpre.t(), x2), w)
            else:
                dw = torch.matmul(dpre.t(), x2)
        return dx, dw, db, None, None, None, dres_in, None, None, None


# ---------------------------------------------------------------- deferred wgrad
# Zero-bubble style split of the linear backward: inside ``deferred_wgrad()``
# the backward computes only dX (and the bias gradient) -- what the upstream
# pipeline stage waits for -- and queues (dY, X) per weight; ``flush_wgrad()``
# then runs ONE K-segmented GEMM per weight over all queued micro-batches
# (``linear_wgrad_segments``).  A pipeline rank thereby sends its input
# gradients (n-1) weight-gradient times earlier in the drain, and the fp32
# main_grad read-modify-write happens once per step instead of once per
# micro-batch.  Module-level (not thread-local): autograd runs backward on its
# own device threads.
_DEFERRED: Optional[dict] = None
# Bias gradients folded into the weight-gradient GEMMs of the flush
# (MIPIPE_FUSE_BIAS=0: separate column-sum kernels, for A/B runs).
_FUSE_BIAS = os.environ.get("MIPIPE_FUSE_BIAS", "1") != "0"
# Where the K-contiguous x^T of the transposed weight-gradient GEMM
# (C^T = X^T . dY, ~15 % faster than reading both operands I-contiguous:
# profiles/wgrad_layout_probe.txt) comes from -- MIPIPE_WGRAD_XT:
#   auto (default): the flush transposes x (transpose_b16, a streaming kernel)
#        for weights with more than 4608 output features, where the GEMM
#        saving outgrows the transpose (~N_out / 3600 x its cost) -- and the
#        bias gradient folds into the GEMM (split-K grids included) instead of
#        a column-sum pass over dY.  Measured: GPT-2-XL's qkv (4800 outputs)
#        +0.5 % on the step, every weight (1600 outputs too) -1.4 %
#        (tools/gpu_runs/r6_g11.sh); enc12's 4096-wide weights stay I-contiguous;
#   emit: the forward GEMM writes x^T from its staged A tiles (every tile-path
#        linear; +x^T bytes of activation memory, and ~40 us per forward GEMM:
#        a wash on enc12, profiles/wgrad_xt_ab.txt);
#   0:   never (both operands read I-contiguous), for A/B runs.
_XT_MODE = os.environ.get("MIPIPE_WGRAD_XT", "auto")
_EMIT_XT = _XT_MODE in ("1", "emit")
_XT_MIN_N = int(os.environ.get("MIPIPE_WGRAD_XT_MIN_N", "4608"))
_XT_MIN_TILES = int(os.environ.get("MIPIPE_WGRAD_XT_MIN_TILES", "0"))
# GELU forwards save GELU'(pre) rather than pre (MIPIPE_GELU_SAVE_GRAD=1).  Off by
# default: the second erf/exp per element in the forward GEMM's epilogue cost the
# GPT-2-XL step more than the one-multiply backward saved (the elementwise GELU
# backward is memory-bound either way: 157 -> 149 us); it pays where the
# backward folds into the consumer's dgrad (GELU without dropout after it).
_GELU_SAVE_GRAD = os.environ.get("MIPIPE_GELU_SAVE_GRAD", "0") == "1"
KACT_SAVED_GRAD = 3  # kernels.h kActSavedGrad
KACT_RELU_BITS = 4   # kernels.h kActReluBits
# ReLU (+ dropout) outputs handed to the consumer's folded dgrad as a bit mask (MIPIPE_RELU_BITS=0: the bf16
# output itself, for A/B runs)
_RELU_BITS = os.environ.get("MIPIPE_RELU_BITS", "1") != "0"


def _defer(w: Tensor, dy: Tensor, x: Tensor, transposed: bool = False) -> None:
    """Queues (dY, X) -- or (dY, X^T) when ``transposed`` -- for ``w``."""
    entry = _DEFERRED.setdefault(id(w), (w, [], [], []))
    entry[1].append(dy)
    entry[2].append(x)
    entry[3].append(transposed)


def _defer_bias(b: Tensor, dy: Tensor) -> None:
    """Bias gradients: column sums of every queued dY, ONE reduction per bias."""
    entry = _DEFERRED.setdefault(id(b), (b, [], None, None))
    entry[1].append(dy)


def accumulate_wgrad(dy: Tensor, x: Tensor, w: Tensor) -> Optional[Tensor]:
    """Weight gradient ``dy^T x`` of ``w`` (2-D operands) for ops with their own
    backward: into ``w.main_grad`` (deferred inside :func:`deferred_wgrad`) when
    it exists, else returned for autograd."""
    main = getattr(w, "main_grad", None)
    k = kernels_for(dy) if dy.is_cuda else None
    tile = (k is not None and dy.dtype == x.dtype and _gemm_supported(k, dy.dtype, w.shape[0], w.shape[1], dy.shape[0]))
    if main is not None and tile:
        dy, x = gemm_operand(dy), gemm_operand(x)
        if _DEFERRED is not None:
            _defer(w, dy, x)
        else:
            k.linear_wgrad(dy, x, main, _claim(w))
        return None
    g = torch.matmul(dy.t(), x)
    if main is not None:
        _add_or_copy(main, g, w)
        return None
    return g.to(w.dtype)


# Objects told when weight gradients become final during a flush (data-parallel
# gradient buckets start their all-reduce then, overlapping the remaining
# weight-gradient GEMMs): ``flush_begin(pending)`` with the parameters whose
# GEMMs are about to be queued, then ``wgrad_done(param)`` after each one.
_WGRAD_LISTENERS: list = []


def add_wgrad_listener(listener) -> None:
    _WGRAD_LISTENERS.append(listener)


def remove_wgrad_listener(listener) -> None:
    if listener in _WGRAD_LISTENERS:
        _WGRAD_LISTENERS.remove(listener)


def flush_wgrad() -> None:
    """Runs every queued weight-gradient GEMM (accumulating into main_grad)."""
    global _DEFERRED
    if not _DEFERRED:
        return
    queue, _DEFERRED = _DEFERRED, {}
    listeners = list(_WGRAD_LISTENERS)
    for li in listeners:
        li.flush_begin([e[0] for e in queue.values()])
    # A bias queued with the very dY tensors of a weight (one Linear) has its
    # column sums folded into that weight's GEMMs (GemmArgs::rowsum / colsum)
    # when the shape allows; it is reduced when its weight is processed.
    weight_dys = {tuple(id(d) for d in e[1]) for e in queue.values() if e[2] is not None}
    bias_of = {}
    for b, dys, xs, _ in queue.values():
        key = tuple(id(d) for d in dys)
        if xs is None and key in weight_dys:
            bias_of[key] = b
    for w, dys, xs, trans in queue.values():
        key = tuple(id(d) for d in dys)
        if xs is None and bias_of.get(key) is w:
            continue  # with its weight
        k = kernels_for(dys[0])
        # a single-process Pipe queues weights of several devices: launch each on its own
        dev = dys[0].device
        done = [w]
        with (torch.cuda.device(dev) if dev.type == "cuda" else contextlib.nullcontext()):
            if xs is None:  # a bias
                k.column_sum_segments(dys, w.main_grad, True)
            else:
                b = bias_of.get(key)
                fused = _flush_weight(k, w, dys, xs, trans, b.main_grad if (b is not None and _FUSE_BIAS) else None)
                if b is not None:
                    if not fused:
                        k.column_sum_segments(dys, b.main_grad, True)
                    done.append(b)
        for li in listeners:
            for p in done:
                li.wgrad_done(p)


def _uniform(ts) -> bool:
    return all(t.shape == ts[0].shape and t.stride() == ts[0].stride() for t in ts)


def _flush_weight(k, w: Tensor, dys, xs, trans, bias_main: Optional[Tensor]) -> bool:
    """One weight's queued gradients: the transposed K-segmented GEMM over the
    micro-batches that saved x^T, the plain one over those that saved x (a
    queue may mix them, e.g. a tensor that bypassed the tile path).  Returns
    whether ``bias_main`` received the bias gradient (folded into a GEMM)."""
    t_idx = [i for i, t in enumerate(trans) if t]
    x_idx = [i for i, t in enumerate(trans) if not t]
    T = dys[0].shape[0]
    fused = False
    if t_idx:
        tdys, txts = [dys[i] for i in t_idx], [xs[i] for i in t_idx]
        if _uniform(tdys) and _uniform(txts) and T % 64 == 0:
            fused = k.linear_wgrad_xt_segments(tdys, txts, w.main_grad, _claim(w),
                                               bias_main if not x_idx else None)
        else:
            for d, xt in zip(tdys, txts):
                k.linear_wgrad_xt_segments([d], [xt], w.main_grad, _claim(w))
    if x_idx:
        pdys, pxs = [dys[i] for i in x_idx], [xs[i] for i in x_idx]
        if not t_idx and _transpose_pays(w, pdys, pxs, T):
            return k.linear_wgrad_xt_segments(pdys, [k.transpose_b16(x) for x in pxs], w.main_grad, _claim(w),
                                              bias_main)
        if _uniform(pdys) and _uniform(pxs) and T % 64 == 0:
            fused = k.linear_wgrad_segments(pdys, pxs, w.main_grad, _claim(w),
                                            bias_main if not t_idx else None)
        else:
            for d, x in zip(pdys, pxs):
                k.linear_wgrad(d, x, w.main_grad, _claim(w))
    return fused


def _transpose_pays(w: Tensor, dys, xs, T: int) -> bool:
    """The flush transposes x for the transposed GEMM (MIPIPE_WGRAD_XT=auto):
    wide enough outputs, bf16, shapes the transpose and the GEMM accept."""
    if _XT_MODE != "auto" or w.shape[0] < _XT_MIN_N or T % 64 != 0:
        return False
    # split-K grids too: GPT-2-XL's fc1 (175 tiles, split 7 ways) runs the two
    # layouts level, but its 6400-wide bias gradient folds into the transposed
    # GEMM instead of a column-sum pass over dY -- +0.47 % on the GPT-2-XL step
    # (tools/gpu_runs/r4_b20.sh; MIPIPE_WGRAD_XT_MIN_TILES restores a tile floor)
    if ((w.shape[1] + 255) // 256) * ((w.shape[0] + 255) // 256) < _XT_MIN_TILES:
        return False
    x0 = xs[0]
    return (x0.dtype == torch.bfloat16 and dys[0].dtype == torch.bfloat16 and x0.dim() == 2
            and x0.stride(1) == 1 and x0.shape[1] % 8 == 0 and x0.stride(0) % 8 == 0
            and _uniform(dys) and _uniform(xs) and all(x.data_ptr() % 16 == 0 for x in xs))


def begin_deferred_wgrad() -> bool:
    """Starts queueing weight gradients (as :class:`deferred_wgrad` does) until
    :func:`end_deferred_wgrad`; for callers whose backward is the user's own
    ``loss.backward()`` (``FlatAdam(defer_wgrad=True)`` around a ``Pipe``).
    Returns False (and does nothing) when a deferral is already active."""
    global _DEFERRED
    if _DEFERRED is not None:
        return False
    _DEFERRED = {}
    return True


def deferred_param_ids() -> set:
    """ids of the weights/biases with queued gradient GEMMs (empty when none)."""
    return set(_DEFERRED) if _DEFERRED else set()


def drop_deferred_wgrad(param_ids: Optional[set] = None) -> None:
    """Discards queued weight gradients without running them: those of
    ``param_ids`` (the deferral stays active), or the whole queue and the
    deferral itself when ``param_ids`` is None."""
    global _DEFERRED
    if param_ids is None:
        _DEFERRED = None
    elif _DEFERRED:
        for key in param_ids:
            _DEFERRED.pop(key, None)


def end_deferred_wgrad() -> None:
    """Runs the queued weight-gradient GEMMs and stops queueing."""
    global _DEFERRED
    try:
        flush_wgrad()
    finally:
        _DEFERRED = None


class deferred_wgrad:
    """Context: queue weight gradients of tile-path linears; flush on exit."""

    def __enter__(self):
        global _DEFERRED
        if _DEFERRED is not None:
            raise RuntimeError("deferred_wgrad() does not nest")
        _DEFERRED = {}
        return self

    def __exit__(self, *exc):
        global _DEFERRED
        try:
            if exc[0] is None:
                flush_wgrad()
        finally:
            _DEFERRED = None
        return False


def linear(
    x: Tensor,
    weight: Tensor,
    bias: Optional[Tensor] = None,
    activation: Optional[str] = None,
    dropout_p: float = 0.0,
    training: bool = True,
    *,
    act_fold_out: Optional[ActFold] = None,
    act_fold_in: Optional[ActFold] = None,
) -> Tensor:
    """``dropout(act(x @ weight.T + bias))``.  ``act_fold_out`` / ``act_fold_in``:
    see :class:`ActFold` (this layer's activation / its input's activation)."""
    p = float(dropout_p) if training else 0.0
    if not x.is_cuda:
        y = F.linear(x, weight)
        return bias_act_reference(y, bias, activation, p, True)
    return _Linear.apply(x, weight, bias, ACTIVATIONS[activation], p, False, None, act_fold_out, act_fold_in,
                         torch.is_grad_enabled())


def linear_residual(
    x: Tensor,
    weight: Tensor,
    bias: Optional[Tensor],
    res: Tensor,
    dropout_p: float = 0.0,
    training: bool = True,
    *,
    act_fold_in: Optional[ActFold] = None,
) -> Tensor:
    """``res + dropout(x @ weight.T + bias)`` -- a pre-norm residual branch's
    output projection with the residual add folded into the GEMM epilogue (no
    separate add kernel: one fewer read of two activations and write of one)."""
    p = float(dropout_p) if training else 0.0
    if not x.is_cuda:
        return res + linear(x, weight, bias, None, p, True)
    return _Linear.apply(x, weight, bias, 0, p, False, res, None, act_fold_in)


def linear_fanout(
    x: Tensor,
    weight: Tensor,
    bias: Optional[Tensor] = None,
    activation: Optional[str] = None,
    dropout_p: float = 0.0,
    training: bool = True,
    *,
    act_fold_out: Optional[ActFold] = None,
):
    """``(linear(x, ...), x')`` where ``x'`` is ``x`` for the input's OTHER
    consumer (a post-norm residual branch).  Mathematically the identity; the
    point is the backward: the gradient reaching ``x'`` is added to ``dx`` in
    the dgrad GEMM's epilogue instead of by a separate autograd add kernel
    (one full read/write pass of the activation per fan-out)."""
    if not x.is_cuda or not torch.is_grad_enabled() or not x.requires_grad:
        return linear(x, weight, bias, activation, dropout_p, training, act_fold_out=act_fold_out), x
    p = float(dropout_p) if training else 0.0
    return _Linear.apply(x, weight, bias, ACTIVATIONS[activation], p, True, None, act_fold_out)
