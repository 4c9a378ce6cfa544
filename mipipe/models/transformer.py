"""Transformer blocks on the mipipe HIP ops (SURVEY §7.1 'Models').

A :class:`TransformerEncoderLayer` is the drop-in equivalent of
``nn.TransformerEncoderLayer`` as the reference driver uses it
(``/root/reference/main.py:115-120,139-157``: post-norm, ReLU, dropout, no
mask), but batch-first ``[B, S, E]`` and built from two *pipeline-splittable*
halves, each a single-tensor module:

* :class:`SelfAttentionBlock` -- ``LN1(x + drop(out_proj(attn(qkv(x)))))``
  (pre-norm: ``x + drop(out_proj(attn(qkv(LN1(x)))))``);
* :class:`FeedForwardBlock`   -- ``LN2(x + drop(W2 drop(act(W1 x))))``.

Splitting at sub-layer granularity lets the balancer put stage boundaries
between the attention and MLP halves, which matters when 12 layers are spread
over 8 MI355X stages.

Hot path per block: MFMA GEMMs with fused bias/activation/dropout epilogues,
flash attention, fused dropout+residual+LayerNorm -- see ``mipipe.ops``.
``from_torch`` copies weights from an ``nn.TransformerEncoderLayer`` so the
blocks can be checked against PyTorch.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import torch
from torch import Tensor, nn

from .. import ops
from ..ops.linear import ActFold, mark_gemm_weight

# Fan-out fusion of the residual-branch gradient (see AttentionCore.forward_fanout);
# MIPIPE_FANOUT=0 turns it off (A/B measurements).
FANOUT = os.environ.get("MIPIPE_FANOUT", "1") != "0"
# MLP activation backward in fc_out's dgrad epilogue (ops.linear.ActFold), for
# the activations in FOLD_ACTS.  ReLU's backward is a sign test on the saved
# output, nearly free in the epilogue (enc12 FFN dgrad + act backward 240 -> 222
# us).  GELU's is one multiply as well when its forward saves GELU'(pre)
# (ops.linear MIPIPE_GELU_SAVE_GRAD=1, not the default); with pre saved, the
# erf/exp per element made the epilogue slower than the separate memory-bound
# kernel (GPT-2-XL fc2 dgrad 244 -> 251 us; tools/gemm_dact_probe.py), so GELU
# is then not folded.  MIPIPE_FOLD_ACT=0: off, =relu: ReLU only, =all: both.
_FOLD_ENV = os.environ.get("MIPIPE_FOLD_ACT", "auto")
if _FOLD_ENV == "auto":
    _FOLD_ENV = "all" if os.environ.get("MIPIPE_GELU_SAVE_GRAD", "0") == "1" else "relu"
FOLD_ACTS = () if _FOLD_ENV == "0" else (("relu", "gelu") if _FOLD_ENV == "all" else ("relu",))


def _folds(fc_in, training: bool) -> bool:
    """Fold fc_in's activation backward into fc_out's dgrad?  GELU only without
    dropout after it: the GEMM epilogue would regenerate the mask with Philox per
    element, which cost more than the separate pass saves (GPT-2-XL PP=1, p =
    0.1: 62.3k vs 62.9k tok/s) -- ReLU's saved output carries its mask."""
    act = fc_in.activation
    if act not in FOLD_ACTS:
        return False
    return act != "gelu" or not (training and fc_in.dropout > 0.0)

__all__ = [
    "AttentionCore",
    "AttentionOutput",
    "PackedAttentionCore",
    "PackedAttentionOutput",
    "SelfAttentionBlock",
    "FeedForwardBlock",
    "FeedForwardIn",
    "FeedForwardOut",
    "PackedFeedForwardIn",
    "PackedFeedForwardOut",
    "TransformerEncoderLayer",
    "transformer_blocks",
    "block_flops",
]


class AttentionCore(nn.Module):
    """QKV projection + scaled-dot-product attention (pre-norm: LN first).

    ``x [B, S, E] -> o [B, S, E]`` (attention output before ``out_proj``).
    """

    def __init__(self, d_model: int, nhead: int, dropout: float, *, norm_first: bool, causal: bool,
                 layer_norm_eps: float, device=None, dtype=None) -> None:
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.d_model, self.nhead, self.head_dim = d_model, nhead, d_model // nhead
        self.dropout, self.norm_first, self.causal, self.eps = dropout, norm_first, causal, layer_norm_eps
        self.in_proj_weight = mark_gemm_weight(nn.Parameter(torch.empty(3 * d_model, d_model, **fk)))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * d_model, **fk))
        if norm_first:
            self.norm_weight = nn.Parameter(torch.empty(d_model, **fk))
            self.norm_bias = nn.Parameter(torch.empty(d_model, **fk))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        # nn.MultiheadAttention's init: xavier on in_proj, zero biases.
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.in_proj_bias)
        if self.norm_first:
            nn.init.ones_(self.norm_weight)
            nn.init.zeros_(self.norm_bias)

    def forward(self, x: Tensor) -> Tensor:
        return self.forward_fanout(x, fanout=False)[0]

    def forward_fanout(self, x: Tensor, fanout: bool = True):
        """``(o, x')``: ``x'`` is the block input for the residual branch.  With
        ``fanout`` the first consumer of ``x`` (LN1 for pre-norm, the QKV
        projection for post-norm) also returns it, so the residual gradient is
        added inside that op's backward kernel (no autograd add pass)."""
        B, S, E = x.shape
        H, D = self.nhead, self.head_dim
        xr = x
        if self.norm_first:
            if fanout:
                x, xr = ops.layer_norm_fanout(x, self.norm_weight, self.norm_bias, self.eps)
            else:
                x = ops.add_dropout_layer_norm(x, None, self.norm_weight, self.norm_bias, self.eps, 0.0,
                                               self.training)
            qkv = ops.linear(x, self.in_proj_weight, self.in_proj_bias)
        elif fanout:
            qkv, xr = ops.linear_fanout(x, self.in_proj_weight, self.in_proj_bias)
        else:
            qkv = ops.linear(x, self.in_proj_weight, self.in_proj_bias)
        # The projection output viewed as [B, S, 3, H, D] feeds the kernel in
        # place; its output [B, S, H, D] is already [B, S, E] -- no transposes.
        o = ops.attention_packed(qkv.view(B, S, 3, H, D), causal=self.causal, dropout_p=self.dropout,
                                 training=self.training)
        return o.reshape(B, S, E), xr

    def flops_per_token(self, seq_len: int) -> float:
        e = self.d_model
        return 2 * 3 * e * e + 4 * seq_len * e * (0.5 if self.causal else 1.0)


class AttentionOutput(nn.Module):
    """``out_proj`` + dropout + residual (+ LayerNorm for post-norm): ``(x, o) -> y``."""

    def __init__(self, d_model: int, dropout: float, *, norm_first: bool, layer_norm_eps: float,
                 device=None, dtype=None) -> None:
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.d_model, self.dropout, self.norm_first, self.eps = d_model, dropout, norm_first, layer_norm_eps
        self.out_proj_weight = mark_gemm_weight(nn.Parameter(torch.empty(d_model, d_model, **fk)))
        self.out_proj_bias = nn.Parameter(torch.empty(d_model, **fk))
        if not norm_first:
            self.norm_weight = nn.Parameter(torch.empty(d_model, **fk))
            self.norm_bias = nn.Parameter(torch.empty(d_model, **fk))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        bound = 1.0 / math.sqrt(self.d_model)
        nn.init.uniform_(self.out_proj_weight, -bound, bound)
        nn.init.zeros_(self.out_proj_bias)
        if not self.norm_first:
            nn.init.ones_(self.norm_weight)
            nn.init.zeros_(self.norm_bias)

    def forward(self, x: Tensor, o: Tensor) -> Tensor:
        p = self.dropout if self.training else 0.0
        if self.norm_first:
            return ops.linear_residual(o, self.out_proj_weight, self.out_proj_bias, x, p, self.training)
        a = ops.linear(o, self.out_proj_weight, self.out_proj_bias)
        return ops.add_dropout_layer_norm(a, x, self.norm_weight, self.norm_bias, self.eps, p, self.training)

    def flops_per_token(self, seq_len: int) -> float:
        return 2 * self.d_model * self.d_model


class SelfAttentionBlock(nn.Module):
    """Attention half of a Transformer layer: ``y = out(x, core(x))``.

    Post-norm: ``LN1(x + drop(out_proj(attn(qkv(x)))))``; pre-norm:
    ``x + drop(out_proj(attn(qkv(LN1(x)))))``.
    """

    def __init__(self, d_model: int, nhead: int, dropout: float = 0.1, *, norm_first: bool = False,
                 causal: bool = False, layer_norm_eps: float = 1e-5, device=None, dtype=None) -> None:
        super().__init__()
        if d_model % nhead != 0:
            raise ValueError("d_model must be divisible by nhead")
        self.core = AttentionCore(d_model, nhead, dropout, norm_first=norm_first, causal=causal,
                                  layer_norm_eps=layer_norm_eps, device=device, dtype=dtype)
        self.out = AttentionOutput(d_model, dropout, norm_first=norm_first, layer_norm_eps=layer_norm_eps,
                                   device=device, dtype=dtype)

    def reset_parameters(self) -> None:
        self.core.reset_parameters()
        self.out.reset_parameters()

    def forward(self, x: Tensor) -> Tensor:
        o, xr = self.core.forward_fanout(x, FANOUT)
        return self.out(xr, o)

    def flops_per_token(self, seq_len: int) -> float:
        return self.core.flops_per_token(seq_len) + self.out.flops_per_token(seq_len)


class _Unpack(torch.autograd.Function):
    """A packed stage-boundary activation -> its parts, as contiguous views.

    The packs are block-concatenated (part after part in memory, not
    interleaved per row), so every part is a contiguous view -- the consumer
    needs no ``.contiguous()`` copies -- and the backward writes the parts'
    gradients into one packed gradient with a single concatenation (autograd's
    own slice/select backward would zero-fill a packed-size tensor per part
    and add them)."""

    @staticmethod
    def forward(ctx, packed: Tensor, lead, widths):  # type: ignore[override]
        flat = packed.reshape(-1)
        n = math.prod(lead)
        outs, o = [], 0
        for w in widths:
            outs.append(flat[o:o + n * w].view(*lead, w))
            o += n * w
        ctx.packed_shape, ctx.lead, ctx.widths = packed.shape, lead, widths
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):  # type: ignore[override]
        ref = next(g for g in grads if g is not None)
        n = math.prod(ctx.lead)
        parts = [g.reshape(-1) if g is not None else ref.new_zeros(n * w) for g, w in zip(grads, ctx.widths)]
        return torch.cat(parts).view(ctx.packed_shape), None, None


def unpack(packed: Tensor, lead, widths):
    return _Unpack.apply(packed, tuple(lead), tuple(widths))


class PackedAttentionCore(nn.Module):
    """Pipeline unit: ``x -> stack(x, core(x))`` so a stage boundary can fall
    between the attention core and its output projection."""

    def __init__(self, core: AttentionCore) -> None:
        super().__init__()
        self.core = core

    def reset_parameters(self) -> None:
        self.core.reset_parameters()

    def forward(self, x: Tensor) -> Tensor:
        # x's residual-branch gradient comes back through the QKV dgrad epilogue (fan-out)
        o, xr = self.core.forward_fanout(x, FANOUT)
        return torch.stack((xr, o))

    def flops_per_token(self, seq_len: int) -> float:
        return self.core.flops_per_token(seq_len)


class PackedAttentionOutput(nn.Module):
    """Pipeline unit: ``stack(x, o) -> out(x, o)``."""

    def __init__(self, out: AttentionOutput) -> None:
        super().__init__()
        self.out = out

    def reset_parameters(self) -> None:
        self.out.reset_parameters()

    def forward(self, packed: Tensor) -> Tensor:
        e = packed.shape[-1]
        x, o = unpack(packed, packed.shape[1:-1], (e, e))
        return self.out(x, o)

    def flops_per_token(self, seq_len: int) -> float:
        return self.out.flops_per_token(seq_len)


class FeedForwardIn(nn.Module):
    """First half of the MLP: ``h = drop(act(W1 x + b1))`` (pre-norm: of ``LN2(x)``)."""

    def __init__(self, d_model: int, dim_feedforward: int, dropout: float, activation: str, *, norm_first: bool,
                 layer_norm_eps: float, device=None, dtype=None) -> None:
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.d_model, self.dim_feedforward = d_model, dim_feedforward
        self.dropout, self.activation, self.norm_first, self.eps = dropout, activation, norm_first, layer_norm_eps
        self.linear1_weight = mark_gemm_weight(nn.Parameter(torch.empty(dim_feedforward, d_model, **fk)))
        self.linear1_bias = nn.Parameter(torch.empty(dim_feedforward, **fk))
        if norm_first:
            self.norm_weight = nn.Parameter(torch.empty(d_model, **fk))
            self.norm_bias = nn.Parameter(torch.empty(d_model, **fk))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        nn.init.kaiming_uniform_(self.linear1_weight, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(self.linear1_weight.shape[1])
        nn.init.uniform_(self.linear1_bias, -bound, bound)
        if self.norm_first:
            nn.init.ones_(self.norm_weight)
            nn.init.zeros_(self.norm_bias)

    def forward(self, x: Tensor) -> Tensor:
        return self.forward_fanout(x, fanout=False)[0]

    def forward_fanout(self, x: Tensor, fanout: bool = True, fold: Optional[ActFold] = None):
        """``(h, x')`` -- see :meth:`AttentionCore.forward_fanout`.  ``fold``: h's
        only consumer applies the activation backward (:class:`ActFold`)."""
        p = self.dropout if self.training else 0.0
        w, b, act = self.linear1_weight, self.linear1_bias, self.activation
        if self.norm_first:
            if fanout:
                xn, xr = ops.layer_norm_fanout(x, self.norm_weight, self.norm_bias, self.eps)
            else:
                xn, xr = ops.add_dropout_layer_norm(x, None, self.norm_weight, self.norm_bias, self.eps, 0.0,
                                                    self.training), x
            return ops.linear(xn, w, b, act, p, self.training, act_fold_out=fold), xr
        if fanout:
            return ops.linear_fanout(x, w, b, act, p, self.training, act_fold_out=fold)
        return ops.linear(x, w, b, act, p, self.training, act_fold_out=fold), x

    def flops_per_token(self, seq_len: int) -> float:
        return 2 * self.d_model * self.dim_feedforward


class FeedForwardOut(nn.Module):
    """Second half: ``LN2(x + drop(W2 h + b2))`` (pre-norm: ``x + drop(W2 h + b2)``)."""

    def __init__(self, d_model: int, dim_feedforward: int, dropout: float, *, norm_first: bool, layer_norm_eps: float,
                 device=None, dtype=None) -> None:
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.d_model, self.dim_feedforward = d_model, dim_feedforward
        self.dropout, self.norm_first, self.eps = dropout, norm_first, layer_norm_eps
        self.linear2_weight = mark_gemm_weight(nn.Parameter(torch.empty(d_model, dim_feedforward, **fk)))
        self.linear2_bias = nn.Parameter(torch.empty(d_model, **fk))
        if not norm_first:
            self.norm_weight = nn.Parameter(torch.empty(d_model, **fk))
            self.norm_bias = nn.Parameter(torch.empty(d_model, **fk))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        nn.init.kaiming_uniform_(self.linear2_weight, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(self.linear2_weight.shape[1])
        nn.init.uniform_(self.linear2_bias, -bound, bound)
        if not self.norm_first:
            nn.init.ones_(self.norm_weight)
            nn.init.zeros_(self.norm_bias)

    def forward(self, x: Tensor, h: Tensor, fold: Optional[ActFold] = None) -> Tensor:
        p = self.dropout if self.training else 0.0
        if self.norm_first:
            return ops.linear_residual(h, self.linear2_weight, self.linear2_bias, x, p, self.training,
                                       act_fold_in=fold)
        h = ops.linear(h, self.linear2_weight, self.linear2_bias, act_fold_in=fold)
        return ops.add_dropout_layer_norm(h, x, self.norm_weight, self.norm_bias, self.eps, p, self.training)

    def flops_per_token(self, seq_len: int) -> float:
        return 2 * self.d_model * self.dim_feedforward


class FeedForwardBlock(nn.Module):
    """``LN2(x + drop(W2 drop(act(W1 x))))`` as two halves (:class:`FeedForwardIn`,
    :class:`FeedForwardOut`) so a pipeline boundary may fall between them."""

    def __init__(
        self,
        d_model: int,
        dim_feedforward: int,
        dropout: float = 0.1,
        activation: str = "relu",
        *,
        norm_first: bool = False,
        layer_norm_eps: float = 1e-5,
        device=None,
        dtype=None,
    ) -> None:
        super().__init__()
        self.d_model, self.dim_feedforward = d_model, dim_feedforward
        self.norm_first = norm_first
        self.fc_in = FeedForwardIn(d_model, dim_feedforward, dropout, activation, norm_first=norm_first,
                                   layer_norm_eps=layer_norm_eps, device=device, dtype=dtype)
        self.fc_out = FeedForwardOut(d_model, dim_feedforward, dropout, norm_first=norm_first,
                                     layer_norm_eps=layer_norm_eps, device=device, dtype=dtype)

    def reset_parameters(self) -> None:
        self.fc_in.reset_parameters()
        self.fc_out.reset_parameters()

    def forward(self, x: Tensor) -> Tensor:
        # h's only consumer is fc_out: its dgrad applies the activation backward
        fold = ActFold() if _folds(self.fc_in, self.training) else None
        h, xr = self.fc_in.forward_fanout(x, FANOUT, fold)
        out = self.fc_out(xr, h, fold)
        if fold is not None:
            fold.release()
        return out

    def flops_per_token(self, seq_len: int) -> float:
        return 2 * 2 * self.d_model * self.dim_feedforward


class PackedFeedForwardIn(nn.Module):
    """Pipeline unit: ``x -> [.., E + F]`` holding x and h block-concatenated
    (all of x, then all of h: see :class:`_Unpack`)."""

    def __init__(self, fc_in: FeedForwardIn) -> None:
        super().__init__()
        self.fc_in = fc_in

    def reset_parameters(self) -> None:
        self.fc_in.reset_parameters()

    def forward(self, x: Tensor) -> Tensor:
        h, xr = self.fc_in.forward_fanout(x, FANOUT)
        return torch.cat((xr.reshape(-1), h.reshape(-1))).view(*x.shape[:-1], x.shape[-1] + h.shape[-1])

    def flops_per_token(self, seq_len: int) -> float:
        return self.fc_in.flops_per_token(seq_len)


class PackedFeedForwardOut(nn.Module):
    """Pipeline unit: ``cat(x, h) -> fc_out(x, h)``."""

    def __init__(self, fc_out: FeedForwardOut) -> None:
        super().__init__()
        self.fc_out = fc_out

    def reset_parameters(self) -> None:
        self.fc_out.reset_parameters()

    def forward(self, packed: Tensor) -> Tensor:
        e = self.fc_out.d_model
        x, h = unpack(packed, packed.shape[:-1], (e, packed.shape[-1] - e))
        return self.fc_out(x, h)

    def flops_per_token(self, seq_len: int) -> float:
        return self.fc_out.flops_per_token(seq_len)


class TransformerEncoderLayer(nn.Sequential):
    """``nn.TransformerEncoderLayer`` equivalent (batch-first) as a 2-block Sequential."""

    def __init__(
        self,
        d_model: int,
        nhead: int,
        dim_feedforward: int = 2048,
        dropout: float = 0.1,
        activation: str = "relu",
        layer_norm_eps: float = 1e-5,
        norm_first: bool = False,
        causal: bool = False,
        device=None,
        dtype=None,
    ) -> None:
        super().__init__(
            SelfAttentionBlock(d_model, nhead, dropout, norm_first=norm_first, causal=causal,
                               layer_norm_eps=layer_norm_eps, device=device, dtype=dtype),
            FeedForwardBlock(d_model, dim_feedforward, dropout, activation, norm_first=norm_first,
                             layer_norm_eps=layer_norm_eps, device=device, dtype=dtype),
        )

    @torch.no_grad()
    def load_from_torch(self, layer: nn.TransformerEncoderLayer) -> "TransformerEncoderLayer":
        """Copies weights from ``nn.TransformerEncoderLayer``."""
        attn, ff = self[0], self[1]
        attn.core.in_proj_weight.copy_(layer.self_attn.in_proj_weight)
        attn.core.in_proj_bias.copy_(layer.self_attn.in_proj_bias)
        attn.out.out_proj_weight.copy_(layer.self_attn.out_proj.weight)
        attn.out.out_proj_bias.copy_(layer.self_attn.out_proj.bias)
        norm1 = attn.core if attn.core.norm_first else attn.out
        norm1.norm_weight.copy_(layer.norm1.weight)
        norm1.norm_bias.copy_(layer.norm1.bias)
        ff.fc_in.linear1_weight.copy_(layer.linear1.weight)
        ff.fc_in.linear1_bias.copy_(layer.linear1.bias)
        ff.fc_out.linear2_weight.copy_(layer.linear2.weight)
        ff.fc_out.linear2_bias.copy_(layer.linear2.bias)
        norm2 = ff.fc_in if ff.norm_first else ff.fc_out
        norm2.norm_weight.copy_(layer.norm2.weight)
        norm2.norm_bias.copy_(layer.norm2.bias)
        return self


def transformer_blocks(
    num_layers: int,
    d_model: int,
    nhead: int,
    dim_feedforward: int,
    dropout: float,
    activation: str = "relu",
    *,
    norm_first: bool = False,
    causal: bool = False,
    device=None,
    dtype=None,
) -> List[nn.Module]:
    """``2 * num_layers`` single-tensor blocks (attention, MLP, attention, ...)."""
    blocks: List[nn.Module] = []
    for _ in range(num_layers):
        layer = TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation,
                                        norm_first=norm_first, causal=causal, device=device, dtype=dtype)
        blocks.extend(layer.children())
    return blocks


def pipeline_units(blocks: List[nn.Module]) -> List[nn.Module]:
    """Expands every :class:`SelfAttentionBlock` and :class:`FeedForwardBlock`
    into its two packed halves so a pipeline stage boundary may fall inside it
    (see :func:`merge_units`): 4 units per layer."""
    units: List[nn.Module] = []
    for b in blocks:
        if isinstance(b, SelfAttentionBlock):
            units += [PackedAttentionCore(b.core), PackedAttentionOutput(b.out)]
        elif isinstance(b, FeedForwardBlock):
            units += [PackedFeedForwardIn(b.fc_in), PackedFeedForwardOut(b.fc_out)]
        else:
            units.append(b)
    return units


def merge_units(units: List[nn.Module]) -> List[nn.Module]:
    """Inverse of :func:`pipeline_units` within one stage: an adjacent
    (PackedAttentionCore, PackedAttentionOutput) pair of the same layer runs
    unpacked (no stack copy)."""
    out: List[nn.Module] = []
    i = 0
    while i < len(units):
        u = units[i]
        nxt = units[i + 1] if i + 1 < len(units) else None
        if isinstance(u, PackedAttentionCore) and isinstance(nxt, PackedAttentionOutput):
            blk = SelfAttentionBlock.__new__(SelfAttentionBlock)
            nn.Module.__init__(blk)
            blk.core = u.core
            blk.out = nxt.out
            out.append(blk)
            i += 2
            continue
        if isinstance(u, PackedFeedForwardIn) and isinstance(nxt, PackedFeedForwardOut):
            blk = FeedForwardBlock.__new__(FeedForwardBlock)
            nn.Module.__init__(blk)
            blk.d_model, blk.dim_feedforward = u.fc_in.d_model, u.fc_in.dim_feedforward
            blk.norm_first = u.fc_in.norm_first
            blk.fc_in = u.fc_in
            blk.fc_out = nxt.fc_out
            out.append(blk)
            i += 2
            continue
        out.append(u)
        i += 1
    return out


def block_flops(block: nn.Module, seq_len: int) -> float:
    """Training FLOPs per token of a block (forward x 3)."""
    f = getattr(block, "flops_per_token", None)
    if f is None:
        return 0.0
    return 3.0 * f(seq_len)
