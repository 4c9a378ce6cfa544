"""Language-model front/back ends and model builders.

Mirrors the reference driver's model (``/root/reference/main.py:24-73,115-157``):
``Encoder`` (embedding x sqrt(E) + sinusoidal positions + dropout) ->
N x TransformerEncoderLayer -> ``Decoder`` (Linear E -> V).  Batch-first
throughout (the reference transposes to seq-first for nn.TransformerEncoder and
back in the decoder; here no transpose is needed).

Builders return flat lists of single-tensor blocks so the pipeline balancer can
place stage boundaries anywhere, including between the attention and MLP
halves of a layer.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch
from torch import Tensor, nn

from .. import ops
from ..ops.linear import mark_gemm_weight
from .transformer import FeedForwardBlock, transformer_blocks

__all__ = [
    "Encoder",
    "Decoder",
    "LMConfig",
    "CONFIGS",
    "build_lm_blocks",
    "sinusoidal_positions",
]


def sinusoidal_positions(max_len: int, d_model: int) -> Tensor:
    """The reference's PositionalEncoding table (``main.py:57-70``), fp32 [max_len, d]."""
    pe = torch.zeros(max_len, d_model)
    position = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe


class Encoder(nn.Module):
    """Token embedding x sqrt(E) + positional encoding + dropout: ``[B, S] -> [B, S, E]``.

    ``learned_positions=True`` gives GPT-2's learned position embedding instead
    of the sinusoidal table.
    """

    def __init__(self, ntoken: int, d_model: int, dropout: float = 0.5, max_len: int = 5000, *,
                 learned_positions: bool = False, scale_embedding: bool = True, device=None, dtype=None) -> None:
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.ntoken, self.d_model, self.dropout = ntoken, d_model, dropout
        self.scale = math.sqrt(d_model) if scale_embedding else 1.0
        self.weight = nn.Parameter(torch.empty(ntoken, d_model, **fk))
        self.learned_positions = learned_positions
        if learned_positions:
            self.pos_weight = nn.Parameter(torch.empty(max_len, d_model, device=device, dtype=torch.float32))
        else:
            self.register_buffer("pe", sinusoidal_positions(max_len, d_model).to(device), persistent=False)
        self.max_len = max_len
        self.reset_parameters()

    def reset_parameters(self) -> None:
        nn.init.uniform_(self.weight, -0.1, 0.1)  # main.py:32-34
        if self.learned_positions:
            nn.init.normal_(self.pos_weight, std=0.01)
        elif self.pe.device.type != "meta":
            with torch.no_grad():
                self.pe.copy_(sinusoidal_positions(self.max_len, self.d_model))

    def forward(self, tokens: Tensor) -> Tensor:
        # learned positions: the fused kernels add them and accumulate their gradient
        pe = self.pos_weight if self.learned_positions else self.pe
        return ops.embed_scale_posenc_dropout(tokens, self.weight, pe, self.scale, self.dropout, self.training)

    def flops_per_token(self, seq_len: int) -> float:
        return 0.0


class _VocabSlice(torch.autograd.Function):
    """``y[..., :V]`` of the padded logits.  Backward: when the incoming
    gradient is the fused cross-entropy's zero-padded buffer (its usual
    producer), that buffer IS the padded gradient -- no zero-fill + copy."""

    @staticmethod
    def forward(ctx, y, v):  # type: ignore[override]
        ctx.shape = y.shape
        return y[..., :v]

    @staticmethod
    def backward(ctx, g):  # type: ignore[override]
        from ..ops.loss import take_zero_padded

        width = ctx.shape[-1]
        if take_zero_padded(g, width):
            return torch.as_strided(g, ctx.shape, torch.empty(ctx.shape, device="meta").stride()), None
        out = g.new_zeros(ctx.shape)
        out[..., : g.shape[-1]] = g
        return out, None


class Decoder(nn.Module):
    """Linear ``E -> V`` (``main.py:42-55``).

    The weight is stored with the vocabulary padded to a multiple of
    ``pad_to`` (256: the large GEMM tile) -- zero rows, zero bias -- so the logits
    GEMM runs on the MFMA tile kernel; ``forward`` returns the ``[..., :V]``
    view and the fused cross-entropy reads it in place (strided rows).
    """

    def __init__(self, ntoken: int, d_model: int, *, pad_to: int = 256, device=None, dtype=None) -> None:
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.ntoken = ntoken
        self.padded = (ntoken + pad_to - 1) // pad_to * pad_to
        self.weight = mark_gemm_weight(nn.Parameter(torch.empty(self.padded, d_model, **fk)))
        self.bias = nn.Parameter(torch.zeros(self.padded, **fk))
        self.reset_parameters()

    def reset_parameters(self) -> None:
        with torch.no_grad():
            nn.init.uniform_(self.weight, -0.1, 0.1)  # main.py:47-50
            self.weight[self.ntoken:].zero_()
            nn.init.zeros_(self.bias)

    def forward(self, x: Tensor) -> Tensor:
        y = ops.linear(x, self.weight, self.bias)
        if self.padded == self.ntoken:
            return y
        if y.is_cuda and torch.is_grad_enabled() and y.requires_grad:
            return _VocabSlice.apply(y, self.ntoken)
        return y[..., : self.ntoken]

    def flops_per_token(self, seq_len: int) -> float:
        return 2.0 * self.weight.shape[0] * self.weight.shape[1]


class FinalNorm(nn.Module):
    """Pre-norm models' final LayerNorm (GPT-2's ln_f)."""

    def __init__(self, d_model: int, eps: float = 1e-5, *, device=None, dtype=None) -> None:
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d_model, device=device, dtype=dtype))
        self.bias = nn.Parameter(torch.zeros(d_model, device=device, dtype=dtype))
        self.eps = eps

    def reset_parameters(self) -> None:
        nn.init.ones_(self.weight)
        nn.init.zeros_(self.bias)

    def forward(self, x: Tensor) -> Tensor:
        return ops.add_dropout_layer_norm(x, None, self.weight, self.bias, self.eps, 0.0, self.training)

    def flops_per_token(self, seq_len: int) -> float:
        return 0.0


@dataclass
class LMConfig:
    name: str
    num_layers: int
    d_model: int
    nhead: int
    dim_feedforward: int
    vocab: int
    seq_len: int
    dropout: float = 0.2
    activation: str = "relu"
    norm_first: bool = False
    causal: bool = False
    learned_positions: bool = False
    scale_embedding: bool = True
    # dropout between the MLP's activation and its second linear: None = `dropout` (torch's
    # TransformerEncoderLayer: linear2(dropout(act(linear1(x))))); GPT-2's MLP has none there
    # (c_fc -> gelu -> c_proj -> resid dropout)
    act_dropout: Optional[float] = None
    notes: str = ""

    def params(self) -> int:
        e, f, v = self.d_model, self.dim_feedforward, self.vocab
        layer = 4 * e * e + 4 * e + 2 * e * f + f + e + 4 * e
        return self.num_layers * layer + v * e + (v * e + v)


CONFIGS = {
    # BASELINE.json config #2/#3: 12-layer TransformerEncoder d_model=4096 nhead=16.
    # dim_feedforward = d_model and dropout 0.2 follow the reference driver's
    # convention (main.py:116-120: nhid = emsize, dropout = 0.2); the LM
    # front/back end and vocabulary are the driver's (WikiText-2, 28,782 tokens).
    "enc12_d4096": LMConfig("enc12_d4096", 12, 4096, 16, 4096, 28782, 128,
                            notes="post-norm ReLU TransformerEncoder, FF=d_model, LM head as main.py"),
    # The reference's own run (main.py): 16 layers, d=2048, 32 heads, FF=2048.
    "ref_main": LMConfig("ref_main", 16, 2048, 32, 2048, 28782, 128, notes="reference main.py model"),
    # BASELINE.json config #4: GPT-2-XL 1.5B (pre-norm, causal, GELU, learned positions).
    "gpt2_xl": LMConfig("gpt2_xl", 48, 1600, 25, 6400, 50257, 1024, dropout=0.1, activation="gelu",
                        norm_first=True, causal=True, learned_positions=True, scale_embedding=False,
                        act_dropout=0.0,
                        notes="GPT-2's block: attention / residual / embedding dropout 0.1, none after the GELU"),
    # Tiny config for smoke tests.
    "tiny": LMConfig("tiny", 2, 256, 4, 512, 1000, 64, dropout=0.1),
}


def build_lm_blocks(cfg: LMConfig, *, device=None, dtype=None) -> List[nn.Module]:
    """``[Encoder, attn0, mlp0, attn1, mlp1, ..., (FinalNorm), Decoder]``."""
    blocks: List[nn.Module] = [
        Encoder(cfg.vocab, cfg.d_model, cfg.dropout, max_len=max(cfg.seq_len, 1024),
                learned_positions=cfg.learned_positions, scale_embedding=cfg.scale_embedding,
                device=device, dtype=dtype)
    ]
    blocks += transformer_blocks(cfg.num_layers, cfg.d_model, cfg.nhead, cfg.dim_feedforward, cfg.dropout,
                                 cfg.activation, norm_first=cfg.norm_first, causal=cfg.causal,
                                 device=device, dtype=dtype)
    if cfg.act_dropout is not None:
        for b in blocks:
            if isinstance(b, FeedForwardBlock):
                b.fc_in.dropout = cfg.act_dropout
    if cfg.norm_first:
        blocks.append(FinalNorm(cfg.d_model, device=device, dtype=dtype))
    blocks.append(Decoder(cfg.vocab, cfg.d_model, device=device, dtype=dtype))
    return blocks


class TargetSequential(nn.Sequential):
    """``nn.Sequential`` that also hands the micro-batch targets to the children
    that want them (``wants_target``: the vocabulary-split decoder units)."""

    @property
    def wants_target(self) -> bool:
        return any(getattr(m, "wants_target", False) for m in self)

    @property
    def fused_loss(self) -> bool:
        return len(self) > 0 and getattr(self[-1], "fused_loss", False)

    def forward(self, x, target=None):  # type: ignore[override]
        for m in self:
            x = m(x, target) if getattr(m, "wants_target", False) else m(x)
        return x


def lm_pipeline_units(blocks: List[nn.Module], *, split_decoder: bool = False) -> List[nn.Module]:
    """:func:`~mipipe.models.transformer.pipeline_units` of an LM, optionally with
    the decoder cut along the vocabulary (:mod:`mipipe.models.vocab_split`)."""
    from .transformer import pipeline_units
    from .vocab_split import split_decoder as _split

    units = pipeline_units(blocks)
    if split_decoder and isinstance(units[-1], Decoder):
        head, tail = _split(units[-1])
        units = units[:-1] + [head, tail]
    return units
