"""MI355X compute ops used by ``mipipe.models``.

Each op has one GPU implementation -- a hand-written CDNA4 HIP kernel in
``mipipe/csrc/kernels`` -- and an eager CPU implementation used only for
CPU tensors (plumbing tests).  GPU tensors never fall back to eager PyTorch:
a missing extension raises (``mipipe._native_loader.kernels``).
"""
from .layernorm import add_dropout_layer_norm, layer_norm_fanout, layer_norm_reference
from .linear import deferred_wgrad, flush_wgrad, linear, linear_fanout, linear_residual
from .attention import attention, attention_packed, attention_reference
from .activation import bias_act_dropout
from .loss import cross_entropy
from .embedding import embed_scale_posenc_dropout

__all__ = [
    "add_dropout_layer_norm",
    "layer_norm_fanout",
    "layer_norm_reference",
    "linear",
    "linear_fanout",
    "linear_residual",
    "deferred_wgrad",
    "flush_wgrad",
    "attention",
    "attention_packed",
    "attention_reference",
    "bias_act_dropout",
    "cross_entropy",
    "embed_scale_posenc_dropout",
]
