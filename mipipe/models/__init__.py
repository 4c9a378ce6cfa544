"""Model families built on mipipe ops: post-norm TransformerEncoder (reference
driver), GPT-2 style pre-norm causal decoder, LM embedding/head."""
from .transformer import (
    FeedForwardBlock,
    SelfAttentionBlock,
    TransformerEncoderLayer,
    block_flops,
    transformer_blocks,
)
from .lm import (CONFIGS, Decoder, Encoder, FinalNorm, LMConfig, TargetSequential, build_lm_blocks,
                 lm_pipeline_units, sinusoidal_positions)
from .vocab_split import DecoderHead, DecoderTail, split_decoder

__all__ = [
    "SelfAttentionBlock",
    "FeedForwardBlock",
    "TransformerEncoderLayer",
    "transformer_blocks",
    "block_flops",
    "Encoder",
    "Decoder",
    "FinalNorm",
    "LMConfig",
    "CONFIGS",
    "build_lm_blocks",
    "lm_pipeline_units",
    "TargetSequential",
    "DecoderHead",
    "DecoderTail",
    "split_decoder",
    "sinusoidal_positions",
]
