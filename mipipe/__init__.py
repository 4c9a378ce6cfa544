"""mipipe -- an MI355X-native GPipe pipeline-parallel engine.

Public API mirrors ``torch.distributed.pipeline.sync`` (``/root/reference/pipe.py:24``):

    from mipipe import Pipe, WithDevice, NoChunk
    pipe = Pipe(nn.Sequential(stage0.to("cuda:0"), stage1.to("cuda:1")), chunks=8,
                checkpoint="except_last")
    out = pipe(x).local_value()

Layers: ``stream`` (L2), ``copy``/``dependency``/``phony``/
``checkpoint`` (L3), ``skip`` (L3'), ``microbatch`` (L4), ``worker``/``pipeline``
(L5), ``pipe`` (L6).  MI355X compute lives in ``mipipe.ops`` (hand-written
CDNA4 HIP kernels in ``mipipe/csrc``), models in ``mipipe.models`` and the
multi-process RCCL pipeline runtime in ``mipipe.parallel``.
"""
from .microbatch import NoChunk
from .pipe import BalanceError, Pipe, PipeSequential, WithDevice
from .rref import LocalRRef
from .checkpoint import checkpoint, is_checkpointing, is_recomputing
from .batchnorm import DeferredBatchNorm
from .skip import Namespace, pop, skippable, stash, verify_skippables

__all__ = [
    "Pipe",
    "BalanceError",
    "PipeSequential",
    "WithDevice",
    "NoChunk",
    "LocalRRef",
    "checkpoint",
    "is_checkpointing",
    "is_recomputing",
    "DeferredBatchNorm",
    "skippable",
    "stash",
    "pop",
    "Namespace",
    "verify_skippables",
]

__version__ = "0.1.0"
