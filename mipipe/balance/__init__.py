"""Automatic partition balancing.

Upstream ``torch.distributed.pipeline.sync.balance`` -- recommended by the
reference's dead helper ``_recommend_auto_balance`` (``/root/reference/pipe.py:42-58``)::

    from mipipe.balance import balance_by_time
    balance = balance_by_time(torch.cuda.device_count(), model, sample)
    model = mipipe.utils.partition_model(model, balance)
    pipe = mipipe.Pipe(model, chunks=8)

Also :func:`balance_by_cost` for analytic costs (e.g. FLOPs from
``mipipe.models``) -- what the multi-process benchmark uses, since profiling a
1.2B-parameter model layer by layer is slower than counting its FLOPs.
"""
from __future__ import annotations

from typing import Any, List, Sequence, Union

import torch
from torch import Tensor, nn

from . import blockpartition
from .profile import profile_sizes, profile_times

__all__ = ["balance_by_time", "balance_by_size", "balance_by_cost", "balance_cost"]

Device = Union[torch.device, int, str]


def balance_cost(cost: Sequence[float], partitions: int) -> List[int]:
    """Balance (layers per partition) minimising the largest partition cost."""
    return blockpartition.solve_balance(list(cost), partitions)


balance_by_cost = balance_cost


def _default_device() -> torch.device:
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def balance_by_time(
    partitions: int,
    module: nn.Sequential,
    sample: Union[List[Any], Tensor],
    *,
    timeout: float = 1.0,
    device: Device = None,  # type: ignore[assignment]
) -> List[int]:
    """Balance by measured per-layer forward+backward time.

    ``sample`` is a representative *micro*-batch.  Raises ``ValueError`` if the
    module already has gradients (the profile runs backward on copies).
    """
    device = torch.device(device) if device is not None else _default_device()
    times = profile_times(module, sample, timeout, device)
    return balance_cost(times, partitions)


def balance_by_size(
    partitions: int,
    module: nn.Sequential,
    input: Union[List[Any], Tensor],
    *,
    chunks: int = 1,
    param_scale: float = 2.0,
    device: Device = None,  # type: ignore[assignment]
) -> List[int]:
    """Balance by per-layer memory (activations + ``param_scale`` x parameters).

    ``param_scale`` 2 covers weights+grads; 4 also covers Adam's two moments.
    """
    device = torch.device(device) if device is not None else torch.device("cuda")
    sizes = profile_sizes(module, input, chunks, param_scale, device)
    return balance_cost(sizes, partitions)
