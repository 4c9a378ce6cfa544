"""``partition_model`` (upstream ``torch.distributed.pipeline.sync.utils``).

Groups the children of a flat ``nn.Sequential`` according to ``balance`` and
moves each group to its device, producing the nested Sequential that
:class:`~mipipe.Pipe` splits one partition per group.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import torch
from torch import nn

__all__ = ["partition_model"]

Device = Union[torch.device, int, str]


def partition_model(
    module: nn.Sequential,
    balance: Sequence[int],
    devices: Optional[Sequence[Device]] = None,
) -> nn.Sequential:
    """Returns ``nn.Sequential(group_0, group_1, ...)`` with group ``k`` holding
    ``balance[k]`` consecutive layers on ``devices[k]`` (``cuda:k`` by default).
    """
    from ..pipe import BalanceError

    if sum(balance) != len(module):
        raise BalanceError(f"module and sum of balance have different length (module: {len(module)}, sum of balance: {sum(balance)})")
    if any(b <= 0 for b in balance):
        raise BalanceError(f"all balance numbers must be positive integer (balance: {list(balance)})")
    if devices is None:
        devices = [torch.device("cuda", k) for k in range(len(balance))]
    elif len(devices) < len(balance):
        raise IndexError(f"too few devices to hold given partitions (devices: {len(devices)}, partitions: {len(balance)})")

    layers = list(module.children())
    groups: List[nn.Module] = []
    start = 0
    for k, count in enumerate(balance):
        group = nn.Sequential(*layers[start : start + count])
        group.to(torch.device(devices[k]))
        groups.append(group)
        start += count
    return nn.Sequential(*groups)
