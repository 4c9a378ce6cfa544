"""Static routing of skip tensors between partitions.

``inspect_skip_layout(partitions)`` (called at ``/root/reference/pipe.py:348``)
records, for every ``(namespace, name)``, the partition that stashes it and the
partition that pops it.  ``copy_policy(j)`` then lists the skips partition ``j``
must receive at its fence (``/root/reference/pipeline.py:136-138``).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Tuple

from torch import nn

from .namespace import Namespace

__all__ = ["SkipLayout", "inspect_skip_layout"]

Key = Tuple[Optional[Namespace], str]


def _route_key(entry: Tuple[int, Optional[Namespace], str]):
    prev_j, ns, name = entry
    return (prev_j, -1 if ns is None else ns.id, name)


class SkipLayout:
    """Skip routes: ``(ns, name) -> (stash partition, pop partition)``."""

    def __init__(self, num_partitions: int, skip_routes: Dict[Key, Tuple[int, int]]) -> None:
        self.by_ns_name = dict(skip_routes)
        self.by_partition: List[List[Tuple[int, Optional[Namespace], str]]] = [[] for _ in range(num_partitions)]
        for (ns, name), (prev_j, next_j) in skip_routes.items():
            self.by_partition[next_j].append((prev_j, ns, name))
        for entries in self.by_partition:
            entries.sort(key=_route_key)

    def copy_policy(self, next_j: int) -> Iterable[Tuple[int, Optional[Namespace], str]]:
        """Skips to copy into partition ``next_j``: ``(prev_j, ns, name)``."""
        for prev_j, ns, name in self.by_partition[next_j]:
            if prev_j != next_j:
                yield prev_j, ns, name

    def requires_copy(self, ns: Optional[Namespace], name: str) -> bool:
        """Whether the skip crosses a partition boundary (i.e. needs a portal)."""
        prev_j, next_j = self.by_ns_name.get((ns, name), (-1, -1))
        return prev_j != next_j


def inspect_skip_layout(partitions: List[nn.Sequential]) -> SkipLayout:
    from .skippable import Skippable

    routes: Dict[Key, Tuple[int, int]] = {}
    stashed_at: Dict[Key, int] = {}

    def visit(layer: nn.Module, j: int) -> None:
        if not isinstance(layer, Skippable):
            return
        for key in layer.stashable():
            stashed_at[key] = j
        for key in layer.poppable():
            routes[key] = (stashed_at.pop(key), j)

    for j, partition in enumerate(partitions):
        if isinstance(partition, nn.Sequential):
            for layer in partition:
                visit(layer, j)
        else:
            visit(partition, j)

    return SkipLayout(len(partitions), routes)
