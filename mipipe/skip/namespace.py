"""Namespaces that keep repeated skip names apart.

Two instances of the same ``@skippable`` class stash under the same *name*;
``layer.isolate(Namespace())`` gives each pair its own key ``(ns, name)``.
"""
from __future__ import annotations

import itertools
from typing import Any, Optional

__all__ = ["Namespace"]

_ids = itertools.count()


class Namespace:
    """An opaque, totally ordered, hashable token."""

    __slots__ = ("id", "label")

    def __init__(self, label: Optional[str] = None) -> None:
        self.id = next(_ids)
        # A label names the namespace the same way in every process: the
        # multi-process engine keys cross-stage skips by it (ids depend on
        # construction order).  Labels must be unique within a model.
        self.label = label

    def __repr__(self) -> str:
        return f"<Namespace '{self.label if self.label is not None else self.id}'>"

    def __hash__(self) -> int:
        return hash(("mipipe.Namespace", self.id))

    # Ordering lets skip routes be sorted deterministically (None < Namespace).
    def __lt__(self, other: Any) -> bool:
        if isinstance(other, Namespace):
            return self.id < other.id
        return False

    def __eq__(self, other: Any) -> bool:
        return isinstance(other, Namespace) and self.id == other.id
