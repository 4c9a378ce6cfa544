"""Namespaces that keep repeated skip names apart.

Two instances of the same ``@skippable`` class stash under the same *name*;
``layer.isolate(Namespace())`` gives each pair its own key ``(ns, name)``.
"""
from __future__ import annotations

import itertools
from typing import Any

__all__ = ["Namespace"]

_ids = itertools.count()


class Namespace:
    """An opaque, totally ordered, hashable token."""

    __slots__ = ("id",)

    def __init__(self) -> None:
        self.id = next(_ids)

    def __repr__(self) -> str:
        return f"<Namespace '{self.id}'>"

    def __hash__(self) -> int:
        return hash(("mipipe.Namespace", self.id))

    # Ordering lets skip routes be sorted deterministically (None < Namespace).
    def __lt__(self, other: Any) -> bool:
        if isinstance(other, Namespace):
            return self.id < other.id
        return False

    def __eq__(self, other: Any) -> bool:
        return isinstance(other, Namespace) and self.id == other.id
