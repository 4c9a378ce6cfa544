"""Skip trackers: where stashed tensors wait for their pop.

* :class:`SkipTracker` -- plain dict; used outside pipelines and for skips whose
  stash and pop land in the same partition.
* :class:`SkipTrackerThroughPortals` -- one per micro-batch inside a pipeline
  (``/root/reference/pipeline.py:113``); cross-partition skips go through
  :class:`~mipipe.skip.portal.Portal` so they bypass the intermediate stages and
  are copied exactly once, stash device -> pop device, at the pop partition's
  fence (``/root/reference/pipeline.py:136-138``).

The tracker for the running task is found through a thread-local set by
:func:`use_skip_tracker` (``/root/reference/pipeline.py:208,228``).

Attribution: the portal design (three autograd functions on the phony chain,
the 3-vs-2 forward-user tensor life, PortalCopy reusing Copy's forward /
backward) follows upstream PyTorch's torch.distributed.pipeline.sync.skip
(BSD-3-Clause, originally from torchgpipe); this file re-implements that
behaviour, which SURVEY.md C14 requires bit-for-bit.
"""
from __future__ import annotations

import threading
from contextlib import contextmanager
from typing import Dict, Generator, Optional, Tuple

from torch import Tensor

from ..checkpoint import is_checkpointing
from ..dependency import fork, join
from ..microbatch import Batch
from ..stream import AbstractStream, current_stream, record_stream
from .layout import SkipLayout
from .namespace import Namespace
from .portal import Portal

__all__ = [
    "SkipTracker",
    "SkipTrackerThroughPortals",
    "SkipTrackerThroughPotals",
    "use_skip_tracker",
    "current_skip_tracker",
]

Key = Tuple[Optional[Namespace], str]


class SkipTracker:
    """In-memory stash for skip tensors that stay on one device."""

    def __init__(self) -> None:
        self.tensors: Dict[Key, Optional[Tensor]] = {}

    def save(self, batch: Batch, ns: Optional[Namespace], name: str, tensor: Optional[Tensor]) -> None:
        self.tensors[(ns, name)] = tensor

    def load(self, batch: Batch, ns: Optional[Namespace], name: str) -> Optional[Tensor]:
        return self.tensors.pop((ns, name))

    def copy(
        self, batch: Batch, prev_stream: AbstractStream, next_stream: AbstractStream, ns: Optional[Namespace], name: str
    ) -> None:
        raise TypeError("copy is not supported for non-portal skip tensors")


class SkipTrackerThroughPortals(SkipTracker):
    """Routes cross-partition skips through portals."""

    def __init__(self, skip_layout: SkipLayout) -> None:
        super().__init__()
        self.skip_layout = skip_layout
        self.portals: Dict[Key, Portal] = {}

    def save(self, batch: Batch, ns: Optional[Namespace], name: str, tensor: Optional[Tensor]) -> None:
        if not self.skip_layout.requires_copy(ns, name):
            super().save(batch, ns, name, tensor)
            return

        # Forward users of the portal's tensor, in order:
        #   blue() at the stash            (1)
        #   orange() at the pop            (2)
        #   orange() again when the pop partition is recomputed  (3, checkpointed only)
        # and when the stash partition is itself recomputed its save() comes
        # back here with an existing portal; that tensor only serves blue().
        portal = self.portals.get((ns, name))
        if portal is None:
            portal = Portal(tensor, 3 if is_checkpointing() else 2)
            self.portals[(ns, name)] = portal
        else:
            portal.put_tensor(tensor, 1)

        phony = portal.blue()
        idx = batch.find_tensor_idx()
        batch[idx] = join(batch[idx], phony)

    def load(self, batch: Batch, ns: Optional[Namespace], name: str) -> Optional[Tensor]:
        if not self.skip_layout.requires_copy(ns, name):
            return super().load(batch, ns, name)
        portal = self.portals[(ns, name)]
        idx = batch.find_tensor_idx()
        batch[idx], phony = fork(batch[idx])
        tensor = portal.orange(phony)
        if tensor is not None and tensor.is_cuda:
            # popped on this partition's compute stream, which may not be the
            # stream the portal copy recorded (a dedicated same-GPU stage stream)
            record_stream(tensor, current_stream(tensor.device))
        return tensor

    def copy(
        self, batch: Batch, prev_stream: AbstractStream, next_stream: AbstractStream, ns: Optional[Namespace], name: str
    ) -> None:
        assert self.skip_layout.requires_copy(ns, name)
        idx = batch.find_tensor_idx()
        batch[idx], phony = fork(batch[idx])
        portal = self.portals[(ns, name)]
        phony = portal.copy(prev_stream, next_stream, phony)
        batch[idx] = join(batch[idx], phony)


# Upstream spelling kept as an alias for drop-in compatibility.
SkipTrackerThroughPotals = SkipTrackerThroughPortals


class _Local(threading.local):
    def __init__(self) -> None:
        self.tracker: Optional[SkipTracker] = None


_local = _Local()


@contextmanager
def use_skip_tracker(tracker: SkipTracker) -> Generator[None, None, None]:
    prev = _local.tracker
    _local.tracker = tracker
    try:
        yield
    finally:
        _local.tracker = prev


def current_skip_tracker() -> SkipTracker:
    """The active tracker, or a fresh thread-local plain one outside pipelines."""
    tracker = _local.tracker
    if tracker is None:
        tracker = SkipTracker()
        _local.tracker = tracker
    return tracker
