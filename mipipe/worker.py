"""Per-device worker threads that launch partition work.

Behaviour (``/root/reference/README.md:36-47,291-314``): one daemon thread per
*unique* device pulls :class:`Task` objects from its in-queue, runs
``task.compute()`` with that device current, and posts ``(True, (task, batch))``
or ``(False, exc_info)``; a ``None`` task stops the thread.

Differences from the reference:

* workers are reference-counted and shut down (joined) when the last pipeline
  using them is garbage-collected, instead of leaking daemons forever;
* when the native runtime is loaded every task is bracketed by a
  ``roctxRangePush("chunk{i}-part{j}")`` range so rocprofv3 timelines show the
  pipeline cells (the reference removed its ``record_function`` labels,
  ``/root/reference/pipeline.py:205-210``).
"""
from __future__ import annotations

import sys
import threading
from contextlib import contextmanager
from queue import Queue
from types import TracebackType
from typing import Callable, Dict, List, Optional, Tuple, Type, Union, cast

import torch

from .microbatch import Batch
from .stream import AbstractStream, _native, use_device, use_stream

__all__ = ["Task", "worker", "create_workers", "release_workers", "label_range"]

ExcInfo = Tuple[Type[BaseException], BaseException, TracebackType]
InQueue = Queue
OutQueue = Queue


@contextmanager
def label_range(label: Optional[str]):
    """roctx range around a block when profiling is possible, else a no-op."""
    rt = _native() if label else None
    if rt is None:
        yield
        return
    rt.range_push(label)
    try:
        yield
    finally:
        rt.range_pop()


class Task:
    """A unit of partition work bound to a stream.

    ``compute`` runs on a worker thread; ``finalize`` runs on the scheduling
    thread after the result is collected (it schedules recomputation).
    The grad mode of the creating thread is captured and re-applied.
    """

    __slots__ = ("stream", "_compute", "_finalize", "_grad_enabled", "label")

    def __init__(
        self,
        stream: AbstractStream,
        *,
        compute: Callable[[], Batch],
        finalize: Optional[Callable[[Batch], None]],
        label: Optional[str] = None,
    ) -> None:
        self.stream = stream
        self._compute = compute
        self._finalize = finalize
        self._grad_enabled = torch.is_grad_enabled()
        self.label = label

    def compute(self) -> Batch:
        with use_stream(self.stream), torch.set_grad_enabled(self._grad_enabled), label_range(self.label):
            return self._compute()

    def finalize(self, batch: Batch) -> None:
        if self._finalize is None:
            return
        with use_stream(self.stream), torch.set_grad_enabled(self._grad_enabled):
            self._finalize(batch)


def worker(in_queue: InQueue, out_queue: OutQueue, device: torch.device) -> None:
    """Main loop of a worker thread."""
    with use_device(device):
        while True:
            task = in_queue.get()
            if task is None:
                break
            try:
                batch = task.compute()
            except Exception:
                out_queue.put((False, sys.exc_info()))
                continue
            out_queue.put((True, (task, batch)))
    # Tell whoever is listening that this worker is gone.
    out_queue.put((False, None))


def _normalize_device(device: torch.device) -> torch.device:
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        return torch.device("cuda", index=torch.cuda.current_device())
    if device.type == "cpu" and device.index is not None:
        return torch.device("cpu")
    return device


class _WorkerEntry:
    __slots__ = ("in_queue", "out_queue", "thread", "refs")

    def __init__(self, device: torch.device) -> None:
        self.in_queue: InQueue = Queue()
        self.out_queue: OutQueue = Queue()
        self.thread = threading.Thread(
            target=worker,
            args=(self.in_queue, self.out_queue, device),
            name=f"mipipe-worker-{device}",
            daemon=True,
        )
        self.thread.start()
        self.refs = 0


_registry_lock = threading.Lock()
# Workers are private to each ``create_workers`` call: two pipelines on the same
# device must not consume each other's results from a shared out-queue.


def create_workers(devices: List[torch.device]) -> Tuple[List[InQueue], List[OutQueue], List[_WorkerEntry]]:
    """Spawns one worker per unique device; returns per-partition queues."""
    entries: Dict[torch.device, _WorkerEntry] = {}
    in_queues: List[InQueue] = []
    out_queues: List[OutQueue] = []
    with _registry_lock:
        for device in devices:
            device = _normalize_device(device)
            entry = entries.get(device)
            if entry is None:
                entry = _WorkerEntry(device)
                entries[device] = entry
            entry.refs += 1
            in_queues.append(entry.in_queue)
            out_queues.append(entry.out_queue)
    return in_queues, out_queues, list(entries.values())


def release_workers(entries: List[_WorkerEntry], timeout: float = 5.0) -> None:
    """Stops the given workers and joins them."""
    for entry in entries:
        entry.in_queue.put(None)
    for entry in entries:
        if entry.thread is not threading.current_thread():
            entry.thread.join(timeout)
