"""GPipe clock schedule and the single-process pipeline executor.

``clock_cycles(m, n)`` yields, for tick ``k = 0 .. m+n-2``, the wavefront of cells
``(i, j)`` with ``i + j = k`` -- micro-batch ``i`` on partition ``j``
(``/root/reference/pipeline.py:63-79``).  Each tick is executed in two phases:

* **fence** -- for every cell: add the cross-micro-batch dependency that fixes
  the backward order (``i>0, j>0``: fork micro-batch ``i-1``'s current tensor and
  join it into micro-batch ``i``), copy skip tensors that this partition pops,
  and copy the activation from partition ``j-1`` on the per-(partition,
  micro-batch) copy streams.
* **compute** -- for every cell: make the compute stream wait for the copy,
  build a task (checkpointed or not), hand it to the device's worker thread;
  then collect the results in schedule order, make the copy stream wait for the
  compute stream, schedule recomputation and keep the *first* exception, which
  is re-raised after the tick has drained (``/root/reference/pipeline.py:239-266``).

Deliberate differences from the reference (documented in README.md):

* the checkpoint boundary is derived from the *actual* number of micro-batches,
  so ``except_last`` really leaves the last one un-checkpointed when ``chunk``
  produced fewer micro-batches than requested (the bug noted at
  ``/root/reference/README.md:398``);
* worker threads are joined when the pipeline is garbage-collected;
* ``MIPIPE_SYNC_DEBUG=1`` synchronises every device after each tick, which turns
  a missing stream wait into a deterministic failure (§5.2).
"""
from __future__ import annotations

import os
import weakref
from typing import Iterable, List, Optional, Sequence, Tuple, Union, cast

import torch
from torch import nn

from .checkpoint import Checkpointing
from .copy import Copy, Wait, transfer_policy
from .dependency import fork, join
from .microbatch import Batch
from .skip.layout import SkipLayout
from .skip.tracker import SkipTrackerThroughPortals, use_skip_tracker
from .stream import AbstractStream, current_stream, synchronize_all, use_device
from .worker import ExcInfo, Task, create_workers, release_workers

__all__ = ["Pipeline", "clock_cycles", "checkpoint_stop_for"]

Cell = Tuple[int, int]


def clock_cycles(m: int, n: int) -> Iterable[List[Cell]]:
    """Cells ``(micro-batch i, partition j)`` runnable at each clock tick.

    ::

        k   cells
        0   (0,0)
        1   (1,0) (0,1)
        2   (2,0) (1,1) (0,2)
        3         (2,1) (1,2)
        4               (2,2)      # m = 3, n = 3
    """
    for k in range(m + n - 1):
        first_j = max(0, k - m + 1)
        last_j = min(k, n - 1)
        yield [(k - j, j) for j in range(first_j, last_j + 1)]


# Kept for callers that use the upstream private name.
_clock_cycles = clock_cycles


def checkpoint_stop_for(checkpoint: Union[str, int], m: int) -> int:
    """Number of leading micro-batches to checkpoint for ``m`` micro-batches."""
    if isinstance(checkpoint, int):
        return min(checkpoint, m)
    if checkpoint == "always":
        return m
    if checkpoint == "except_last":
        return max(m - 1, 0)
    if checkpoint == "never":
        return 0
    raise ValueError(f"unknown checkpoint mode {checkpoint!r}")


def _detach_non_float(values) -> Tuple:
    # Gradients are only defined for floating-point tensors.
    return tuple(x.detach() if torch.is_tensor(x) and not x.is_floating_point() else x for x in values)


def _depend(fork_from: Batch, join_to: Batch) -> None:
    src = fork_from.find_tensor_idx()
    dst = join_to.find_tensor_idx()
    fork_from[src], phony = fork(fork_from[src])
    join_to[dst] = join(join_to[dst], phony)


def _copy(batch: Batch, prev_stream: AbstractStream, next_stream: AbstractStream) -> None:
    batch[:] = _detach_non_float(Copy.apply(prev_stream, next_stream, *batch))


def _wait(batch: Batch, prev_stream: AbstractStream, next_stream: AbstractStream) -> None:
    batch[:] = _detach_non_float(Wait.apply(prev_stream, next_stream, *batch))


class Pipeline:
    """Runs micro-batches through partitions with the GPipe schedule."""

    def __init__(
        self,
        partitions: Sequence[nn.Sequential],
        devices: Sequence[torch.device],
        copy_streams: Sequence[Sequence[AbstractStream]],
        skip_layout: SkipLayout,
        checkpoint_stop: Union[int, str],
        compute_streams: Optional[Sequence[Optional[AbstractStream]]] = None,
        copy_same_device: bool = False,
        copy_engine: Optional[str] = None,
    ) -> None:
        self.partitions = partitions
        self.devices = list(devices)
        self.copy_streams = copy_streams
        # per partition: None = the device's current stream at run time
        self.dedicated_streams: List[Optional[AbstractStream]] = (
            list(compute_streams) if compute_streams is not None else [None] * len(self.devices))
        self.copy_same_device = copy_same_device
        self.copy_engine = copy_engine
        self.skip_layout = skip_layout
        self.checkpoint = checkpoint_stop
        self.in_queues, self.out_queues, entries = create_workers(self.devices)
        self._finalizer = weakref.finalize(self, release_workers, entries)
        self.sync_debug = os.environ.get("MIPIPE_SYNC_DEBUG") == "1"

    # Upstream attribute name.
    @property
    def checkpoint_stop(self) -> Union[int, str]:
        return self.checkpoint

    def close(self) -> None:
        """Stops the worker threads (also done automatically at GC)."""
        self._finalizer()

    def run(self, batches: List[Batch]) -> None:
        """Runs all micro-batches; ``batches`` is updated in place with the outputs."""
        m = len(batches)
        n = len(self.partitions)
        stop = checkpoint_stop_for(self.checkpoint, m)
        # Evaluation never checkpoints (/root/reference/pipeline.py:153-155).
        if not self.partitions[0].training:
            stop = 0
        trackers = [SkipTrackerThroughPortals(self.skip_layout) for _ in batches]
        with transfer_policy(self.copy_same_device, self.copy_engine):
            for cells in clock_cycles(m, n):
                self.fence(batches, cells, trackers)
                self.compute(batches, cells, trackers, stop)
                if self.sync_debug:
                    synchronize_all(self.devices)
        last = self.dedicated_streams[n - 1]
        if last is not None:
            # The caller reads the output on the device's current stream.
            out_stream = current_stream(self.devices[n - 1])
            for batch in batches:
                _wait(batch, last, out_stream)

    def compute_streams(self) -> List[AbstractStream]:
        """The stream each partition computes on (for this thread)."""
        return [s if s is not None else current_stream(d) for s, d in zip(self.dedicated_streams, self.devices)]

    def fence(self, batches: List[Batch], cells: List[Cell], trackers: List[SkipTrackerThroughPortals]) -> None:
        """Dependencies and copies that must precede this tick's computation."""
        streams = self.copy_streams
        for i, j in cells:
            if i > 0 and j > 0:
                _depend(batches[i - 1], batches[i])

            next_stream = streams[j][i]
            for prev_j, ns, name in self.skip_layout.copy_policy(j):
                trackers[i].copy(batches[i], streams[prev_j][i], next_stream, ns, name)

            if j > 0:
                _copy(batches[i], streams[j - 1][i], next_stream)

    def compute(
        self,
        batches: List[Batch],
        cells: List[Cell],
        trackers: List[SkipTrackerThroughPortals],
        checkpoint_stop: Optional[int] = None,
    ) -> None:
        """Launches this tick's cells on the workers and collects the results."""
        partitions = self.partitions
        devices = self.devices
        copy_streams = self.copy_streams
        n = len(partitions)
        if checkpoint_stop is None:
            checkpoint_stop = checkpoint_stop_for(self.checkpoint, len(batches))
            if not partitions[0].training:
                checkpoint_stop = 0
        compute_streams = self.compute_streams()

        for i, j in cells:
            batch = batches[i]
            if j > 0:
                # [1] the compute stream waits for the copied input.
                _wait(batch, copy_streams[j][i], compute_streams[j])
            task = self._make_task(batch, partitions[j], trackers[i], compute_streams[j], i, j, i < checkpoint_stop)
            # [2] run on the device's worker.
            self.in_queues[j].put(task)

        first_error: Optional[ExcInfo] = None
        for i, j in cells:
            ok, payload = self.out_queues[j].get()
            if first_error is not None:
                continue
            if not ok:
                first_error = cast(ExcInfo, payload)
                continue
            task, batch = cast(Tuple[Task, Batch], payload)
            if j < n - 1:
                # [3] the copy stream waits for the compute stream's output.
                _wait(batch, compute_streams[j], copy_streams[j][i])
            # [4] hang recomputation off the graph for checkpointed cells.
            with use_device(devices[j]):
                task.finalize(batch)
            batches[i] = batch

        if first_error is not None:
            raise first_error[1].with_traceback(first_error[2])

    @staticmethod
    def _make_task(
        batch: Batch,
        partition: nn.Module,
        tracker: SkipTrackerThroughPortals,
        stream: AbstractStream,
        i: int,
        j: int,
        checkpointed: bool,
    ) -> Task:
        label = f"chunk{i}-part{j}"
        if checkpointed:

            def run_partition(*inputs, _partition=partition, _tracker=tracker):
                with use_skip_tracker(_tracker):
                    return _partition(*inputs)

            chk = Checkpointing(run_partition, batch)
            return Task(stream, compute=chk.checkpoint, finalize=chk.recompute, label=label)

        def compute(_batch=batch, _partition=partition, _tracker=tracker) -> Batch:
            with use_skip_tracker(_tracker):
                return _batch.call(_partition)

        return Task(stream, compute=compute, finalize=None, label=label)
