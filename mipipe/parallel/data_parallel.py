"""Data parallelism across pipeline replicas: bucketed gradient all-reduce over RCCL.

The reference is pipeline-only; its docstring allows wrapping a ``Pipe`` in
DDP when ``checkpoint='never'`` (``/root/reference/pipe.py:290-293``, SURVEY
§2.5).  ``mipipe.Pipe`` keeps that interop (``tests/test_data_parallel.py``
wraps it in DDP).  For the multi-process engine this module is the MI355X-
native form: ``dp`` replicas of a ``pp``-stage pipeline, ``world = pp * dp``
ranks, each stage's gradients averaged over its ``dp`` replicas.

Design for the hardware rather than DDP's per-parameter hooks:

* the gradients already live in ONE fp32 ``main_grad`` buffer per device
  (:class:`mipipe.optim.FlatAdam`), so a bucket is a contiguous slice of it
  (no packing copies) and the all-reduce reduces in fp32 (no bf16 rounding of
  the summed gradient);
* buckets are large (default 256 MiB): an 8-GPU MI355X node is fully
  connected by xGMI (7 links x ~153 GB/s per GPU), and RCCL's ring/direct
  algorithms are link-bound, so fewer, larger collectives beat many small ones;
* overlap comes from the deferred weight gradients: the engine's backward
  computes only input gradients and queues the weight-gradient GEMMs, which
  run at the end of the rank's backward (``ops.deferred_wgrad``).  A bucket's
  all-reduce is issued the moment its last weight-gradient GEMM is queued --
  so it runs on the RCCL stream while the remaining GEMMs run on the compute
  stream -- and buckets whose gradients were final before the flush (LayerNorm,
  biases, embedding) go first;
* averaging is free: the engine seeds its backward with
  ``loss / (chunks * dp)`` (``PipelineEngine(grad_divisor=dp)``), so the
  all-reduce SUM is already the mean.

Process-group layout (:func:`make_pp_dp_groups`): replica ``d`` owns global
ranks ``d*pp .. d*pp+pp-1`` (stage ``s`` on rank ``d*pp+s``); every pair of
ranks has its own xGMI link, so the layout only has to be consistent.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

from ..ops.linear import add_wgrad_listener, remove_wgrad_listener
from .p2p import Channels

__all__ = ["DataParallelGrads", "make_pp_dp_groups", "PPDPGroups"]


class DataParallelGrads:
    """All-reduces the ``main_grad`` buffers of a :class:`~mipipe.optim.FlatAdam`
    over ``group`` in contiguous buckets, overlapped with the deferred
    weight-gradient GEMMs.

    Use per step::

        dpg.begin()            # before the engine step (registers the flush hook)
        engine.step(...)
        dpg.finish()           # issues what is left, makes the stream wait for all

    ``average``: divide by the group size after the reduction (not needed when
    the loss was already scaled by ``1/dp``, e.g. ``PipelineEngine(grad_divisor=dp)``).
    """

    def __init__(self, optimizer, group: Optional[dist.ProcessGroup] = None, bucket_mb: float = 256.0,
                 average: bool = False) -> None:
        self.opt = optimizer
        self.group = group
        self.world = dist.get_world_size(group)
        self.average = average
        limit = max(int(bucket_mb * 2**20) // 4, 1)  # fp32 elements per bucket
        self.buckets: List[Tensor] = []
        self._members: List[List] = []
        self._bucket_of: Dict[int, int] = {}
        for g in optimizer.groups:
            start = off = 0
            members: List = []
            for p in g.params:
                members.append(p)
                self._bucket_of[id(p)] = len(self.buckets)
                off += p.numel()
                if off - start >= limit:
                    self._close(g.main_grad, start, off, members)
                    start, members = off, []
            if members:
                self._close(g.main_grad, start, off, members)
        self._left: List[int] = []
        self._works: List = []
        self._issued: List[bool] = []
        self._active = False

    def _close(self, flat: Tensor, start: int, end: int, members: List) -> None:
        self.buckets.append(flat[start:end])
        self._members.append(members)

    @property
    def bucket_sizes_mb(self) -> List[float]:
        return [b.numel() * 4 / 2**20 for b in self.buckets]

    # ------------------------------------------------------------------ step
    def begin(self) -> None:
        """Arms the buckets for one step and hooks the weight-gradient flush."""
        if self._active:
            raise RuntimeError("DataParallelGrads.begin() called twice without finish()")
        self._left = [len(m) for m in self._members]
        self._issued = [False] * len(self.buckets)
        self._works = []
        self._active = True
        add_wgrad_listener(self)

    def _ready(self, p) -> None:
        b = self._bucket_of.get(id(p))
        if b is None or self._issued[b]:
            return
        self._left[b] -= 1
        if self._left[b] == 0:
            self._issue(b)

    def _issue(self, b: int) -> None:
        self._issued[b] = True
        self._works.append((b, dist.all_reduce(self.buckets[b], group=self.group, async_op=True)))

    # flush listener (mipipe.ops.linear.flush_wgrad)
    def flush_begin(self, pending) -> None:
        """The rank's backward is over: every parameter without a queued
        weight-gradient GEMM and without an autograd ``.grad`` to fold has its
        final main_grad now."""
        queued = {id(w) for w in pending}
        for members in self._members:
            for p in members:
                if id(p) in queued or p.grad is not None:
                    continue
                if getattr(p, "_mg_fresh", False):  # lazily zeroed, written by nothing this step
                    p.main_grad.zero_()
                    p._mg_fresh = False
                self._ready(p)

    def wgrad_done(self, w) -> None:
        self._ready(w)

    def finish(self) -> None:
        """Folds autograd ``.grad`` leftovers, issues every bucket not yet issued
        (in bucket order, identical on every replica) and makes the current
        stream wait for all reductions."""
        if not self._active:
            raise RuntimeError("DataParallelGrads.finish() without begin()")
        remove_wgrad_listener(self)
        self._active = False
        self.opt.fold_grads()
        for b in range(len(self.buckets)):
            if not self._issued[b]:
                self._issue(b)
        for b, w in self._works:
            w.wait()
            if self.average:
                self.buckets[b].div_(self.world)
        self._works = []

    def abort(self) -> None:
        """Unhooks after a failed step (the reductions issued so far are left to the process group)."""
        remove_wgrad_listener(self)
        self._active = False


class PPDPGroups:
    """Process groups of a ``pp`` x ``dp`` layout, from this rank's view."""

    def __init__(self, pp: int, dp: int, channels: Channels, pipeline_group, dp_group, replica: int, stage: int):
        self.pp, self.dp = pp, dp
        self.channels = channels          # this replica's pipeline links
        self.pipeline_group = pipeline_group  # this replica's ranks (grad-norm all-reduce)
        self.dp_group = dp_group          # the ranks holding the same stage (gradient all-reduce)
        self.replica, self.stage = replica, stage


def make_pp_dp_groups(pp: int, dp: int, wrap: bool = False, *, transport: str = "rccl",
                      ipc_options: Optional[dict] = None) -> PPDPGroups:
    """Creates every pipeline's channels, every pipeline group and every
    data-parallel group (``dist.new_group`` is collective: all ranks create all
    of them, in one order) and returns this rank's.  ``transport="ipc"``
    builds :class:`~mipipe.parallel.ipc.IpcChannels` (``ipc_options`` needs
    ``device`` and ``recv_bytes``) instead of RCCL channels."""
    world = dist.get_world_size()
    if pp * dp != world:
        raise ValueError(f"pp {pp} x dp {dp} != world size {world}")
    me = dist.get_rank()
    replica, stage = divmod(me, pp)
    mine_ch = mine_pg = mine_dg = None
    for d in range(dp):
        ranks = list(range(d * pp, (d + 1) * pp))
        if transport == "ipc":
            from .ipc import IpcChannels

            ch = IpcChannels(ranks, wrap=wrap and pp > 1, **(ipc_options or {}))
        else:
            ch = Channels(ranks, wrap=wrap and pp > 1)
        if d == replica:
            mine_ch = ch
    for d in range(dp):
        g = dist.new_group(list(range(d * pp, (d + 1) * pp)))
        if d == replica:
            mine_pg = g
    for s in range(pp):
        g = dist.new_group([d * pp + s for d in range(dp)])
        if s == stage:
            mine_dg = g
    return PPDPGroups(pp, dp, mine_ch, mine_pg, mine_dg, replica, stage)
