"""Point-to-point transport between pipeline ranks over RCCL:
the engine's ``transport="rccl"`` and the common fall-back of ``"auto"``.

On ROCm the ``nccl`` backend of ``torch.distributed`` *is* RCCL; between two
MI355X GPUs of a node a send/recv pair moves over the single xGMI link that
joins them (every GPU pair has its own link, so stage placement order does not
matter).  Receives are posted ahead of use so transfers overlap compute; a
received tensor is made usable on the current compute stream by
``Work.wait()`` (a stream wait, not a host block).

With the ``gloo`` backend (CPU tests, or several ranks sharing one GPU, which
RCCL refuses) device tensors are staged through host memory: the send copies
to a host buffer, the receive lands in one and ``wait()`` copies it to the
device tensor.  That path is for testing the engine, not for speed.
"""
from __future__ import annotations

import os
import warnings
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

__all__ = ["P2P", "Channels", "DirectLinks", "exchange_shape", "MIN_HW_QUEUES", "check_hw_queues"]

# Hardware queues a pipeline rank wants: the compute stream plus one per RCCL
# communicator stream (4 channel directions, the grad-norm all-reduce, skip
# links), each on a queue of its own.
MIN_HW_QUEUES = 16


def check_hw_queues() -> bool:
    """Warns when HIP will put RCCL streams on shared hardware queues.

    HIP maps streams onto ``GPU_MAX_HW_QUEUES`` in-order hardware queues
    (default 4).  Two streams on one queue run their kernels in submission
    order, so a pre-posted receive -- a kernel that spins until the peer's data
    arrives -- holds back every kernel queued behind it: the pipeline loses its
    overlap, and a looping pipeline (rank 0 receiving from rank n-1) can
    deadlock.  ``tools/micro/queue_share*.py`` measure this on the box
    (``profiles/hw_queue_sharing.txt``).  The variable is read when HIP
    initialises: set it before the process touches the GPU, as ``bench.py``
    does."""
    try:
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    except ValueError:
        q = 4
    if q < MIN_HW_QUEUES:
        warnings.warn(f"mipipe: GPU_MAX_HW_QUEUES={q}: RCCL communicator streams may share in-order hardware "
                      f"queues with the compute stream, and a pre-posted receive then blocks compute (lost overlap "
                      f"or deadlock); export GPU_MAX_HW_QUEUES={MIN_HW_QUEUES} before the process initialises HIP",
                      RuntimeWarning, stacklevel=3)
        return False
    return True


class _HostStagedWork:
    """Work handle of a host-staged transfer; ``wait()`` completes the device copy."""

    def __init__(self, work: dist.Work, host: Tensor, dst: Optional[Tensor] = None) -> None:
        self.work, self.host, self.dst = work, host, dst

    def wait(self) -> bool:
        self.work.wait()
        if self.dst is not None:
            self.dst.copy_(self.host)
            self.dst = None
        return True

    def is_completed(self) -> bool:
        return self.work.is_completed()


class P2P:
    """Sends/receives tensors to/from neighbour ranks of a process group."""

    def __init__(self, group: Optional[dist.ProcessGroup] = None) -> None:
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.host_staged = dist.get_backend(group) == "gloo"

    def global_rank(self, group_rank: int) -> int:
        if self.group is None:
            return group_rank
        return dist.get_global_rank(self.group, group_rank)

    def _meta_device(self, device: torch.device) -> torch.device:
        return torch.device("cpu") if self.host_staged else device

    def isend(self, t: Tensor, dst: int):
        if self.host_staged and t.device.type != "cpu":
            host = t.detach().to("cpu")
            return _HostStagedWork(dist.isend(host, self.global_rank(dst), group=self.group), host)
        return dist.isend(t.contiguous(), self.global_rank(dst), group=self.group)

    def irecv(self, t: Tensor, src: int):
        if self.host_staged and t.device.type != "cpu":
            host = torch.empty(t.shape, dtype=t.dtype)
            return _HostStagedWork(dist.irecv(host, self.global_rank(src), group=self.group), host, t)
        return dist.irecv(t, self.global_rank(src), group=self.group)

    def send_obj_shape(self, shape: Sequence[int], dtype_code: int, dst: int, device: torch.device) -> None:
        meta = torch.tensor([len(shape), dtype_code, *shape] + [0] * (8 - len(shape)), dtype=torch.int64,
                            device=self._meta_device(device))
        dist.send(meta, self.global_rank(dst), group=self.group)

    def recv_obj_shape(self, src: int, device: torch.device) -> Tuple[List[int], int]:
        meta = torch.empty(10, dtype=torch.int64, device=self._meta_device(device))
        dist.recv(meta, self.global_rank(src), group=self.group)
        m = meta.tolist()
        n = m[0]
        return m[2 : 2 + n], m[1]


class Channels:
    """One process group per DIRECTION of every pipeline link.

    RCCL (like NCCL) gives each rank pair one communicator and one stream, and
    runs that stream's sends and receives in issue order.  With activations
    flowing one way and gradients the other -- and, for looping placements,
    activations flowing back from the last rank to the first -- sharing that
    stream would couple the two directions (a pre-posted receive would hold
    back a send queued behind it).  A 2-rank group per direction gives every
    direction its own communicator and stream, so the only ordering rule left
    is per channel: the receiver posts in the order the sender sends.

    For pipeline rank ``r`` of ``n``: ``act_out`` (r -> r+1), ``act_in``
    (r-1 -> r), ``grad_out`` (r -> r-1), ``grad_in`` (r+1 -> r); indices mod n,
    the wrap-around links (n-1 -> 0 for activations, 0 -> n-1 for gradients)
    only exist when ``wrap`` (looping placement).  Every process of the default
    group must construct Channels for every pipeline, in the same order
    (``dist.new_group`` is collective).
    """

    def __init__(self, ranks: Sequence[int], wrap: bool = False) -> None:
        self.ranks = list(ranks)  # global ranks of the pipeline, in stage order
        n = len(self.ranks)
        me = dist.get_rank()
        self.rank = self.ranks.index(me) if me in self.ranks else -1
        self.world = n
        self.host_staged = dist.get_backend() == "gloo"
        if not self.host_staged and n > 1:
            check_hw_queues()
        fwd, bwd = {}, {}
        links = range(n) if wrap and n > 1 else range(n - 1)
        for r in links:
            a, b = self.ranks[r], self.ranks[(r + 1) % n]
            fwd[r] = (dist.new_group([a, b]) if n > 1 else None, a, b)  # activations a -> b
        for r in links:
            a, b = self.ranks[r], self.ranks[(r + 1) % n]
            bwd[r] = (dist.new_group([a, b]) if n > 1 else None, b, a)  # gradients b -> a
        self._fwd, self._bwd = fwd, bwd
        self.warmed = set()

    def warmup(self, device: torch.device) -> None:
        """Creates every channel's communicator up front.

        RCCL builds a pair's communicator lazily, host-blocking, on the first
        send/recv.  A looping pipeline pre-posts rank 0's receive from rank
        n-1 before rank 0 has computed anything, so a lazy init there would
        wait on a send that can never happen.  Here every link does one tiny
        blocking exchange, links visited in the same global order on every
        rank (a chain of pairwise rendezvous: always deadlock-free)."""
        import time

        dev = torch.device("cpu") if self.host_staged else device
        me = dist.get_rank()
        t0 = time.perf_counter()
        for table in (self._fwd, self._bwd):
            for r in sorted(table):
                group, src, dst = table[r]
                if me == src:
                    dist.send(torch.zeros(1, device=dev), dst, group=group)
                elif me == dst:
                    dist.recv(torch.zeros(1, device=dev), src, group=group)
                else:
                    continue
                self.warmed.add((table is self._fwd, r))
        self.warmup_s = time.perf_counter() - t0

    warmed: set = frozenset()  # (is_activation_link, link index) this rank exchanged over in warmup()
    warmup_s = None

    def comm_info(self) -> List[dict]:
        """This rank's channels as the communicators report them: direction,
        global (src, dst), the group's backend and ``get_world_size`` (2 for a
        live pair communicator), whether :meth:`warmup` exchanged over it."""
        me = dist.get_rank()
        out = []
        for kind, table in (("act", self._fwd), ("grad", self._bwd)):
            for r in sorted(table):
                group, src, dst = table[r]
                if me not in (src, dst) or group is None:
                    continue
                out.append({"dir": f"{kind} {src}->{dst}", "backend": str(dist.get_backend(group)),
                            "group_world": dist.get_world_size(group), "group_rank": dist.get_rank(group),
                            "warmed": (table is self._fwd, r) in self.warmed})
        return out

    def _link(self, table, r):
        return table.get(r % self.world) if self.world > 1 else None

    def _send(self, link, t: Tensor):
        group, _, dst = link
        if self.host_staged and t.device.type != "cpu":
            host = t.detach().to("cpu")
            return _HostStagedWork(dist.isend(host, dst, group=group), host)
        return dist.isend(t.detach().contiguous(), dst, group=group)

    def _recv(self, link, t: Tensor):
        group, src, _ = link
        if self.host_staged and t.device.type != "cpu":
            host = torch.empty(t.shape, dtype=t.dtype)
            return _HostStagedWork(dist.irecv(host, src, group=group), host, t)
        return dist.irecv(t, src, group=group)

    def send_act(self, t: Tensor):
        return self._send(self._link(self._fwd, self.rank), t)

    def recv_act(self, t: Tensor):
        return self._recv(self._link(self._fwd, self.rank - 1), t)

    def send_grad(self, t: Tensor):
        return self._send(self._link(self._bwd, self.rank - 1), t)

    def recv_grad(self, t: Tensor):
        return self._recv(self._link(self._bwd, self.rank), t)


class DirectLinks:
    """One communicator per DIRECTED pipeline-rank pair ``(src, dst)`` of ``pairs``.

    Carries cross-stage skip tensors (``@skippable`` stash -> pop) straight
    from the stashing rank to the popping rank, and their gradients back.
    Every MI355X of a node has its own xGMI link to every other, so a skip
    from stage 0 to stage 3 is one hop on a link the activation traffic does
    not use, not a relay through stages 1 and 2 (the reference's portals do
    the same with one peer copy, ``/root/reference/pipeline.py:136-138``).
    One communicator per direction for the reason given in :class:`Channels`.
    Every process of the default group constructs the same DirectLinks in
    the same order (``dist.new_group`` is collective)."""

    def __init__(self, ranks: Sequence[int], pairs: Sequence[Tuple[int, int]]) -> None:
        self.ranks = list(ranks)
        self.host_staged = dist.get_backend() == "gloo"
        self._links = {}
        for src, dst in sorted(set(pairs)):
            a, b = self.ranks[src], self.ranks[dst]
            self._links[(src, dst)] = (dist.new_group(sorted([a, b])), a, b)

    def warmup(self, device: torch.device) -> None:
        """Eager communicator creation, pairs in one global order (see :meth:`Channels.warmup`)."""
        dev = torch.device("cpu") if self.host_staged else device
        me = dist.get_rank()
        for key in sorted(self._links):
            group, src, dst = self._links[key]
            if me == src:
                dist.send(torch.zeros(1, device=dev), dst, group=group)
            elif me == dst:
                dist.recv(torch.zeros(1, device=dev), src, group=group)

    def send(self, src: int, dst: int, t: Tensor):
        group, _, gdst = self._links[(src, dst)]
        if self.host_staged and t.device.type != "cpu":
            host = t.detach().to("cpu")
            return _HostStagedWork(dist.isend(host, gdst, group=group), host)
        return dist.isend(t.detach().contiguous(), gdst, group=group)

    def recv(self, src: int, dst: int, t: Tensor):
        group, gsrc, _ = self._links[(src, dst)]
        if self.host_staged and t.device.type != "cpu":
            host = torch.empty(t.shape, dtype=t.dtype)
            return _HostStagedWork(dist.irecv(host, gsrc, group=group), host, t)
        return dist.irecv(t, gsrc, group=group)


_DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32]


def dtype_code(dt: torch.dtype) -> int:
    return _DTYPES.index(dt)


def code_dtype(code: int) -> torch.dtype:
    return _DTYPES[code]


def exchange_shape(p2p: P2P, out: Optional[Tensor], device: torch.device) -> Optional[Tuple[List[int], torch.dtype]]:
    """Stage j sends its output's (shape, dtype) to j+1 and receives its input's from j-1."""
    recv = None
    if p2p.rank > 0:
        shape, code = p2p.recv_obj_shape(p2p.rank - 1, device)
        recv = (shape, code_dtype(code))
    if p2p.rank < p2p.world - 1 and out is not None:
        p2p.send_obj_shape(list(out.shape), dtype_code(out.dtype), p2p.rank + 1, device)
    return recv
