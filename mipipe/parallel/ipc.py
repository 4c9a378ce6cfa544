"""Pipeline channels over device-memory IPC links instead of RCCL.

:class:`IpcChannels` is a drop-in for :class:`~mipipe.parallel.p2p.Channels`
(same ``send_act`` / ``recv_act`` / ``send_grad`` / ``recv_grad`` and work
handles with ``wait()``), built on the native :class:`mipipe._C.IpcLink`
(``csrc/runtime/ipc.{h,cpp}``):

* every receiving rank owns a ring of device slots per incoming link,
  exported once (``hipIpcGetMemHandle``); the sending rank maps them and
  copies each message into the next slot on a dedicated copy stream with the
  DMA engines (``hipMemcpyAsync``) or a blit kernel -- no RCCL kernel
  occupies CUs next to the GEMMs, and several ranks may share ONE GPU (RCCL
  refuses that: ``profiles/nccl_probe_one_gpu.txt``);
* completion crosses the process boundary through a proxy thread that
  publishes the slot once the sender's copy has completed (default), or
  through interprocess events (``ipc_events=True``: the receiver's compute
  stream waits for the sender's copy on the GPU -- limited on ROCm 7.2 to
  about 32 records per event, see ``_ipc_events_default``);
* the receiver's ``wait()`` copies the slot into the engine's tensor on the
  current stream and releases the slot.

The reference moves activations with peer copies on copy streams
(``/root/reference/README.md:196-212``); this is the same transport for one
process per GPU.  Without a GPU (``device.type == "cpu"``) the links live in
shared memory and copies are ``memcpy`` -- the same protocol, for CPU tests.

Construction is collective over the default process group (it gathers each
rank's incoming-message size and shares a job-unique name prefix).
"""
from __future__ import annotations

import os
import uuid
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist
from torch import Tensor

from .. import _native_loader
from ..stream import record_stream

__all__ = ["IpcChannels", "ENGINES"]

ENGINES = {"sdma": 0, "blit": 1}


def _ipc_events_default() -> bool:
    # Off by default: ROCm 7.2's interprocess events stop working after about
    # 32 records of one event (a record then blocks, a wait fails with
    # "invalid argument"; tools/ipc_bw.py --events reproduces it), and a
    # training run re-records every slot's event once per step.  The proxy
    # thread completes a message once its copy is done, at the price of a
    # host-side wait in the receiver.
    return os.environ.get("MIPIPE_IPC_EVENTS", "0") == "1"


class _SendWork:
    def __init__(self, link, seq: int, device: torch.device) -> None:
        self.link, self.seq, self.device = link, seq, device

    def wait(self) -> bool:
        """Orders the current stream after the copy (the RCCL isend contract)."""
        if self.device.type == "cuda":
            rt = _native_loader.kernels()
            rt.stream_wait(torch.cuda.current_stream(self.device).cuda_stream, self.link.copy_stream,
                           self.device.index)
        return True

    def is_completed(self) -> bool:
        return bool(self.link.done(self.seq))


class _RecvWork:
    def __init__(self, link, seq: int, dst: Tensor, timeout: float) -> None:
        self.link, self.seq, self.dst, self.timeout = link, seq, dst, timeout
        self._done = False

    def wait(self) -> bool:
        """Blocks the host until the sender has issued the message, then copies
        it into the destination on the current stream (stream-ordered after the
        sender's copy)."""
        if not self._done:
            dst = self.dst
            stream = torch.cuda.current_stream(dst.device).cuda_stream if dst.is_cuda else 0
            self.link.wait(self.seq, dst, stream, self.timeout)
            self._done = True
            self.dst = None
        return True

    def is_completed(self) -> bool:
        return self._done or bool(self.link.done(self.seq))


class IpcChannels:
    """Activation / gradient channels of one pipeline over IPC links.

    Args:
        ranks: global ranks of the pipeline in stage order.
        wrap: looping placement (links n-1 -> 0 for activations, 0 -> n-1 for
            gradients).
        device: this rank's device (``cpu``: shared-memory host links).
        recv_bytes: the largest activation (bytes) this rank RECEIVES; the
            gradients it receives are sized by its downstream neighbour's.
        slots: messages in flight per link (default: 64); a sender blocks
            its host only when all are unreleased.  ``chunks x virtual`` (what
            the engine passes) never blocks within a step; fewer is safe for
            a plain GPipe chain but can deadlock a looping placement.
        engine: ``"sdma"`` (DMA engines) or ``"blit"`` (copy kernel) for the
            sender's copy.
        ipc_events: complete through interprocess events (``MIPIPE_IPC_EVENTS=1``)
            instead of the proxy thread (default).
        timeout: seconds a host wait may block before it raises (the engine's
            watchdog usually fires first).
    """

    host_staged = False

    def __init__(self, ranks: Sequence[int], wrap: bool = False, *, device: torch.device, recv_bytes: int,
                 slots: int = 64, engine: str = "sdma", ipc_events: Optional[bool] = None,
                 timeout: float = 300.0) -> None:
        if engine not in ENGINES:
            raise ValueError(f"engine must be one of {sorted(ENGINES)}, got {engine!r}")
        k = _native_loader.kernels()
        self.ranks = list(ranks)
        n = len(self.ranks)
        me = dist.get_rank()
        self.rank = self.ranks.index(me) if me in self.ranks else -1
        self.world = n
        self.device = torch.device(device)
        self.timeout = float(timeout)
        dev_index = self.device.index if self.device.type == "cuda" else -1
        if self.device.type == "cuda" and dev_index is None:
            dev_index = torch.cuda.current_device()
        use_events = _ipc_events_default() if ipc_events is None else bool(ipc_events)
        # job-unique prefix + every rank's incoming activation size (collective)
        prefix = [uuid.uuid4().hex[:12] if me == 0 else None]
        dist.broadcast_object_list(prefix, src=0)
        sizes: List[Optional[int]] = [None] * dist.get_world_size()
        dist.all_gather_object(sizes, (me, int(recv_bytes)))
        by_rank = dict(s for s in sizes)
        self._act_in = self._act_out = self._grad_in = self._grad_out = None
        self._links: list = []
        if self.rank < 0 or n < 2:
            dist.barrier()
            dist.barrier()
            return
        r = self.rank
        has_prev = r > 0 or wrap
        has_next = r < n - 1 or wrap
        prev_g, next_g = self.ranks[(r - 1) % n], self.ranks[(r + 1) % n]

        def name(kind: str, src: int, dst: int) -> str:
            return f"/mipipe-{prefix[0]}-{kind}-{src}-{dst}"

        # receivers first (they create the shm blocks and slot rings) ...
        if has_prev:
            self._act_in = k.IpcLink.create(name("act", prev_g, me), dev_index, slots,
                                            max(by_rank[me], 256), use_events)
        if has_next:
            self._grad_in = k.IpcLink.create(name("grad", next_g, me), dev_index, slots,
                                             max(by_rank[next_g], 256), use_events)
        dist.barrier()
        # ... then senders attach to the neighbours' blocks
        eng = ENGINES[engine]
        if has_next:
            self._act_out = k.IpcLink.attach(name("act", me, next_g), dev_index, eng, self.timeout)
        if has_prev:
            self._grad_out = k.IpcLink.attach(name("grad", me, prev_g), dev_index, eng, self.timeout)
        dist.barrier()
        self._links = [x for x in (self._act_in, self._grad_in, self._act_out, self._grad_out) if x is not None]
        for link in self._links:
            if not link.is_sender:
                link.unlink()  # everyone is attached: no name left behind in /dev/shm
        self._copy_streams: Dict[int, torch.cuda.Stream] = {}

    # ------------------------------------------------------------------ API
    def warmup(self, device: torch.device) -> None:
        """Nothing to do: the links are connected at construction."""

    def describe(self) -> List[str]:
        return [link.describe() for link in self._links]

    def abort(self) -> None:
        """Unblocks every peer waiting on this rank's links with an error."""
        for link in self._links:
            link.abort()

    def _copy_stream(self, link):
        s = self._copy_streams.get(id(link))
        if s is None:
            s = torch.cuda.ExternalStream(link.copy_stream, device=self.device)
            self._copy_streams[id(link)] = s
        return s

    def _send(self, link, t: Tensor):
        if link is None:
            raise RuntimeError(f"rank {self.rank}: no link in that direction")
        src = t.detach()
        if not src.is_contiguous():
            src = src.contiguous()
        if src.is_cuda:
            # the copy runs on the link's stream after the current one: keep the
            # source block alive until then
            record_stream(src, self._copy_stream(link))
            seq = link.send(src, torch.cuda.current_stream(src.device).cuda_stream, self.timeout)
        else:
            seq = link.send(src, 0, self.timeout)
        return _SendWork(link, seq, src.device)

    def _recv(self, link, t: Tensor):
        if link is None:
            raise RuntimeError(f"rank {self.rank}: no link in that direction")
        if not t.is_contiguous():
            raise ValueError("receive buffers must be contiguous")
        return _RecvWork(link, link.post(), t, self.timeout)

    def send_act(self, t: Tensor):
        return self._send(self._act_out, t)

    def recv_act(self, t: Tensor):
        return self._recv(self._act_in, t)

    def send_grad(self, t: Tensor):
        return self._send(self._grad_out, t)

    def recv_grad(self, t: Tensor):
        return self._recv(self._grad_in, t)

    def close(self) -> None:
        """Tears the links down: every sender unmaps its peer's ring, then (after
        a barrier, when a process group is up) every receiver frees its own.
        Collective when ``dist`` is initialised."""
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self._act_out = self._grad_out = None
        self._links = [x for x in self._links if not x.is_sender]
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
        self._links = []
        self._act_in = self._grad_in = None
