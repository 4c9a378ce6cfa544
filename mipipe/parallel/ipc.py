"""Pipeline channels over device-memory IPC links instead of RCCL.

:class:`IpcChannels` is a drop-in for :class:`~mipipe.parallel.p2p.Channels`
(same ``send_act`` / ``recv_act`` / ``send_grad`` / ``recv_grad`` and work
handles with ``wait()``), built on the native :class:`mipipe._C.IpcLink`
(``csrc/runtime/ipc.{h,cpp}``):

* every receiving rank owns a ring of device slots per incoming link behind
  an array of "full" flag words, exported once (``hipIpcGetMemHandle``);
* the sender's copy stream waits for the producer (an event: a barrier
  packet), copies the message into the slot and then a staged sequence word
  into the receiver's full flag -- with the ``sdma`` engines both are
  ``hipMemcpyDeviceToDeviceNoCU`` copies, so the link's copy stream runs on
  the DMA engines and dispatches no kernel at all; the slot being free is a
  host-side check of a counter in the shared block (never a GPU-side wait);
* the receiver's compute stream waits for the flag (``hipStreamWaitValue64``,
  in order with its own work) and reads the slot IN PLACE
  (:meth:`IpcChannels.recv_act_view`: the slot is the receive buffer, one
  copy per message), then releases it by writing the shared release counter
  (host memory registered with its GPU) on that same stream.

Neither host waits for the other inside a step (a slot per message of the
step): completion is stream-ordered end to end, as the reference's ``Wait``
(an event record plus a stream wait, ``/root/reference/README.md:332-369``)
and ``Copy`` (a copy on copy streams, ``/root/reference/README.md:193-213``).
The legacy ``recv_act(t)`` form copies the slot into ``t`` on the consumer
stream and releases it right away.

Slots: the engine sends ``chunks x virtual`` messages per link and step, each
into its own slot (``slots`` >= that), so a slot is a persistent
per-(chunk, micro-batch) receive buffer; the engine releases the slots it
read in place at the end of each step (:meth:`end_step`).

Without a GPU (``device.type == "cpu"``) the links live in shared memory and
copies are ``memcpy`` -- the same protocol with host atomics, for CPU tests.

Construction is collective over the default process group (it gathers each
rank's incoming-message size and shares a job-unique name prefix), and every
phase of it ends in an all-rank agreement: a rank whose ``create`` /
``attach`` raises makes EVERY rank raise :class:`LinkSetupError` at the same
point (no rank is left in a barrier), which :func:`verified_ipc` turns into a
common fall-back.  ``MIPIPE_IPC_FAULT=<phase>:<rank>`` (phase ``create``,
``attach`` or ``selftest``) injects a failure on one rank, for the tests.
"""
from __future__ import annotations

import os
import time
import uuid
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

from .. import _native_loader
from ..stream import record_stream

__all__ = ["IpcChannels", "ENGINES", "LinkSetupError", "ranks_share_a_device", "verified_ipc"]

# sdma / blit: the sender's copy on the link's own copy stream (overlaps the
# producer's next kernels; two cross-stream dependencies per message);
# inline / inline-sdma: the copy on the producer's stream (no cross-stream hop:
# the lowest latency, ordered before the producer's later work).  The sdma
# engines copy payload and flag with the DMA engines (no kernel); blit / inline
# use a copy kernel and a stream write-value kernel.
ENGINES = {"sdma": 0, "blit": 1, "inline": 2, "inline-sdma": 3}


class LinkSetupError(RuntimeError):
    """Raised on EVERY rank when any rank failed a phase of the link set-up."""


def _fault(phase: str, rank: int) -> None:
    """``MIPIPE_IPC_FAULT=<phase>:<rank>``: fail ``phase`` on ``rank`` (tests)."""
    want = os.environ.get("MIPIPE_IPC_FAULT", "")
    if want and want == f"{phase}:{rank}":
        raise RuntimeError(f"injected fault ({want})")


def _agree(ok: bool, device: torch.device) -> bool:
    """All-rank AND of ``ok`` over the default group (also a barrier)."""
    on_dev = dist.get_backend() == "nccl" and device.type == "cuda"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def _reasons(reason: Optional[str]) -> str:
    """Every rank's failure, one string (collective)."""
    got: List[Optional[str]] = [None] * dist.get_world_size()
    dist.all_gather_object(got, reason)
    return "; ".join(f"rank {i}: {r}" for i, r in enumerate(got) if r)


class _SendWork:
    def __init__(self, link, seq: int, device: torch.device) -> None:
        self.link, self.seq, self.device = link, seq, device

    def wait(self) -> bool:
        """Orders the current stream after the copy (the RCCL isend contract)."""
        if self.device.type == "cuda" and not self.link.inline_copy:  # inline: already on the producer's stream
            rt = _native_loader.kernels()
            rt.stream_wait(torch.cuda.current_stream(self.device).cuda_stream, self.link.copy_stream,
                           self.device.index)
        return True

    def is_completed(self) -> bool:
        return bool(self.link.done(self.seq))


class _RecvWork:
    """Copying receive: ``wait()`` enqueues (GPU-side wait for the message, copy
    into ``dst``, slot release) on the current stream; the host never blocks
    on a device link."""

    def __init__(self, link, seq: int, dst: Tensor, timeout: float) -> None:
        self.link, self.seq, self.dst, self.timeout = link, seq, dst, timeout
        self._done = False

    def wait(self) -> bool:
        if not self._done:
            dst = self.dst
            stream = torch.cuda.current_stream(dst.device).cuda_stream if dst.is_cuda else 0
            self.link.wait(self.seq, dst, stream, self.timeout)
            self._done = True
            self.dst = None
        return True

    def is_completed(self) -> bool:
        return self._done and bool(self.link.done(self.seq))


class _ViewWork:
    """Zero-copy receive: ``wait()`` makes the current stream wait (on the GPU)
    for the message; the tensor handed out with this work is the slot."""

    def __init__(self, chan: "IpcChannels", link, seq: int, device: torch.device) -> None:
        self.chan, self.link, self.seq, self.device = chan, link, seq, device
        self.waited = False

    def wait(self) -> bool:
        if not self.waited:
            self.link.acquire(self.seq, torch.cuda.current_stream(self.device).cuda_stream)
            self.waited = True
        return True

    def is_completed(self) -> bool:
        # arrival is a GPU-side event the host does not poll: a receive counts as
        # complete once its wait is on the stream AND the sender has enqueued the
        # message (the shared block's send count), so a stalled peer shows up in
        # the watchdog's pending-transfer report
        return self.waited and self.link.message_bytes(self.seq) != -1


class IpcChannels:
    """Activation / gradient channels of one pipeline over IPC links.

    Args:
        ranks: global ranks of the pipeline in stage order.
        wrap: looping placement (links n-1 -> 0 for activations, 0 -> n-1 for
            gradients).
        device: this rank's device (``cpu``: shared-memory host links).
        recv_bytes: the largest activation (bytes) this rank RECEIVES; the
            gradients it receives are sized by its downstream neighbour's.
        slots: messages in flight per link (default: 64).  The engine passes
            ``chunks x virtual`` so every message of a step has its own slot:
            a slot read in place is released only at :meth:`end_step`.
        engine: the sender's copy (:data:`ENGINES`); default ``$MIPIPE_IPC_ENGINE``
            or ``"inline"`` (one-way 15.7 us at 1 MiB against ~150 us through a
            copy stream; the 2-rank shared-GPU step +3.2 %:
            profiles/ipc_stream_ordered.txt).  ``"sdma"`` / ``"inline-sdma"``
            copy payload and completion flag with ``hipMemcpyDeviceToDeviceNoCU``:
            the copy engines only, no kernel on the copy stream (what transport
            ``auto`` uses across GPUs; profiles/ipc_cu_free_r6.txt).
        timeout: seconds a host wait may block before it raises -- a host-mode
            receive, or a send whose slot still holds an unreleased message (the
            engine's watchdog usually fires first).
    """

    host_staged = False
    setup_s = selftest_s = None  # set by verified_ipc

    def __init__(self, ranks: Sequence[int], wrap: bool = False, *, device: torch.device, recv_bytes: int,
                 slots: int = 64, engine: Optional[str] = None, timeout: float = 300.0) -> None:
        engine = engine or os.environ.get("MIPIPE_IPC_ENGINE", "inline")
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
        # zero-copy receives hold their slot until end_step(): only with a slot
        # per message of a step (the caller checks slots against its step)
        self.zero_copy = self.device.type == "cuda"
        self.slots = int(slots)
        dev_index = self.device.index if self.device.type == "cuda" else -1
        if self.device.type == "cuda" and dev_index is None:
            dev_index = torch.cuda.current_device()
            self.device = torch.device("cuda", dev_index)
        # job-unique prefix + every rank's incoming activation size (collective)
        prefix = [uuid.uuid4().hex[:12] if me == 0 else None]
        dist.broadcast_object_list(prefix, src=0)
        sizes: List[Optional[int]] = [None] * dist.get_world_size()
        dist.all_gather_object(sizes, (me, int(recv_bytes)))
        by_rank = dict(s for s in sizes)
        self._act_in = self._act_out = self._grad_in = self._grad_out = None
        self._links: list = []
        self._copy_streams: Dict[int, torch.cuda.ExternalStream] = {}
        self._held: List[Tuple[object, int, int]] = []  # (link, seq, bytes) read in place, released at end_step
        members = sorted(set(self.ranks))
        if self.rank < 0 or n < 2:
            # every process takes part in the same agreements (one per phase below)
            for _ in range(1 + len(members) if n >= 2 else 1):
                self._phase("set-up (not a member)", None, me)
            return
        r = self.rank
        has_prev = r > 0 or wrap
        has_next = r < n - 1 or wrap
        prev_g, next_g = self.ranks[(r - 1) % n], self.ranks[(r + 1) % n]

        def name(kind: str, src: int, dst: int) -> str:
            return f"/mipipe-{prefix[0]}-{kind}-{src}-{dst}"

        def create() -> None:
            # receivers first (they create the shm blocks and slot rings) ...
            _fault("create", me)
            if has_prev:
                self._act_in = k.IpcLink.create(name("act", prev_g, me), dev_index, slots, max(by_rank[me], 256))
            if has_next:
                self._grad_in = k.IpcLink.create(name("grad", next_g, me), dev_index, slots,
                                                 max(by_rank[next_g], 256))

        self._phase("create", create, me)
        # ... then senders attach to the neighbours' blocks (importing their rings) -- ONE PROCESS AT A TIME: with
        # every rank importing a neighbour's handle at once (a ring of imports) hipIpcOpenMemHandle deadlocked in the
        # runtime (4 and 8 ranks on one MI355X: every rank blocked inside it; tools/ipc_attach_probe.py,
        # tools/gpu_runs/r5_g25.sh).
        eng = ENGINES[engine]

        def attach() -> None:
            _fault("attach", me)
            if has_next:
                self._act_out = k.IpcLink.attach(name("act", me, next_g), dev_index, eng, self.timeout)
            if has_prev:
                self._grad_out = k.IpcLink.attach(name("grad", me, prev_g), dev_index, eng, self.timeout)

        for turn in members:
            self._phase(f"attach (rank {turn}'s turn)", attach if turn == me else None, me)
        self._links = [x for x in (self._act_in, self._grad_in, self._act_out, self._grad_out) if x is not None]
        for link in self._links:
            if not link.is_sender:
                link.unlink()  # everyone is attached: no name left behind in /dev/shm

    def _phase(self, what: str, fn, me: int) -> None:
        """Runs one set-up phase on this rank, then agrees with every rank: if any
        rank's phase raised, every rank drops its half-built links and raises
        :class:`LinkSetupError` naming the failures -- together, within one
        collective, instead of leaving the others in a barrier until a watchdog
        kills the job."""
        err = None
        if fn is not None:
            try:
                fn()
            except Exception as exc:  # noqa: BLE001 -- reported to every rank
                err = f"{what}: {type(exc).__name__}: {exc}"
        if _agree(err is None, self.device):
            return
        why = _reasons(err)
        for link in (self._act_in, self._grad_in, self._act_out, self._grad_out):
            if link is not None:
                link.abort()
        self._act_in = self._act_out = self._grad_in = self._grad_out = None
        self._links = []
        raise LinkSetupError(f"IPC link set-up failed ({why})")

    # ------------------------------------------------------------------ self-test
    def self_test(self, rounds: int = 2, timeout: float = 30.0) -> Optional[str]:
        """Exercises every link of this rank exactly as the engine will: whole-slot
        messages through the sender's engine into the peer's ring, the GPU-side
        flag wait, a kernel reading the slot in place, the release -- and checks
        every word (a pattern unique to link, direction and message) -- then
        once more after the ring has wrapped onto the first slot read, so a
        receiver reading stale cached lines of a reused slot is caught too.

        Returns ``None`` on success or the reason it failed.  Bounded: the GPU
        work runs on a side stream polled for ``timeout`` seconds; on a timeout
        the links are aborted (this rank's flags saturated), so nothing stays
        blocked.  Every rank of the pipeline must call it (each receives what
        its neighbours send).  A cross-GPU link that never ran on hardware gets
        checked before it carries a step (the cross-GPU path had
        only ever been exercised with the ranks sharing one GPU).
        """
        if self.rank < 0 or self.world < 2:
            return None
        _fault("selftest", self.ranks[self.rank])
        dev = self.device
        if dev.type != "cuda":
            return None
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # made on the stream every `ok &=` runs on
            ok = torch.ones((), dtype=torch.int32, device=dev)

        def pattern(n: int, kind: str, src: int, dst: int, seq: int, device) -> Tensor:
            # the same on both sides of a link (no per-process hash seeds)
            base = (((1 if kind == "act" else 2) * 131 + src) * 131 + dst) * 65536 + seq * 7919
            return (torch.arange(n, dtype=torch.int64, device=device) * 3 + base).remainder(2**31).to(torch.int32)

        me = self.ranks[self.rank]
        n = self.world
        r = self.rank
        prev_g, next_g = self.ranks[(r - 1) % n], self.ranks[(r + 1) % n]
        t0 = time.perf_counter()

        def left() -> float:
            # a send whose slot is still held blocks the host (the release counter is polled): within the
            # self-test's budget, so a peer that never releases -- it failed before its own self-test -- ends
            # this one in time too (the exception becomes the reason in verified_ipc)
            return max(0.1, timeout - (time.perf_counter() - t0))

        with torch.cuda.stream(side):
            for rd in range(rounds):
                for kind, link, dst in (("act", self._act_out, next_g), ("grad", self._grad_out, prev_g)):
                    if link is None:
                        continue
                    peer_slot = int(link.slot_bytes) // 4
                    msg = pattern(peer_slot, kind, me, dst, rd, dev)
                    self._send(link, msg, left())
                for kind, link, src in (("act", self._act_in, prev_g), ("grad", self._grad_in, next_g)):
                    if link is None:
                        continue
                    words = int(link.slot_bytes) // 4
                    t, work = self._recv_view(link, (words,), torch.int32)
                    work.wait()
                    ok &= (t == pattern(words, kind, src, me, rd, dev)).all().to(torch.int32)
            self.end_step()
            # Slot reuse: tiny filler messages walk every ring round to the slot the first round used and read
            # (its lines are in this GPU's caches now), then one more checked whole-slot message lands there --
            # a receiver that kept reading stale cached lines of its slot would fail here, not in a step.
            outs = [(kind, link, dst) for kind, link, dst in (("act", self._act_out, next_g),
                                                              ("grad", self._grad_out, prev_g)) if link is not None]
            ins = [(kind, link, src) for kind, link, src in (("act", self._act_in, prev_g),
                                                            ("grad", self._grad_in, next_g)) if link is not None]
            filler = torch.zeros(64, dtype=torch.int32, device=dev)
            for i in range(max([(-rounds) % int(link.nslots) for _, link, _ in outs + ins] or [0])):
                for _, link, _ in outs:
                    if i < (-rounds) % int(link.nslots):
                        self._send(link, filler, left())
                for _, link, _ in ins:
                    if i < (-rounds) % int(link.nslots):
                        _, work = self._recv_view(link, (64,), torch.int32)
                        work.wait()
                self.end_step()
            for kind, link, dst in outs:
                self._send(link, pattern(int(link.slot_bytes) // 4, kind, me, dst, rounds, dev), left())
            for kind, link, src in ins:
                words = int(link.slot_bytes) // 4
                t, work = self._recv_view(link, (words,), torch.int32)
                work.wait()
                ok &= (t == pattern(words, kind, src, me, rounds, dev)).all().to(torch.int32)
            self.end_step()
            ev = torch.cuda.Event()
            ev.record(side)
        while not ev.query():
            if time.perf_counter() - t0 > timeout:
                self.abort()
                return f"self-test timed out after {timeout:.0f} s ({'; '.join(self.describe())})"
            time.sleep(0.001)
        if int(ok.item()) != 1:
            return "self-test read wrong data through a link (" + "; ".join(self.describe()) + ")"
        torch.cuda.current_stream(dev).wait_stream(side)
        return None

    # ------------------------------------------------------------------ API
    def warmup(self, device: torch.device) -> None:
        """Nothing to do: the links are connected at construction."""

    warmup_s = 0.0

    def describe(self) -> List[str]:
        return [link.describe() for link in self._links]

    def comm_info(self) -> List[dict]:
        """This rank's links, for the bench JSON (the RCCL channels report theirs)."""
        out = []
        for kind, link, peer_is_src in (("act in", self._act_in, True), ("grad in", self._grad_in, True),
                                        ("act out", self._act_out, False), ("grad out", self._grad_out, False)):
            if link is not None:
                out.append({"dir": kind, "backend": "ipc", "group_world": 2, "group_rank": int(not peer_is_src),
                            "warmed": True, "slots": int(link.nslots), "slot_bytes": int(link.slot_bytes)})
        return out

    def abort(self) -> None:
        """A failed step: unblocks every host-mode wait on this rank's links with
        an error, and lets every pending GPU-side wait on a flag this rank owns
        pass (``IpcLink.abort``), so the streams drain instead of hanging."""
        for link in self._links:
            link.abort()

    def _copy_stream(self, link):
        s = self._copy_streams.get(id(link))
        if s is None:
            s = torch.cuda.ExternalStream(link.copy_stream, device=self.device)
            self._copy_streams[id(link)] = s
        return s

    def _send(self, link, t: Tensor, timeout: Optional[float] = None):
        if link is None:
            raise RuntimeError(f"rank {self.rank}: no link in that direction")
        src = t.detach()
        if not src.is_contiguous():
            src = src.contiguous()
        if src.is_cuda:
            # the copy runs on the link's stream after the current one: keep the
            # source block alive until then
            if not link.inline_copy:
                record_stream(src, self._copy_stream(link))
            seq = link.send(src, torch.cuda.current_stream(src.device).cuda_stream,
                            self.timeout if timeout is None else timeout)
        else:
            seq = link.send(src, 0, self.timeout if timeout is None else timeout)
        return _SendWork(link, seq, src.device)

    def _recv(self, link, t: Tensor):
        if link is None:
            raise RuntimeError(f"rank {self.rank}: no link in that direction")
        if not t.is_contiguous():
            raise ValueError("receive buffers must be contiguous")
        return _RecvWork(link, link.post(), t, self.timeout)

    def _recv_view(self, link, shape, dtype) -> Tuple[Tensor, object]:
        """Zero-copy receive: (the slot as a tensor, its work).  Read the tensor
        only after ``work.wait()`` (on the stream that waited) and not after
        :meth:`end_step`."""
        if link is None:
            raise RuntimeError(f"rank {self.rank}: no link in that direction")
        if not self.zero_copy:
            t = torch.empty(shape, dtype=dtype, device=self.device)
            return t, self._recv(link, t)
        seq = link.post()
        t = link.slot_tensor(seq, list(shape), dtype, self.device.index)  # the GPU wait comes with work.wait()
        self._held.append((link, seq, t.numel() * t.element_size()))
        return t, _ViewWork(self, link, seq, self.device)

    def send_act(self, t: Tensor):
        return self._send(self._act_out, t)

    def recv_act(self, t: Tensor):
        return self._recv(self._act_in, t)

    def recv_act_view(self, shape, dtype):
        return self._recv_view(self._act_in, shape, dtype)

    def send_grad(self, t: Tensor):
        return self._send(self._grad_out, t)

    def recv_grad(self, t: Tensor):
        return self._recv(self._grad_in, t)

    def recv_grad_view(self, shape, dtype):
        return self._recv_view(self._grad_in, shape, dtype)

    def end_step(self) -> None:
        """Releases every slot read in place this step, after the work queued on
        the current stream (the step's last reader of them): one release-counter
        write per link."""
        if not self._held:
            return
        stream = torch.cuda.current_stream(self.device).cuda_stream
        bad = []
        by_link: Dict[int, Tuple[object, List[int]]] = {}
        for link, seq, nbytes in self._held:
            by_link.setdefault(id(link), (link, []))[1].append(seq)
            # the device-side wait cannot compare sizes: check the sender's byte
            # count here, once it has enqueued the message (-1: not yet, -2: gone)
            sent = link.message_bytes(seq)
            if sent >= 0 and sent != nbytes:
                bad.append(f"message {seq} on {link.describe()}: sender wrote {sent} B, the receive read {nbytes} B")
        for link, seqs in by_link.values():
            link.release_many(seqs, stream)
        self._held = []
        if bad:
            raise RuntimeError("mipipe ipc: message size mismatch (the ranks disagree on a boundary shape): "
                               + "; ".join(bad))

    def close(self) -> None:
        """Tears the links down: every sender unmaps its peer's ring, then (after
        a barrier, when a process group is up) every receiver frees its own.
        Collective when ``dist`` is initialised."""
        if self.device.type == "cuda":
            self.end_step()
            # bounded: a link whose peer died would otherwise block the
            # synchronize forever (abort() saturates this side's flags first)
            stuck = [link.describe() for link in self._links if not link.drain(60.0)]
            if stuck:
                raise RuntimeError("mipipe ipc: links did not drain in 60 s: " + "; ".join(stuck))
            torch.cuda.synchronize(self.device)
        # the links' copy streams come from the runtime's process-lifetime pool (tensors recorded on them may
        # outlive the links); only the wrappers go
        self._copy_streams = {}
        self._act_out = self._grad_out = None
        self._links = [x for x in self._links if not x.is_sender]
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
        self._links = []
        self._act_in = self._grad_in = None



def ranks_share_a_device(device: torch.device) -> bool:
    """True if two ranks of the default process group run on one GPU (the
    one-GPU rehearsals).  Collective."""
    me = str(torch.cuda.get_device_properties(device).uuid) if device.type == "cuda" else f"cpu-{os.getpid()}"
    ids: List[Optional[str]] = [None] * dist.get_world_size()
    dist.all_gather_object(ids, me)
    return len(set(ids)) < len(ids)


def verified_ipc(make_ipc, make_fallback, device: torch.device):
    """Builds IPC channels (``make_ipc()``), runs :meth:`IpcChannels.self_test`
    on every rank and agrees over the default process group: all ranks keep
    the IPC channels, or all switch to ``make_fallback()`` (RCCL).  A set-up
    phase that raises on any rank (:class:`LinkSetupError`, raised on every
    rank together) and a self-test that raises count as failures too, so
    every rank always reaches the same agreement.  Returns ``(channels,
    reason)`` -- ``reason`` is ``None`` when IPC passed, else what failed on
    which rank (for the bench JSON).  Collective."""
    t0 = time.perf_counter()
    try:
        chan = make_ipc()
    except LinkSetupError as exc:
        return make_fallback(), str(exc)
    t1 = time.perf_counter()
    try:
        reason = chan.self_test()
    except Exception as exc:  # noqa: BLE001 -- every rank must still reach the agreement
        reason = f"self-test raised {type(exc).__name__}: {exc}"
    if _agree(reason is None, device):
        chan.setup_s, chan.selftest_s = t1 - t0, time.perf_counter() - t1  # for the bench's start-up breakdown
        return chan, None
    why = _reasons(reason)
    chan.abort()  # not closed: a link that failed may never drain; process teardown unmaps it
    return make_fallback(), why
