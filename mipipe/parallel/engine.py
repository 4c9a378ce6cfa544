"""Multi-process synchronous pipeline (GPipe) -- one rank per MI355X.

This is the scale-out form of :class:`mipipe.Pipe` (SURVEY §5.8, §7.2 step
5): instead of one process driving every GPU from worker threads with peer
copies, each GPU is one process (``torchrun --nproc-per-node N``) that owns
slices of the model, and activations / gradients move between neighbouring
ranks over xGMI -- by default through self-tested device-memory IPC links
(DMA copies into the receiver's slot ring, :mod:`mipipe.parallel.ipc`), with
RCCL send/recv (:class:`~mipipe.parallel.p2p.Channels`) as the fall-back every
rank switches to together.  It keeps the reference's semantics:

* micro-batching of the mini-batch on dim 0 into ``chunks`` micro-batches;
* synchronous fill-drain: every forward of the step, then every backward in
  reverse micro-batch order -- the order the reference's fork/join phonies
  force (``/root/reference/pipeline.py:128-132``) -- and one optimizer step on
  the summed gradients (identical to the unpartitioned model);
* ``checkpoint`` in {``always``, ``except_last``, ``never``}: checkpointed
  micro-batches run forward under ``no_grad`` keeping only the stage input and
  the RNG state, and are recomputed (bit-identical dropout) right before their
  backward (``/root/reference/pipe.py:255-260,354``);
* eval mode never checkpoints (``pipeline.py:153-155``);
* ``@skippable`` cross-stage skips (``pipeline.py:136-138``): a stashed tensor
  goes straight from the stashing rank to the popping rank on its own
  communicator, and its gradient comes back the same way
  (:mod:`mipipe.parallel.skips`).

Looping placement (``virtual`` > 1 model chunks per rank): rank ``r`` of ``n``
owns virtual stages ``r, r+n, r+2n, ...``; a micro-batch flows
0 -> 1 -> ... -> n-1 -> 0 -> ... and each rank runs its chunks breadth-first
(all micro-batches of chunk 0, then chunk 1, ...; backward in reverse).  The
step is still a synchronous GPipe step -- same gradients -- but the fill and
drain shrink from (n-1) stage-times to (n-1) CHUNK-times:
bubble = (n-1) / (v*m + n-1) instead of (n-1) / (m + n-1).  MI355X keeps every
chunk's activations resident (288 GB of HBM), so the extra in-flight
activations cost nothing, and the extra boundary messages ride idle xGMI links.

Optionally ``schedule="1f1b"`` (PipeDream-flush, ``virtual == 1``): same
bubble, activation memory bounded by the number of stages instead of chunks.

Transport (:func:`make_transport`): ``auto`` (default) = the IPC links, whose
zero-copy receives are posted for the whole phase (a posted receive costs
nothing: the consumer's stream waits only when it reaches the micro-batch);
``rccl`` = :class:`~mipipe.parallel.p2p.Channels`, one communicator per link
direction, each receive posted just before the action that consumes it (a
posted RCCL receive is a kernel resident on CUs until its data lands, so it
is kept out of the way of the GEMMs until needed).  Per-stage busy time is
measured with HIP events (bubble %).
"""
from __future__ import annotations

import os
import warnings
import time
from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist
from torch import Tensor, nn

from .. import ops
from ..ops.attention import clear_keep_words as _clear_keep_words
from ..checkpoint import enable_checkpointing, enable_recomputing
from ..pipeline import checkpoint_stop_for
from ..skip.tracker import use_skip_tracker
from ..worker import label_range
from .p2p import Channels, DirectLinks
from .skips import EngineSkipTracker, SkipRoute, gather_routes
from .watchdog import Watchdog

__all__ = ["PipelineEngine", "StepStats", "schedule_actions"]


@dataclass
class StepStats:
    losses: List[Tensor] = field(default_factory=list)  # per-micro-batch losses (device scalars)
    busy_ms: float = 0.0          # GPU time of this rank's compute (events)
    step_ms: float = 0.0          # wall time of the step on this rank
    forward_ms: List[float] = field(default_factory=list)
    backward_ms: List[float] = field(default_factory=list)
    _loss: Optional[Tensor] = field(default=None, repr=False)

    @property
    def loss(self) -> Optional[Tensor]:
        """Mean loss over the micro-batches (None off the last stage).  Reduced on
        first access, so a step whose loss nobody reads launches no reduction."""
        if self._loss is None and self.losses:
            self._loss = torch.stack(self.losses).float().mean()
        return self._loss


def schedule_actions(kind: str, m: int, n: int, j: int, virtual: int = 1) -> List[Tuple[str, int, int]]:
    """Ordered (F|B, chunk, micro-batch) actions of rank ``j`` of ``n``.

    ``gpipe``: breadth-first over the rank's ``virtual`` chunks (forward chunk
    0..v-1, each over micro-batches 0..m-1; backward in exact reverse).  With
    ``virtual == 1`` the chunk index is always 0 and callers may ignore it.
    """
    if kind == "gpipe":
        fw = [("F", c, i) for c in range(virtual) for i in range(m)]
        bw = [("B", c, i) for c in reversed(range(virtual)) for i in reversed(range(m))]
        return fw + bw
    if kind == "1f1b":
        if virtual != 1:
            raise ValueError("1f1b supports one chunk per rank")
        warm = min(n - j - 1, m)
        acts: List[Tuple[str, int, int]] = [("F", 0, i) for i in range(warm)]
        f, b = warm, 0
        while f < m:
            acts.append(("F", 0, f))
            f += 1
            acts.append(("B", 0, b))
            b += 1
        while b < m:
            acts.append(("B", 0, b))
            b += 1
        return acts
    raise ValueError(f"unknown schedule {kind!r}")


@contextmanager
def _null():
    yield


class _RNGState:
    __slots__ = ("cpu", "dev")

    def __init__(self, device: torch.device) -> None:
        self.cpu = torch.get_rng_state()
        self.dev = torch.cuda.get_rng_state(device) if device.type == "cuda" else None


class PipelineEngine:
    """Runs one training (or eval) step of this rank's pipeline stage(s).

    Args:
        module: this rank's stage, or a list of its ``virtual`` chunks in
            virtual-stage order (chunk ``c`` is virtual stage ``c*n + rank``).
        chunks: micro-batches per mini-batch.
        checkpoint: ``always`` / ``except_last`` / ``never``.
        act_shape: shape of the activation each chunk RECEIVES per micro-batch
            (one shape, or one per chunk); gradient buffers take the shape of
            the chunk's outputs.
        act_dtype: its dtype.
        loss_fn: ``loss_fn(output, target) -> scalar`` on the last virtual stage.
        group: process group of the pipeline (default: WORLD), or a ready
            :class:`Channels` (then cross-stage skips need ``skip_routes``).
        schedule: ``gpipe`` (reference order; looping when virtual > 1) or ``1f1b``.
        defer_wgrad: run the backward's weight-gradient GEMMs after this rank's
            last backward (:func:`mipipe.ops.deferred_wgrad`): input gradients
            reach the upstream rank sooner, which shortens the pipeline drain
            by (n-1) weight-gradient times, and each weight's micro-batches
            become one K-segmented GEMM.  Same gradients.
        skip_shapes: ``{skip name or key: (shape, dtype)}`` of cross-stage skips
            whose tensor is not shaped like the popping stage's input.
        skip_routes: explicit cross-stage routes (default: gathered from every
            rank's ``@skippable`` layers at construction, a collective).
        watchdog: a :class:`~mipipe.parallel.watchdog.Watchdog` (or a timeout
            in seconds to create one).  The engine arms it during :meth:`step`,
            marks every action, and registers every transfer, so a stalled
            step ends the process with a report naming the transfer that never
            completed.  Callers can arm it around their own waits too.
        sync_debug: synchronise the device after every action (default: the
            ``MIPIPE_SYNC_DEBUG=1`` environment switch) -- the serialised run
            :func:`mipipe.debug.check_engine` compares a scheduled step with.
        grad_divisor: the backward is seeded with ``loss / (chunks * grad_divisor)``;
            data-parallel replicas pass their count, so the gradient all-reduce
            SUM is the mean (:mod:`mipipe.parallel.data_parallel`).
        transport: how activations and gradients move between ranks when the
            engine builds its own channels (:func:`make_transport`):
            ``"auto"`` (default: self-tested IPC links, every rank falling
            back to RCCL together on any failure), ``"rccl"`` (send/recv of
            the process group) or ``"ipc"`` (device-memory IPC links,
            :class:`~mipipe.parallel.ipc.IpcChannels`, without the self-test;
            works with several ranks on one GPU).  ``transport_options`` go to
            the IpcChannels.
    """

    def __init__(
        self,
        module: Union[nn.Module, Sequence[nn.Module]],
        *,
        chunks: int,
        checkpoint: str = "never",
        act_shape: Union[Sequence[int], Sequence[Sequence[int]]],
        act_dtype: torch.dtype,
        loss_fn: Optional[Callable[[Tensor, Tensor], Tensor]] = None,
        group: Union[None, dist.ProcessGroup, Channels] = None,
        device: Optional[torch.device] = None,
        schedule: str = "gpipe",
        measure: bool = False,
        defer_wgrad: bool = True,
        skip_shapes: Optional[Dict[str, Tuple[Sequence[int], torch.dtype]]] = None,
        skip_routes: Optional[Dict[str, SkipRoute]] = None,
        watchdog: Union[None, float, Watchdog] = None,
        sync_debug: Optional[bool] = None,
        grad_divisor: float = 1.0,
        transport: str = "auto",
        transport_options: Optional[dict] = None,
    ) -> None:
        if checkpoint not in ("always", "except_last", "never"):
            raise ValueError("checkpoint is not one of 'always', 'except_last', or 'never'")
        mods = list(module) if isinstance(module, (list, tuple, nn.ModuleList)) else [module]
        self.modules: List[nn.Module] = mods
        self.virtual = len(mods)
        self.module = mods[0] if self.virtual == 1 else nn.ModuleList(mods)
        self.chunks = int(chunks)
        self.checkpoint = checkpoint
        shapes = list(act_shape)
        if shapes and isinstance(shapes[0], (list, tuple, torch.Size)):
            self.act_shapes = [tuple(s) for s in shapes]
        else:
            self.act_shapes = [tuple(shapes)] * self.virtual
        if len(self.act_shapes) != self.virtual:
            raise ValueError("act_shape needs one shape per chunk")
        self.act_shape = self.act_shapes[0]
        self.act_dtype = act_dtype
        self.loss_fn = loss_fn
        self.schedule = schedule
        self.measure = measure
        self.defer_wgrad = defer_wgrad
        self.grad_divisor = float(grad_divisor)
        self._seeds: Dict[tuple, Tensor] = {}
        if schedule == "1f1b" and self.virtual > 1:
            raise ValueError("1f1b supports one chunk per rank")
        if isinstance(watchdog, (int, float)):
            watchdog = Watchdog(float(watchdog))
        self.watchdog: Optional[Watchdog] = watchdog
        # serialised mode: the device is synchronised after every
        # action, so nothing overlaps; mipipe.debug.check_engine compares a
        # step run this way with a scheduled one
        self.sync_debug = (os.environ.get("MIPIPE_SYNC_DEBUG") == "1") if sync_debug is None else bool(sync_debug)
        self._action = "construction"
        self.transport: Optional[str] = None  # what the stage boundaries run on (None: one rank)
        self.transport_note: Optional[str] = None
        if isinstance(group, Channels) or hasattr(group, "send_act"):  # ready channels (RCCL or IPC)
            self.chan: Optional[Channels] = group
            # channels made by make_transport() carry what they are; others are named by type
            self.transport = getattr(group, "transport_name", None) or (
                "ipc" if type(group).__name__ == "IpcChannels" else "rccl")
            self.transport_note = getattr(group, "transport_note", None)
            if group.world > 1:
                with (watchdog.watch("RCCL channel warm-up") if watchdog is not None else _null()):
                    group.warmup(device or next(mods[0].parameters()).device)
        elif dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
            ranks = dist.get_process_group_ranks(group) if group is not None else list(range(dist.get_world_size()))
            dev = device or next(mods[0].parameters()).device
            self.chan, self.transport, self.transport_note = make_transport(
                ranks, device=dev, chunks=self.chunks, virtual=self.virtual, recv_bytes=self.recv_bytes(),
                transport=transport, transport_options=transport_options, watchdog=watchdog)
        else:
            self.chan = None
        if self.chan is not None:
            self.rank, self.world = self.chan.rank, self.chan.world
        else:
            self.rank, self.world = 0, 1
            if self.virtual > 1:
                raise ValueError("several chunks per rank need a multi-rank pipeline")
        self.device = device or next(mods[0].parameters()).device
        n, v = self.world, self.virtual
        self.vstage = [c * n + self.rank for c in range(v)]
        self.nvirtual = n * v
        # kept for callers: rank-level first/last of the whole pipeline
        self.is_first = self.rank == 0
        self.is_last = self.rank == n - 1
        self._action = "idle"
        if self.watchdog is not None and self.watchdog.describe is None:
            self.watchdog.describe = self.describe
        self._setup_skips(group, skip_shapes, skip_routes)


    def close(self) -> None:
        """Releases the transport (IPC links: senders unmap, then receivers
        free; collective).  RCCL channels need nothing."""
        close = getattr(self.chan, "close", None)
        if close is not None:
            close()

    def recv_bytes(self) -> int:
        """Largest activation (bytes) this rank receives per micro-batch."""
        item = torch.empty((), dtype=self.act_dtype).element_size()
        sizes = [int(torch.Size(s).numel()) * item for s in self.act_shapes]
        return max(sizes) if sizes else 0

    # ------------------------------------------------------------------ watchdog
    def describe(self) -> str:
        """One line of engine state for failure reports."""
        return (f"pipeline rank {self.rank}/{self.world}, virtual stages {self.vstage}, chunks {self.chunks}, "
                f"schedule {self.schedule}, checkpoint {self.checkpoint}, current action {self._action}")

    def _mark(self, label: str) -> None:
        self._action = label
        if self.watchdog is not None:
            self.watchdog.progress(label)

    def _track(self, label: str, work):
        if self.watchdog is not None:
            self.watchdog.pending.add(label, work)
        return work

    # ------------------------------------------------------------------ skips
    def _setup_skips(self, group, skip_shapes, skip_routes) -> None:
        """Cross-stage skip routes, the per-chunk key lists and the direct links."""
        if skip_routes is not None:
            routes = dict(skip_routes)
        elif self.chan is not None and not (isinstance(group, Channels) or hasattr(group, "send_act")):
            routes = gather_routes(self.modules, self.vstage, self.act_shapes, self.act_dtype, group=group,
                                   skip_shapes=skip_shapes)
        else:
            routes = {}  # one rank, one chunk: every skip stays inside the chunk
        self.skip_routes: Dict[str, SkipRoute] = routes
        self._pops = [sorted(k for k, r in routes.items() if r.pop_vstage == vs) for vs in self.vstage]
        self._stashes = [sorted(k for k, r in routes.items() if r.stash_vstage == vs) for vs in self.vstage]
        n = self.world
        pairs = []
        for r in routes.values():
            s, d = r.stash_vstage % n, r.pop_vstage % n
            if s != d:
                pairs.append((s, d))
                if r.has_grad:
                    pairs.append((d, s))
        self._skip_links: Optional[DirectLinks] = None
        if pairs:
            self._skip_links = DirectLinks(self.chan.ranks, pairs)
            with (self.watchdog.watch("skip link warm-up") if self.watchdog is not None else _null()):
                self._skip_links.warmup(self.device)

    def _actions_of(self, rank: int, training: bool) -> List[Tuple[str, int, int]]:
        if training:
            return schedule_actions(self.schedule, self.chunks, self.world, rank, self.virtual)
        return [("F", c, i) for c in range(self.virtual) for i in range(self.chunks)]

    def _post_skip_recvs(self, into: Dict, training: bool, grad: bool) -> None:
        """Posts every skip (``grad``: skip-gradient) receive of the step, per
        source rank in the order that rank sends them: its schedule's F (B)
        actions, keys sorted within an action."""
        n = self.world
        want = "B" if grad else "F"
        for src in range(n):
            if src == self.rank:
                continue
            for kind, c, i in self._actions_of(src, training):
                if kind != want:
                    continue
                vs = c * n + src
                for key in sorted(self.skip_routes):
                    r = self.skip_routes[key]
                    if grad and not (r.pop_vstage == vs and r.stash_vstage % n == self.rank and r.has_grad):
                        continue
                    if not grad and not (r.stash_vstage == vs and r.pop_vstage % n == self.rank):
                        continue
                    buf = torch.empty(r.shape, dtype=r.dtype, device=self.device)
                    what = "skip gradient" if grad else "skip"
                    into[(key, i)] = (buf, self._track(f"recv {what} '{key}' micro-batch {i} from rank {src}",
                                                       self._skip_links.recv(src, self.rank, buf)))

    # ------------------------------------------------------------------ helpers
    def _first(self, c: int) -> bool:
        return self.vstage[c] == 0

    def _last(self, c: int) -> bool:
        return self.vstage[c] == self.nvirtual - 1

    def _new_act(self, c: int, like: Optional[Tensor] = None) -> Tensor:
        if like is not None:
            return torch.empty(like.shape, dtype=like.dtype, device=self.device)
        return torch.empty(self.act_shapes[c], dtype=self.act_dtype, device=self.device)

    @staticmethod
    def _run(mod: nn.Module, x: Tensor, targets, i: int, tracker: Optional[EngineSkipTracker] = None) -> Tensor:
        """Chunk forward; chunks that want the targets (vocabulary-split decoder) get them."""
        if tracker is not None:
            with use_skip_tracker(tracker):
                return PipelineEngine._run(mod, x, targets, i)
        if getattr(mod, "wants_target", False):
            if targets is None:
                raise ValueError("this stage needs the targets (vocabulary-split decoder): pass targets on every rank")
            return mod(x, targets[i])
        return mod(x)

    def _loss(self, mod: nn.Module, y: Tensor, targets, i: int) -> Tensor:
        """Loss of the last virtual stage: computed by the chunk itself (``fused_loss``) or by ``loss_fn``."""
        if getattr(mod, "fused_loss", False):
            return y
        return self.loss_fn(y, targets[i])

    def _loss_seed(self, loss: Tensor) -> Tensor:
        """Backward seed of a micro-batch loss: d(mean over the m micro-batches and
        the ``grad_divisor`` replicas)/d(loss) = 1 / (m * grad_divisor), a device
        constant made once, so the loss path launches no divide and no fill."""
        key = (loss.shape, loss.dtype, loss.device, self.chunks, self.grad_divisor)
        seed = self._seeds.get(key)
        if seed is None:
            seed = torch.full(loss.shape, 1.0 / (self.chunks * self.grad_divisor), dtype=loss.dtype,
                              device=loss.device)
            self._seeds[key] = seed
        return seed

    def _timer(self):
        if not self.measure or self.device.type != "cuda":
            return None
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    # ------------------------------------------------------------------ step
    def step(self, inputs: Optional[Sequence[Tensor]] = None, targets: Optional[Sequence[Tensor]] = None) -> StepStats:
        """Forward + backward of one mini-batch given as per-micro-batch lists.

        Every action is a roctx range (``F vs<s> mb<i>``, ``B ...``,
        ``recompute ...``, ``wait recv act/grad ...``, ``post recvs``, ``wgrad
        flush``, ``wait sends``) inside one ``engine step`` range, so a
        rocprofv3 ``--marker-trace`` timeline attributes every idle gap per
        rank and micro-batch (``tools/engine_timeline.py``).
        """
        with label_range("engine step"):
            return self._step(inputs, targets)

    def _step(self, inputs: Optional[Sequence[Tensor]] = None, targets: Optional[Sequence[Tensor]] = None) -> StepStats:
        """Forward + backward of one mini-batch given as per-micro-batch lists.

        ``inputs`` (rank owning virtual stage 0) and ``targets`` (rank owning
        the last virtual stage, and every rank whose chunks want targets) have
        ``chunks`` entries.  Gradients accumulate
        into the parameters (or their ``main_grad``); the caller runs the
        optimizer.  Returns the mean loss on the last stage.
        """
        m, v, n = self.chunks, self.virtual, self.world
        training = self.modules[0].training and torch.is_grad_enabled()
        stop = checkpoint_stop_for(self.checkpoint, m) if self.modules[0].training else 0
        stats = StepStats()
        t0 = time.perf_counter()
        chan = self.chan
        routes = self.skip_routes
        if self.watchdog is not None:
            self.watchdog.pending.clear()

        recv_x = [[None] * m for _ in range(v)]
        recv_w = [[None] * m for _ in range(v)]
        # zero-copy transports (IPC links) hand out the receive slot itself as the
        # buffer, held until the step ends: only with a slot per message of the step
        zc = getattr(chan, "zero_copy", False) and getattr(chan, "slots", 0) >= m * v

        def post_act_recv(c: int, i: int) -> None:
            if self._first(c) or recv_w[c][i] is not None:
                return
            if zc:
                recv_x[c][i], work = chan.recv_act_view(self.act_shapes[c], self.act_dtype)
            else:
                recv_x[c][i] = self._new_act(c)
                work = chan.recv_act(recv_x[c][i])
            recv_w[c][i] = self._track(f"recv activation: virtual stage {self.vstage[c]} micro-batch {i} "
                                       f"from rank {(self.rank - 1) % n}", work)

        # A zero-copy receive only reserves a slot (the consumer's stream waits
        # when it reaches the micro-batch), so every activation receive of the
        # forward phase is posted up front, in the order the upstream rank sends
        # them (chunk-major, micro-batch minor).  Any other receive (RCCL) is a
        # kernel on CUs, ordered on the GPU after the work the compute stream
        # had when it was posted and resident until its data lands: those are
        # posted one action ahead -- the next action's receive just BEFORE an
        # action is issued, so its kernel starts with that action and its
        # transfer lands under that action's compute (posted after it, the
        # transfer would sit exposed between the two actions; posted per phase,
        # the kernel would stay resident across every wait of the phase).
        # profiles/rccl_fallback_r6.txt prices the choice.  Either way every
        # link's receives are posted in the order its sender sends.
        lazy = chan is not None and not zc
        if chan is not None and zc:
            with label_range("post recvs: activations"):
                for c in range(v):
                    for i in range(m):
                        post_act_recv(c, i)
        # ... and every skip receive (each skip has its own directed link).
        sk_rx: Dict = {}
        sk_grad_rx: Dict = {}
        sk_local: Dict = {}        # (key, i) -> skip handed between chunks of this rank
        sk_local_grad: Dict = {}
        if self._skip_links is not None:
            self._post_skip_recvs(sk_rx, training, grad=False)

        stage_in = [[None] * m for _ in range(v)]
        stage_out = [[None] * m for _ in range(v)]
        out_meta = [[None] * m for _ in range(v)]
        rng = [[None] * m for _ in range(v)]
        grad_w = [[None] * m for _ in range(v)]
        grad_buf = [[None] * m for _ in range(v)]
        skip_in = [[None] * m for _ in range(v)]
        skip_out = [[None] * m for _ in range(v)]
        losses: List[Tensor] = []
        sends = []
        events = []

        def skip_tracker(c: int, i: int) -> Optional[EngineSkipTracker]:
            """Tracker of chunk c / micro-batch i, holding its received skips."""
            if not routes:
                return None
            if skip_in[c][i] is None:
                incoming = {}
                for key in self._pops[c]:
                    r = routes[key]
                    if r.stash_vstage % n == self.rank:
                        t = sk_local.pop((key, i))
                    else:
                        t, work = sk_rx.pop((key, i))
                        work.wait()
                    if training and r.has_grad:
                        t.requires_grad_(True)
                    incoming[key] = t
                skip_in[c][i] = incoming
            return EngineSkipTracker(routes, skip_in[c][i])

        def ship_skips(c: int, i: int, tracker: Optional[EngineSkipTracker]) -> None:
            if tracker is None:
                return
            for key in self._stashes[c]:
                if key not in tracker.outgoing:
                    raise RuntimeError(f"stage {self.vstage[c]} did not stash skip '{key}'")
                t = tracker.outgoing[key]
                r = routes[key]
                dst = r.pop_vstage % n
                if dst == self.rank:
                    sk_local[(key, i)] = t.detach()
                    continue
                if tuple(t.shape) != tuple(r.shape) or t.dtype != r.dtype:
                    raise RuntimeError(f"skip '{key}' is {tuple(t.shape)} {t.dtype}, the popping stage expects "
                                       f"{tuple(r.shape)} {r.dtype} (pass skip_shapes=)")
                sends.append(self._track(f"send skip '{key}' micro-batch {i} to rank {dst}",
                                         self._skip_links.send(self.rank, dst, t)))

        def forward(c: int, i: int) -> None:
            mod = self.modules[c]
            last = self._last(c)
            if self._first(c):
                x = inputs[i]
            else:
                with label_range(f"wait recv act vs{self.vstage[c]} mb{i}"):
                    recv_w[c][i].wait()
                x = recv_x[c][i]
                recv_x[c][i] = recv_w[c][i] = None
                if training:
                    x.requires_grad_(True)
            tracker = skip_tracker(c, i)
            tm = self._timer()
            if tm:
                tm[0].record()
            if training and i < stop:
                rng[c][i] = _RNGState(self.device)
                with torch.no_grad(), enable_checkpointing():
                    y = self._run(mod, x, targets, i, tracker)
            else:
                y = self._run(mod, x, targets, i, tracker)
            if last and (self.loss_fn is not None or getattr(mod, "fused_loss", False)):
                loss = self._loss(mod, y, targets, i)
                losses.append(loss.detach())
                y = loss  # its backward is seeded with 1 / (m * grad_divisor) (_loss_seed)
            if tm:
                tm[1].record()
                events.append(("F", tm))
            stage_in[c][i] = x
            stage_out[c][i] = y if (training and i >= stop) else None
            out_meta[c][i] = torch.empty(y.shape, dtype=y.dtype, device="meta")
            if not last:
                sends.append(self._track(f"send activation: virtual stage {self.vstage[c]} micro-batch {i} to rank "
                                         f"{(self.rank + 1) % n}", chan.send_act(y.detach())))
            ship_skips(c, i, tracker)
            if tracker is not None and training and i >= stop:
                skip_out[c][i] = tracker.outgoing

        def post_grad_recv(c: int, i: int) -> None:
            if not self._last(c) and grad_w[c][i] is None:
                if zc:
                    meta = out_meta[c][i]
                    grad_buf[c][i], work = chan.recv_grad_view(meta.shape, meta.dtype)
                else:
                    grad_buf[c][i] = self._new_act(c, out_meta[c][i])
                    work = chan.recv_grad(grad_buf[c][i])
                grad_w[c][i] = self._track(f"recv gradient: virtual stage {self.vstage[c]} micro-batch {i} from rank "
                                           f"{(self.rank + 1) % n}", work)

        def backward(c: int, i: int) -> None:
            mod = self.modules[c]
            last = self._last(c)
            x = stage_in[c][i]
            if stage_out[c][i] is None:
                # Recompute needs no gradient, so it is issued BEFORE the stream
                # waits on the incoming gradient: the recomputed forward overlaps
                # the gradient transfer and the downstream rank's backward, as
                # the reference's Recompute node does (it hangs off a phony that
                # is not ordered after Wait, /root/reference/pipeline.py:161-185).
                # Recompute with the RNG state of the original forward.
                tr = self._timer()
                if tr:
                    tr[0].record()
                st = rng[c][i]
                devices = [self.device] if self.device.type == "cuda" else []
                tracker = skip_tracker(c, i)
                with label_range(f"recompute vs{self.vstage[c]} mb{i}"), torch.random.fork_rng(devices=devices):
                    torch.set_rng_state(st.cpu)
                    if st.dev is not None:
                        torch.cuda.set_rng_state(st.dev, self.device)
                    with torch.enable_grad(), enable_recomputing():
                        y = self._run(mod, x, targets, i, tracker)
                        if last and (self.loss_fn is not None or getattr(mod, "fused_loss", False)):
                            y = self._loss(mod, y, targets, i)
                if tracker is not None:
                    skip_out[c][i] = tracker.outgoing
                if tr:
                    tr[1].record()
                    events.append(("B", tr))
            else:
                y = stage_out[c][i]
            # Stashed skips are outputs of this chunk too: their gradients
            # (from the popping stage) seed the same backward pass.
            has_loss = last and (self.loss_fn is not None or getattr(mod, "fused_loss", False))
            outs, seeds = [y], [(self._loss_seed(y) if has_loss else None) if last else grad_buf[c][i]]
            for key in self._stashes[c]:
                r = routes[key]
                if not r.has_grad:
                    continue
                if r.pop_vstage % n == self.rank:
                    g = sk_local_grad.pop((key, i))
                else:
                    g, work = sk_grad_rx.pop((key, i))
                    work.wait()
                t = skip_out[c][i][key]
                if t.requires_grad:
                    outs.append(t)
                    seeds.append(g)
            if not last:
                with label_range(f"wait recv grad vs{self.vstage[c]} mb{i}"):
                    grad_w[c][i].wait()
            tm = self._timer()
            if tm:
                tm[0].record()
            torch.autograd.backward(outs, seeds)
            if tm:
                tm[1].record()
                events.append(("B", tm))
            stage_out[c][i] = grad_buf[c][i] = grad_w[c][i] = None
            if not self._first(c):
                sends.append(self._track(f"send gradient: virtual stage {self.vstage[c]} micro-batch {i} to rank "
                                         f"{(self.rank - 1) % n}", chan.send_grad(x.grad)))
            for key in self._pops[c]:
                r = routes[key]
                if not r.has_grad:
                    continue
                leaf = skip_in[c][i][key]
                g = leaf.grad if leaf.grad is not None else torch.zeros_like(leaf)
                src = r.stash_vstage % n
                if src == self.rank:
                    sk_local_grad[(key, i)] = g
                else:
                    sends.append(self._track(f"send skip gradient '{key}' micro-batch {i} to rank {src}",
                                             self._skip_links.send(self.rank, src, g)))
            stage_in[c][i] = rng[c][i] = skip_in[c][i] = skip_out[c][i] = None

        actions = self._actions_of(self.rank, training)

        def post_for(kind: str, c: int, i: int) -> None:
            if kind == "F":
                post_act_recv(c, i)
            else:
                post_grad_recv(c, i)

        started_backward = False
        defer = ops.deferred_wgrad() if (training and self.defer_wgrad) else None
        wd = self.watchdog
        armed = wd.watch("step start") if wd is not None else None
        if armed is not None:
            armed.__enter__()
        try:
            for idx, (kind, c, i) in enumerate(actions):
                self._mark(f"{'forward' if kind == 'F' else 'backward'} virtual stage {self.vstage[c]} "
                           f"micro-batch {i}")
                if lazy:
                    post_for(kind, c, i)  # (normally posted one action ago)
                    if idx + 1 < len(actions):
                        nk, nc, ni = actions[idx + 1]
                        if nk == "F" or out_meta[nc][ni] is not None:  # a gradient needs its forward's shape
                            post_for(nk, nc, ni)
                if kind == "F":
                    with label_range(f"F vs{self.vstage[c]} mb{i}"), torch.set_grad_enabled(training):
                        forward(c, i)
                else:
                    if not started_backward:
                        started_backward = True
                        if defer is not None:
                            defer.__enter__()
                        with label_range("post recvs: gradients"):
                            if self.schedule == "gpipe" and not lazy:
                                # Post all (zero-copy) gradient receives of the drain phase at
                                # once, in the downstream rank's send order (reverse).
                                for cc in reversed(range(v)):
                                    for k in reversed(range(m)):
                                        post_grad_recv(cc, k)
                            if self._skip_links is not None:
                                self._post_skip_recvs(sk_grad_rx, training, grad=True)
                    with label_range(f"B vs{self.vstage[c]} mb{i}"):
                        post_grad_recv(c, i)
                        backward(c, i)
                if self.sync_debug and self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
            if defer is not None and started_backward:
                self._mark("deferred weight gradients")
                tm = self._timer()
                if tm:
                    tm[0].record()
                with label_range("wgrad flush"):
                    defer.__exit__(None, None, None)  # the deferred weight-gradient GEMMs
                defer = None
                if tm:
                    tm[1].record()
                    events.append(("B", tm))
            self._mark("waiting for this step's sends")
            with label_range("wait sends"):
                for w in sends:
                    w.wait()
            end_step = getattr(chan, "end_step", None)
            if end_step is not None:
                end_step()  # zero-copy receive slots: released behind the step's last reader
        except BaseException as exc:
            self._on_error(exc)
            raise
        finally:
            if defer is not None and started_backward:
                defer.__exit__(RuntimeError, None, None)
            if armed is not None:
                armed.__exit__(None, None, None)
            # attention keep words carried from checkpointed forwards to their recomputes (ops/attention.py):
            # every recompute of the step has run, so any leftover (an aborted step) is dropped here
            _clear_keep_words()
        self._mark("step done")

        stats.losses = losses
        if events:
            torch.cuda.synchronize(self.device)
            for kind, (a, b) in events:
                ms = a.elapsed_time(b)
                (stats.forward_ms if kind == "F" else stats.backward_ms).append(ms)
            stats.busy_ms = sum(stats.forward_ms) + sum(stats.backward_ms)
        stats.step_ms = (time.perf_counter() - t0) * 1e3
        return stats

    def _on_error(self, exc: BaseException) -> None:
        """An action raised: say where, list the transfers left in flight.

        The exception then propagates (the process ends and ``torchrun`` stops
        the peers, which would otherwise wait for this rank's sends)."""
        import sys

        lines = [f"[mipipe engine] rank {self.rank}: {type(exc).__name__} during {self._action}: {exc}"]
        abort = getattr(self.chan, "abort", None)
        if abort is not None:
            abort()  # peers blocked on this rank's IPC links fail fast instead of timing out
        if self.watchdog is not None:
            left = self.watchdog.pending.unfinished()
            if left:
                lines.append(f"[mipipe engine] rank {self.rank}: {len(left)} transfer(s) left in flight:")
                lines.extend(f"[mipipe engine]   {u}" for u in left[:32])
        print("\n".join(lines), file=sys.stderr, flush=True)


def make_transport(ranks: Sequence[int], *, device: torch.device, chunks: int, virtual: int, recv_bytes: int,
                   transport: str = "auto", transport_options: Optional[dict] = None, watchdog=None):
    """The stage-boundary channels of one pipeline rank: ``(channels, name, note)``.

    What :class:`PipelineEngine` builds from ``transport=``; callable on its own
    so a driver can set the links up before it allocates its stages (bench.py
    does).  ``recv_bytes``: the largest activation this rank receives per
    micro-batch.  Collective over ``ranks``.

    ``transport="auto"``: stage boundaries that keep kernels off the GEMMs'
    CUs.  An RCCL send/receive is a kernel that spins on its CUs until the
    data has moved (footprint of torch's ``rcclGenericKernel``: 256 threads,
    19.7 KiB LDS, ~270 registers -- it can never share a CU with a 256x256
    GEMM block); ``profiles/cu_hold_r5.txt`` measures what such a block
    costs the PP=1 step.  The IPC links move the payload AND the completion
    flag with the DMA engines (the link's copy stream, ``sdma``: two
    ``hipMemcpyDeviceToDeviceNoCU`` copies -- no kernel on that stream); the
    consumer's own stream waits for the flag in order with its work (a
    ``hipStreamWaitValue64``, which this ROCm runs as a one-wave kernel that
    spins only while that stream would idle anyway) and releases the slot
    with one stream write per link and step (profiles/ipc_cu_free_r6.txt) --
    the reference's own design (copies on dedicated copy streams, event
    waits: /root/reference/README.md:193-237, 332-369).  Ranks sharing one GPU
    (rehearsals) copy on the producer's stream (``inline``).  The links are
    self-tested first (:meth:`IpcChannels.self_test`); if any rank fails,
    every rank falls back to RCCL and the note says why.  CPU: RCCL-style
    channels over gloo."""
    dev = torch.device(device)
    wrap = virtual > 1
    note = None
    if transport == "auto":
        if dev.type != "cuda":
            chan = Channels(ranks, wrap=wrap)
            chan.warmup(dev)
            name = "rccl"
        else:
            from .ipc import IpcChannels, ranks_share_a_device, verified_ipc

            shared = ranks_share_a_device(dev)
            opts = dict(transport_options or {})
            opts.setdefault("slots", chunks * virtual)
            opts.setdefault("engine", "inline" if shared else "sdma")
            fallback = {}

            def make_rccl():
                if shared:
                    raise RuntimeError("IPC links failed their self-test and RCCL refuses two ranks on one GPU: "
                                       + str(fallback.get("why")))
                ch = Channels(ranks, wrap=wrap)
                with (watchdog.watch("RCCL channel warm-up") if watchdog is not None else _null()):
                    ch.warmup(dev)
                return ch

            with (watchdog.watch("IPC link self-test") if watchdog is not None else _null()):
                chan, why = verified_ipc(
                    lambda: IpcChannels(ranks, wrap=wrap, device=dev, recv_bytes=recv_bytes, **opts), make_rccl, dev)
            if why is not None:
                note = f"IPC self-test failed, fell back to RCCL: {why}"
                warnings.warn(note)
                name = "rccl"
            else:
                name = f"ipc-{opts['engine']}"
    elif transport == "ipc":
        from .ipc import IpcChannels

        opts = dict(transport_options or {})
        # one slot per message a link carries in a step: a sender never
        # blocks inside a step (with fewer, a looping placement can
        # deadlock: rank 0 would wait for a slot rank 1 frees only
        # after rank 0's own later chunk has run)
        opts.setdefault("slots", chunks * virtual)
        chan = IpcChannels(ranks, wrap=wrap, device=dev, recv_bytes=recv_bytes, **opts)
        name = "ipc"
    elif transport == "rccl":
        chan = Channels(ranks, wrap=wrap)
        with (watchdog.watch("RCCL channel warm-up") if watchdog is not None else _null()):
            chan.warmup(dev)
        name = "rccl"
    else:
        raise ValueError(f"transport must be 'auto', 'rccl' or 'ipc', got {transport!r}")
    try:
        chan.transport_name, chan.transport_note = name, note
    except AttributeError:  # channels without a __dict__: the engine names them by type
        pass
    return chan, name, note
