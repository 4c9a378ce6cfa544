"""The ``Pipe`` module: synchronous GPipe pipeline parallelism.

API parity with ``torch.distributed.pipeline.sync.Pipe`` as vendored in
``/root/reference/pipe.py``:

* ``Pipe(module, chunks=1, checkpoint="except_last", deferred_batch_norm=False)``
  (``pipe.py:308-314``) with the same argument validation (``pipe.py:324-330``);
* placement is implicit from each child's parameters, or explicit through
  :class:`WithDevice`; consecutive children on the same device form one
  partition, and every CPU child is its own partition (``pipe.py:191-218``);
* ``len``/indexing/iteration over the layers (``pipe.py:358-386``);
* ``cuda()``/``cpu()``/``to(device)`` are denied, ``to(dtype)`` is allowed
  (``pipe.py:390-415``);
* one copy stream per (partition, micro-batch) (``pipe.py:417-429``);
* ``forward`` = check -> scatter -> run -> gather, returning an RRef
  (``pipe.py:431-494``; see :mod:`mipipe.rref`).

Extras: ``return_rref=False`` returns the plain output like the reference's
edited copy (``pipe.py:491-494``); :meth:`Pipe.close` stops the workers.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Iterator, List, Optional, Tuple, Union, cast

import torch
from torch import Tensor, nn

from . import microbatch
from .batchnorm import DeferredBatchNorm
from .pipeline import Pipeline
from .rref import make_rref
from .skip.layout import SkipLayout, inspect_skip_layout
from .skip.skippable import verify_skippables
from .stream import AbstractStream, new_stream

__all__ = ["Pipe", "BalanceError", "PipeSequential", "WithDevice"]

Device = Union[torch.device, int, str]

_CHECKPOINT_MODES = ("always", "except_last", "never")


class BalanceError(ValueError):
    """Raised when a requested balance does not fit the module."""


class PipeSequential(nn.Sequential):
    """``nn.Sequential`` whose layers may take several positional inputs.

    A tuple produced by one layer is splatted into the next; any other value is
    passed as a single argument.
    """

    def forward(self, *inputs):  # type: ignore[override]
        carry: Any = inputs
        for layer in self:
            carry = layer(*carry) if isinstance(carry, tuple) else layer(carry)
        return carry


class WithDevice(nn.Module):
    """Pins a child of the ``nn.Sequential`` given to :class:`Pipe` to ``device``.

    Needed for parameter-less layers (dropout, activation, reshapes) that would
    otherwise be treated as CPU layers.  ``Pipe`` moves the wrapped module there.
    """

    def __init__(self, module: nn.Module, device: Device) -> None:
        super().__init__()
        self._module = module
        self._device = torch.device(device)

    def forward(self, *args, **kwargs):
        return self._module(*args, **kwargs)

    @property
    def module(self) -> nn.Module:
        return self._module

    @property
    def device(self) -> torch.device:
        return self._device


def _verify_module(module: nn.Sequential) -> None:
    if not isinstance(module, nn.Sequential):
        raise TypeError("module must be nn.Sequential to be partitioned")
    if len(list(module.named_children())) != len(module):
        raise ValueError("module with duplicate children is not supported")


def _module_device(module: nn.Module) -> torch.device:
    """The single device holding all of ``module``'s parameters (CPU if none)."""
    found: Optional[torch.device] = None
    for p in module.parameters():
        if found is None:
            found = p.device
        elif p.device != found:
            raise ValueError(
                f"nn.Module: {module}, should have all parameters on a single device,"
                " please use .to() to place the module on a single device"
            )
    return found if found is not None else torch.device("cpu")


# Upstream private name.
_retrieve_device = _module_device


def _flatten_partition(layers: List[nn.Module]) -> PipeSequential:
    flat: List[nn.Module] = []
    for layer in layers:
        if isinstance(layer, nn.Sequential):
            flat.extend(layer.children())
        else:
            flat.append(layer)
    return PipeSequential(*flat)


def _placed_children(module: nn.Sequential) -> List[Tuple[Optional[torch.device], nn.Module]]:
    """(device, child) per child; ``WithDevice`` children are moved to their
    device.  The device is ``None`` for a child with no parameters or buffers
    that is not pinned (an activation, a reshape): it runs wherever its
    partition runs."""
    out: List[Tuple[Optional[torch.device], nn.Module]] = []
    for _, child in module.named_children():
        if isinstance(child, WithDevice):
            device: Optional[torch.device] = child.device
            child = child.module
            child.to(device)
        elif next(iter(child.parameters()), None) is None and next(iter(child.buffers()), None) is None:
            device = None
        else:
            device = _module_device(child)
        out.append((device, child))
    return out


def _split_module(module: nn.Sequential, balance: Optional[List[int]] = None
                  ) -> Tuple[List[nn.Sequential], List[torch.device]]:
    """Splits ``module`` into partitions.

    Without ``balance`` (the reference rule, ``/root/reference/pipe.py:191-218``):
    consecutive children on the same device form one partition and every CPU
    child is its own.  With ``balance`` (torchgpipe's explicit split): partition
    ``k`` is the next ``balance[k]`` children, which must share one device --
    several partitions may then sit on the SAME GPU, each computing on a stream
    of its own, with real stage boundaries (copy streams, Copy/Wait) between
    them."""
    placed = _placed_children(module)
    if balance is None:
        groups: List[Tuple[torch.device, List[nn.Module]]] = []
        for device, child in placed:
            device = device if device is not None else torch.device("cpu")
            if groups and groups[-1][0] == device and device.type != "cpu":
                groups[-1][1].append(child)
            else:
                groups.append((device, [child]))
    else:
        balance = [int(b) for b in balance]
        if any(b <= 0 for b in balance):
            raise BalanceError(f"all balance numbers must be positive integer (balance: {balance})")
        if sum(balance) != len(placed):
            raise BalanceError(f"module and sum of balance have different length "
                               f"(module: {len(placed)}, sum of balance: {sum(balance)})")
        groups = []
        start = 0
        for k, b in enumerate(balance):
            chunk = placed[start:start + b]
            start += b
            devs = {d for d, _ in chunk if d is not None}
            if len(devs) > 1:
                raise ValueError(f"partition {k} of balance {balance} spans several devices: "
                                 f"{sorted(str(d) for d in devs)}")
            groups.append((devs.pop() if devs else torch.device("cpu"), [c for _, c in chunk]))
    partitions = cast(List[nn.Sequential], nn.ModuleList([_flatten_partition(layers) for _, layers in groups]))
    devices = [d for d, _ in groups]
    return partitions, devices


def _verify_splitting(module: nn.Sequential, partitions: List[nn.Sequential], devices: List[torch.device]) -> None:
    """A parameter shared between partitions on *different* devices is an error."""
    total = len(list(module.parameters()))
    per_child = sum(len(list(c.parameters())) for c in module.children())
    if total == per_child:
        return  # nothing is shared
    owner: dict = {}
    for idx, part in enumerate(partitions):
        for p in part.parameters():
            prev = owner.get(id(p))
            if prev is not None and devices[prev] != devices[idx]:
                raise ValueError("module with duplicate parameters on distinct devices is not supported")
            owner.setdefault(id(p), idx)


def _enable_peer_access(devices: List[torch.device]) -> None:
    """Direct xGMI access between every pair of the pipeline's GPUs.

    Without it a ``hipMemcpyPeerAsync`` between two devices may be staged
    through host memory; with it the SDMA engine (or a kernel) reads/writes the
    peer's HBM over the link that joins them.  Idempotent; a no-op without the
    native runtime or with fewer than two GPUs."""
    indices = sorted({d.index if d.index is not None else torch.cuda.current_device()
                      for d in devices if d.type == "cuda"})
    if len(indices) < 2:
        return
    from .stream import _native

    rt = _native()
    if rt is not None:
        rt.enable_peer_access(indices)


def _check_queues_for_shared_gpu(streams: int) -> None:
    """Warns when the stage and copy streams of partitions sharing a GPU will
    alias onto few in-order hardware queues: HIP maps streams onto
    ``GPU_MAX_HW_QUEUES`` queues (default 4), and two stage streams on one
    queue run in submission order -- the stages then do not overlap
    (``profiles/hw_queue_sharing.txt``).  Read at HIP initialisation."""
    import os
    import warnings

    try:
        q = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    except ValueError:
        q = 4
    if q < min(streams, 16):
        warnings.warn(f"mipipe Pipe: several partitions share a GPU with GPU_MAX_HW_QUEUES={q}; their stage "
                      f"streams may share in-order hardware queues and not overlap -- export "
                      f"GPU_MAX_HW_QUEUES={min(streams, 16)} before the process initialises HIP",
                      RuntimeWarning, stacklevel=3)


_MOVING_DENIED = "denied to move parameters and buffers, because Pipe should manage device placement"
MOVING_DENIED = TypeError(_MOVING_DENIED)


class Pipe(nn.Module):
    """Wraps an ``nn.Sequential`` for synchronous pipeline-parallel training.

    Args:
        module: the sequential model; children must already sit on their devices
            (or be wrapped in :class:`WithDevice`).
        chunks: number of micro-batches per mini-batch.
        checkpoint: ``"always"``, ``"except_last"`` or ``"never"``.
        deferred_batch_norm: track BatchNorm statistics over the whole mini-batch.
        return_rref: return an RRef (upstream behaviour, default) or the output.
        copy_streams: copy streams per partition, shared round-robin by the
            micro-batches.  ``1`` (default): one per partition.  ``None``: the
            reference's one stream per (partition, micro-batch)
            (``/root/reference/pipe.py:417-429``).  Every stream a HIP process
            drives gets a hardware queue of its own (up to
            ``GPU_MAX_HW_QUEUES``), and with chunks x partitions queues busy at
            once the GPU time-slices them: on one MI355X the reference's
            structure (ref_main fp32, 2 partitions, chunks 4 -> 8 copy streams)
            ran 27.5k tok/s with per-micro-batch copy streams against 36.8k
            with one per partition, the engine's 36.1k
            (``profiles/pipe_gap_r5.txt``).
        balance: explicit partition sizes (number of top-level children per
            partition, torchgpipe style).  Lets several partitions share a
            GPU (see ``stage_streams``).
        stage_streams: how partitions that share a GPU compute.
            ``"dedicated"`` (default): every later partition on a device gets a
            stream of its own, so neighbouring stages' kernels overlap.
            ``"shared"``: all of them on the device's current stream, the
            reference's choice (``streams = [current_stream(d) for d in
            devices]``, ``/root/reference/pipeline.py:158``).  Measured on one
            MI355X (ref_main fp32, 2 partitions, one copy stream each): 36.8k
            tok/s dedicated, 35.5k shared (``profiles/pipe_gap_r5.txt``).
        copy_same_device: make a boundary between two partitions of the same
            GPU a real device-to-device copy on the copy streams (the native
            ``peer_copy`` path a multi-GPU boundary takes) instead of handing
            the tensor over in place.
        copy_engine: ``"sdma"`` (DMA engines, default) or ``"blit"`` (a copy
            kernel) for native stage transfers; ``None`` reads
            ``$MIPIPE_COPY_ENGINE``.
    """

    def __init__(
        self,
        module: nn.Sequential,
        chunks: int = 1,
        checkpoint: str = "except_last",
        deferred_batch_norm: bool = False,
        *,
        return_rref: bool = True,
        copy_streams: Optional[int] = 1,
        balance: Optional[List[int]] = None,
        copy_same_device: bool = False,
        copy_engine: Optional[str] = None,
        stage_streams: str = "dedicated",
    ) -> None:
        super().__init__()
        chunks = int(chunks)
        checkpoint = str(checkpoint)
        if chunks <= 0:
            raise ValueError("number of chunks must be positive integer")
        if checkpoint not in _CHECKPOINT_MODES:
            raise ValueError("checkpoint is not one of 'always', 'except_last', or 'never'")

        _verify_module(module)
        verify_skippables(module)

        if copy_streams is not None and int(copy_streams) <= 0:
            raise ValueError("copy_streams must be a positive integer or None")
        self.chunks = chunks
        self.checkpoint = checkpoint
        self.return_rref = return_rref
        self.copy_streams_per_partition = None if copy_streams is None else int(copy_streams)

        if deferred_batch_norm:
            module = DeferredBatchNorm.convert_deferred_batch_norm(module, chunks)

        from .copy import COPY_ENGINES

        if copy_engine is not None and copy_engine not in COPY_ENGINES:
            raise ValueError(f"copy_engine must be one of {sorted(COPY_ENGINES)}, got {copy_engine!r}")
        self.copy_same_device = bool(copy_same_device)
        self.copy_engine = copy_engine
        if stage_streams not in ("shared", "dedicated"):
            raise ValueError(f"stage_streams must be 'shared' or 'dedicated', got {stage_streams!r}")
        self.stage_streams = stage_streams

        self.partitions, self.devices = _split_module(module, balance)
        _verify_splitting(module, self.partitions, self.devices)
        _enable_peer_access(self.devices)

        self._copy_streams: List[List[AbstractStream]] = []
        self._skip_layout: SkipLayout = inspect_skip_layout(self.partitions)
        copy_streams = self._ensure_copy_streams()
        self._compute_streams = self._ensure_compute_streams()
        if any(st is not None for st in self._compute_streams):
            _check_queues_for_shared_gpu(len(self.partitions) * (1 + self.chunks))

        # The pipeline derives the checkpoint boundary from the actual number of
        # micro-batches at run time (see pipeline.checkpoint_stop_for).
        self.pipeline = Pipeline(self.partitions, self.devices, copy_streams, self._skip_layout, checkpoint,
                                 compute_streams=self._compute_streams, copy_same_device=self.copy_same_device,
                                 copy_engine=copy_engine)

    # -- sequence façade -------------------------------------------------------
    def __len__(self) -> int:
        return sum(len(p) for p in self.partitions)

    def __getitem__(self, index: int) -> nn.Module:
        layers = [layer for part in self.partitions for layer in part]
        if -len(layers) <= index < len(layers):
            return layers[index]
        raise IndexError

    def __iter__(self) -> Iterator[nn.Module]:
        for part in self.partitions:
            yield from part

    # -- placement guards ----------------------------------------------------------
    def cuda(self, device: Optional[Device] = None) -> "Pipe":
        raise MOVING_DENIED

    def cpu(self) -> "Pipe":
        raise MOVING_DENIED

    def to(self, *args: Any, **kwargs: Any) -> "Pipe":
        # Only dtype casts are allowed: to(dtype[, non_blocking]).
        if "device" in kwargs or "tensor" in kwargs:
            raise MOVING_DENIED
        if args and (isinstance(args[0], (torch.device, int, str)) or torch.is_tensor(args[0])):
            raise MOVING_DENIED
        return super().to(*args, **kwargs)

    # -- streams -------------------------------------------------------------------
    def _ensure_copy_streams(self) -> List[List[AbstractStream]]:
        """Copy streams per (partition, micro-batch), created once and cached --
        reusing streams keeps the caching allocator's per-stream pools small
        (``/root/reference/pipe.py:417-424``).  ``copy_streams=None`` gives the
        reference's one dedicated stream per (partition, micro-batch); the
        default (1) shares one per partition across its micro-batches, a
        measured deviation (profiles/pipe_gap_r5.txt)."""
        if not self._copy_streams:
            k = self.copy_streams_per_partition
            for device in self.devices:
                if k is None:
                    self._copy_streams.append([new_stream(device) for _ in range(self.chunks)])
                else:
                    pool = [new_stream(device) for _ in range(min(k, self.chunks))]
                    self._copy_streams.append([pool[i % len(pool)] for i in range(self.chunks)])
        return self._copy_streams

    def _ensure_compute_streams(self) -> List[Optional[AbstractStream]]:
        """Compute stream per partition: ``None`` (= the device's current
        stream, the reference's choice, ``/root/reference/pipeline.py:158``)
        for every partition with ``stage_streams="shared"``; with
        ``"dedicated"``, for the first partition on each device only, and a
        stream of its own for every later partition on the same GPU (then
        micro-batch i+1 of stage j-1 can overlap micro-batch i of stage j)."""
        seen = set()
        out: List[Optional[AbstractStream]] = []
        for device in self.devices:
            key = (device.type, device.index if device.index is not None else -1)
            if device.type == "cuda" and key in seen and self.stage_streams == "dedicated":
                out.append(new_stream(device))
            else:
                out.append(None)
            seen.add(key)
        return out

    def close(self) -> None:
        self.pipeline.close()

    # -- forward -------------------------------------------------------------------
    def forward(self, *inputs: Any):  # type: ignore[override]
        """Runs one mini-batch through the pipeline.

        Tensors are split on dim 0 into ``chunks`` micro-batches (fewer if the
        batch is smaller); non-tensors and :class:`~mipipe.NoChunk` tensors are
        replicated.  All input tensors must be on the first partition's device.
        Returns an RRef to the output (or the output with ``return_rref=False``).
        """
        first_device = self.devices[0] if self.devices else torch.device("cpu")
        microbatch.check(first_device, *inputs)

        if not self.devices:
            # An empty Sequential is legal: identity.
            value = inputs[0] if len(inputs) == 1 else inputs
            return make_rref(value) if self.return_rref else value

        batches = microbatch.scatter(*inputs, chunks=self.chunks)
        self.pipeline.run(batches)
        output = microbatch.gather(batches)
        return make_rref(output) if self.return_rref else output
