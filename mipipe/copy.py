"""Copy / Wait: stream-ordered transfer of micro-batches between partitions.

Semantics (``/root/reference/pipeline.py:51-60``, ``README.md:193-237,332-369``):

* ``Copy.apply(prev_stream, next_stream, *xs)`` moves each tensor to
  ``next_stream``'s device with both copy streams current; forward and backward
  are mirror images.  Allocator lifetimes are pinned with :func:`record_stream`
  on both sides (§2.2 N4).
* ``Wait.apply(prev_stream, next_stream, *xs)`` is an identity whose forward makes
  ``next_stream`` wait for ``prev_stream`` and whose backward makes
  ``prev_stream`` wait for ``next_stream``.

MI355X transport: when the native runtime is loaded and both ends are GPUs,
the transfer is one native copy issued on the source copy stream and fenced
with pooled events (``mipipe/csrc/runtime/runtime.cpp``: ``peer_copy``) -- by
default ``hipMemcpyPeerAsync`` (the SDMA engines over the xGMI link between the
two devices, no CUs taken from the GEMMs), or a 16-byte blit kernel pushing
into the peer's HBM (``engine="blit"``).  Otherwise ``Tensor.to(non_blocking=
True)`` is used, which has the same ordering contract.

Between two partitions of the SAME GPU the reference's ``Tensor.to`` is a
no-op alias; :func:`transfer_policy` (``Pipe(copy_same_device=True)``) makes
such a boundary a real device-to-device copy through the same native path, so
a one-GPU run exercises exactly the stream/event/allocator discipline of a
multi-GPU one.  The policy in force when ``Copy`` runs forward is kept for its
backward (which runs later, on an autograd thread).
"""
from __future__ import annotations

import os
import threading
from collections import deque
from contextlib import contextmanager
from typing import Deque, Generator, List, Optional, Tuple

import torch
from torch import Tensor

from .stream import (
    AbstractStream,
    CPUStream,
    _native,
    as_cuda,
    current_stream,
    get_device,
    record_stream,
    use_device,
    use_stream,
    wait_stream,
)

__all__ = ["Copy", "Wait", "transfer", "transfer_policy", "COPY_ENGINES"]

COPY_ENGINES = {"sdma": 0, "blit": 1}

# (copy same-device boundaries?, engine code)
Policy = Tuple[bool, int]


def _default_engine() -> int:
    name = os.environ.get("MIPIPE_COPY_ENGINE", "sdma")
    if name not in COPY_ENGINES:
        raise ValueError(f"MIPIPE_COPY_ENGINE={name!r}: expected one of {sorted(COPY_ENGINES)}")
    return COPY_ENGINES[name]


class _PolicyLocal(threading.local):
    def __init__(self) -> None:
        self.policy: Optional[Policy] = None


_local = _PolicyLocal()


@contextmanager
def transfer_policy(copy_same_device: bool = False, engine: Optional[str] = None) -> Generator[None, None, None]:
    """Transfers started in the block copy same-device boundaries too
    (``copy_same_device``) and use copy engine ``engine`` (``"sdma"`` or
    ``"blit"``; default ``$MIPIPE_COPY_ENGINE`` or sdma)."""
    if engine is not None and engine not in COPY_ENGINES:
        raise ValueError(f"copy engine must be one of {sorted(COPY_ENGINES)}, got {engine!r}")
    prev = _local.policy
    _local.policy = (bool(copy_same_device), COPY_ENGINES[engine] if engine is not None else _default_engine())
    try:
        yield
    finally:
        _local.policy = prev


def current_policy() -> Policy:
    return _local.policy if _local.policy is not None else (False, _default_engine())


def transfer(x: Tensor, prev_stream: AbstractStream, next_stream: AbstractStream,
             policy: Optional[Policy] = None) -> Tensor:
    """Copies ``x`` (already ordered on ``prev_stream``) to ``next_stream``'s device.

    Must be called with both streams current.  Returns a tensor that is valid on
    ``next_stream``.
    """
    dst_device = get_device(next_stream)
    same_device_copy, engine = policy if policy is not None else current_policy()
    if prev_stream is not CPUStream and next_stream is not CPUStream:
        rt = _native()
        src_device = x.device
        if rt is not None and (src_device != dst_device or same_device_copy) and x.numel() > 0:
            src = x.contiguous()
            # Allocate on the destination with the destination copy stream
            # current so the block belongs to that stream's pool.
            with use_device(dst_device):
                y = torch.empty(src.shape, dtype=src.dtype, device=dst_device)
            rt.peer_copy(
                y, src,
                as_cuda(prev_stream).cuda_stream, as_cuda(next_stream).cuda_stream,
                src_device.index, dst_device.index, engine,
            )
            if src is not x:
                record_stream(src, prev_stream)
            return y
    return x.to(dst_device, non_blocking=True)


class Copy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prev_stream: AbstractStream, next_stream: AbstractStream, *inputs):  # type: ignore[override]
        ctx.prev_stream = prev_stream
        ctx.next_stream = next_stream
        ctx.policy = policy = current_policy()

        outputs: List = []
        # The stream that will *consume* the copied tensors on the next device.
        consumer = current_stream(get_device(next_stream))
        with use_stream(prev_stream), use_stream(next_stream):
            for x in inputs:
                if not torch.is_tensor(x):
                    outputs.append(x)
                    continue
                y = transfer(x, prev_stream, next_stream, policy)
                outputs.append(y)
                # ``x`` was allocated on the previous compute stream but is read
                # on ``prev_stream``; ``y`` lives on ``next_stream`` but will be
                # read on the consumer stream.
                record_stream(x, prev_stream)
                record_stream(y, consumer)
        return tuple(outputs)

    @staticmethod
    def backward(ctx, *grad_outputs: Optional[Tensor]):  # type: ignore[override]
        prev_stream = ctx.prev_stream
        next_stream = ctx.next_stream

        grads: Deque[Optional[Tensor]] = deque(maxlen=len(grad_outputs))
        consumer = current_stream(get_device(prev_stream))
        with use_stream(prev_stream), use_stream(next_stream):
            for g in reversed(grad_outputs):
                if g is None:
                    grads.appendleft(None)
                    continue
                y = transfer(g, next_stream, prev_stream, ctx.policy)
                grads.appendleft(y)
                record_stream(g, next_stream)
                record_stream(y, consumer)
        return (None, None) + tuple(grads)


class Wait(torch.autograd.Function):
    """Stream-order handover.  Besides the wait, the handed-over tensors are
    recorded on the stream that will use them (forward: ``next_stream``,
    backward: ``prev_stream``), so the caching allocator cannot recycle their
    blocks while that stream still reads them -- needed once partitions of one
    GPU compute on streams of their own rather than the device's current one."""

    @staticmethod
    def forward(ctx, prev_stream: AbstractStream, next_stream: AbstractStream, *inputs):  # type: ignore[override]
        ctx.prev_stream = prev_stream
        ctx.next_stream = next_stream
        wait_stream(next_stream, prev_stream)
        outs = tuple(x.detach() if torch.is_tensor(x) else x for x in inputs)
        if next_stream is not CPUStream:
            for x in outs:
                if torch.is_tensor(x) and x.is_cuda and x.numel() > 0:
                    record_stream(x, next_stream)
        return outs

    @staticmethod
    def backward(ctx, *grad_inputs: Optional[Tensor]):  # type: ignore[override]
        wait_stream(ctx.prev_stream, ctx.next_stream)
        if ctx.prev_stream is not CPUStream:
            for g in grad_inputs:
                if g is not None and g.is_cuda and g.numel() > 0:
                    record_stream(g, ctx.prev_stream)
        return (None, None) + grad_inputs

