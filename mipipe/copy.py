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
the transfer is one ``hipMemcpyPeerAsync`` (SDMA over the xGMI link between the
two devices) issued on the source copy stream and fenced with pooled events
(``mipipe/csrc/runtime/runtime.cpp``: ``peer_copy``).  Otherwise
``Tensor.to(non_blocking=True)`` is used, which has the same ordering contract.
"""
from __future__ import annotations

from collections import deque
from typing import Deque, List, Optional

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

__all__ = ["Copy", "Wait", "transfer"]


def transfer(x: Tensor, prev_stream: AbstractStream, next_stream: AbstractStream) -> Tensor:
    """Copies ``x`` (already ordered on ``prev_stream``) to ``next_stream``'s device.

    Must be called with both streams current.  Returns a tensor that is valid on
    ``next_stream``.
    """
    dst_device = get_device(next_stream)
    if prev_stream is not CPUStream and next_stream is not CPUStream:
        rt = _native()
        src_device = x.device
        if rt is not None and src_device != dst_device and x.numel() > 0:
            src = x.contiguous()
            # Allocate on the destination with the destination copy stream
            # current so the block belongs to that stream's pool.
            with use_device(dst_device):
                y = torch.empty(src.shape, dtype=src.dtype, device=dst_device)
            rt.peer_copy(
                y, src,
                as_cuda(prev_stream).cuda_stream, as_cuda(next_stream).cuda_stream,
                src_device.index, dst_device.index,
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

        outputs: List = []
        # The stream that will *consume* the copied tensors on the next device.
        consumer = current_stream(get_device(next_stream))
        with use_stream(prev_stream), use_stream(next_stream):
            for x in inputs:
                if not torch.is_tensor(x):
                    outputs.append(x)
                    continue
                y = transfer(x, prev_stream, next_stream)
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
                y = transfer(g, next_stream, prev_stream)
                grads.appendleft(y)
                record_stream(g, next_stream)
                record_stream(y, consumer)
        return (None, None) + tuple(grads)


class Wait(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prev_stream: AbstractStream, next_stream: AbstractStream, *inputs):  # type: ignore[override]
        ctx.prev_stream = prev_stream
        ctx.next_stream = next_stream
        wait_stream(next_stream, prev_stream)
        return tuple(x.detach() if torch.is_tensor(x) else x for x in inputs)

    @staticmethod
    def backward(ctx, *grad_inputs: Optional[Tensor]):  # type: ignore[override]
        wait_stream(ctx.prev_stream, ctx.next_stream)
        return (None, None) + grad_inputs

