"""Device and stream abstraction.

Parity target: the ``stream`` module the reference imports at
``/root/reference/pipe.py:22`` and ``/root/reference/pipeline.py:22`` and quotes at
``/root/reference/README.md:156,196-208,344-356``.

The pipeline only ever sees an :data:`AbstractStream`: either a real HIP stream
(``torch.cuda.Stream`` is a HIP stream on ROCm) or :data:`CPUStream`, a token that
stands for "synchronous host execution".  Every helper below accepts both, so
the whole scheduler runs unchanged on CPU-only hosts (the plumbing tests) and on
MI355X devices.

MI355X specifics:

* :func:`new_stream` hands out *dedicated* non-blocking HIP streams from the
  native pool in ``mipipe._C`` (``hipStreamCreateWithPriority``) instead of
  torch's 32-entry round-robin pool, so the ``chunks x stages`` copy streams of a
  deep pipeline never alias each other.
* :func:`wait_stream` orders two streams with a pooled, timing-disabled
  ``hipEvent`` (record + ``hipStreamWaitEvent``) from the same extension; no
  event object is created or destroyed per call.
"""
from __future__ import annotations

from contextlib import contextmanager
from typing import Generator, List, Union, cast

import torch

__all__ = [
    "CPUStream",
    "CPUStreamType",
    "AbstractStream",
    "new_stream",
    "current_stream",
    "default_stream",
    "use_device",
    "use_stream",
    "get_device",
    "wait_stream",
    "record_stream",
    "is_cuda",
    "as_cuda",
]


class CPUStreamType:
    """Placeholder stream for host devices: work on it is already ordered."""

    _instance = None

    def __new__(cls):  # singleton, so ``is CPUStream`` checks are cheap
        if cls._instance is None:
            cls._instance = super().__new__(cls)
        return cls._instance

    def __repr__(self) -> str:
        return "CPUStream"

    def synchronize(self) -> None:  # API symmetry with torch.cuda.Stream
        return None


CPUStream = CPUStreamType()

AbstractStream = Union[torch.cuda.Stream, CPUStreamType]


def _native():
    """The native runtime, or ``None`` when it is not built / no GPU is present."""
    from . import _native_loader

    return _native_loader.runtime()


def is_cuda(stream: AbstractStream) -> bool:
    return stream is not CPUStream


def as_cuda(stream: AbstractStream) -> torch.cuda.Stream:
    if stream is CPUStream:
        raise TypeError("expected a device stream, got CPUStream")
    return cast(torch.cuda.Stream, stream)


def new_stream(device: torch.device) -> AbstractStream:
    """A fresh stream on ``device`` (``CPUStream`` for host devices)."""
    device = torch.device(device)
    if device.type != "cuda":
        return CPUStream
    rt = _native()
    if rt is not None:
        index = device.index if device.index is not None else torch.cuda.current_device()
        handle = rt.stream_pool_acquire(index)
        return torch.cuda.ExternalStream(handle, device=torch.device("cuda", index))
    return torch.cuda.Stream(device)


def current_stream(device: torch.device) -> AbstractStream:
    device = torch.device(device)
    if device.type != "cuda":
        return CPUStream
    return torch.cuda.current_stream(device)


def default_stream(device: torch.device) -> AbstractStream:
    device = torch.device(device)
    if device.type != "cuda":
        return CPUStream
    return torch.cuda.default_stream(device)


@contextmanager
def use_device(device: torch.device) -> Generator[None, None, None]:
    """Makes ``device`` current for the block (no-op for host devices)."""
    device = torch.device(device)
    if device.type != "cuda":
        yield
        return
    with torch.cuda.device(device):
        yield


@contextmanager
def use_stream(stream: AbstractStream) -> Generator[None, None, None]:
    """Makes ``stream`` current on its device for the block."""
    if stream is CPUStream:
        yield
        return
    with torch.cuda.stream(as_cuda(stream)):
        yield


def get_device(stream: AbstractStream) -> torch.device:
    if stream is CPUStream:
        return torch.device("cpu")
    return as_cuda(stream).device


def wait_stream(source: AbstractStream, target: AbstractStream) -> None:
    """Work queued on ``source`` after this call runs after all work queued on
    ``target`` so far (``source.wait_stream(target)`` semantics, README.md:349-356).

    A host ``source`` waiting on a device ``target`` has to block the host.
    """
    if source is CPUStream:
        if target is not CPUStream:
            as_cuda(target).synchronize()
        return
    if target is CPUStream:
        return  # host work was already issued before anything queued next
    src, tgt = as_cuda(source), as_cuda(target)
    if src == tgt:
        return
    rt = _native()
    if rt is not None and src.device == tgt.device:
        rt.stream_wait(src.cuda_stream, tgt.cuda_stream, src.device.index)
        return
    src.wait_stream(tgt)


def record_stream(tensor: torch.Tensor, stream: AbstractStream) -> None:
    """Tells the caching allocator that ``tensor``'s memory is in use on
    ``stream`` until the work queued there so far completes (§2.2 N4).

    The record goes on the *base storage* so views of a larger block are
    covered as well.
    """
    if stream is CPUStream or not tensor.is_cuda:
        return
    cuda_stream = as_cuda(stream)
    base = tensor.new_empty([0]).set_(tensor.untyped_storage())
    base.record_stream(cuda_stream)


def synchronize_all(devices: List[torch.device]) -> None:
    """Blocks until every device in ``devices`` is idle (debug helper, §5.2)."""
    for d in devices:
        d = torch.device(d)
        if d.type == "cuda":
            torch.cuda.synchronize(d)
