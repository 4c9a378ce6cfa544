"""Phony tensors: zero-element tensors used purely as autograd edges.

Behaviour documented at ``/root/reference/README.md:140-160``: one cached empty
tensor per ``(device, requires_grad)``, allocated on the device's *default*
stream so that caching-allocator stream bookkeeping never ties it to a copy
stream.  A phony carries no data, so allocating it costs no kernel (§2.3 K18).
"""
from __future__ import annotations

import threading
from typing import Dict, Tuple

import torch

from .stream import default_stream, use_device, use_stream

__all__ = ["get_phony"]

_cache: Dict[Tuple[torch.device, bool], torch.Tensor] = {}
_cache_lock = threading.Lock()


def get_phony(device: torch.device, *, requires_grad: bool) -> torch.Tensor:
    """Returns the cached phony for ``device``.

    The result is a leaf.  Callers that need a phony *output* of an autograd
    function must return ``phony.detach()`` so the cached leaf is never
    re-attached to some graph.
    """
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (device, requires_grad)
    phony = _cache.get(key)
    if phony is not None:
        return phony
    with _cache_lock:
        phony = _cache.get(key)
        if phony is None:
            with use_device(device), use_stream(default_stream(device)):
                phony = torch.empty(0, device=device, requires_grad=requires_grad)
            _cache[key] = phony
    return phony
