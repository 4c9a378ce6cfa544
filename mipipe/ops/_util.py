"""Helpers shared by the op wrappers."""
from __future__ import annotations

from types import ModuleType

from torch import Tensor

from .. import _native_loader


def kernels_for(t: Tensor) -> ModuleType:
    """The kernel module for the GPU tensor ``t``.

    Raises when ``t`` is not on a GPU (the callers route CPU tensors to their
    eager reference before getting here, so a CPU tensor is a caller bug that
    would otherwise surface as an opaque pointer error inside the extension) and
    when the extension is not built: on a GPU the hot path must run the HIP
    kernels, never a silent eager fallback.  The bindings put a device guard on
    the tensor's device, so ``t`` need not be on the current device."""
    if not t.is_cuda:
        raise TypeError(f"mipipe HIP op called with a {t.device.type} tensor; the eager path handles CPU tensors")
    return _native_loader.kernels()
