"""Helpers shared by the op wrappers."""
from __future__ import annotations

from types import ModuleType

from torch import Tensor

from .. import _native_loader


def kernels_for(t: Tensor) -> ModuleType:
    """The kernel module for a GPU tensor.  Raises when it is not built: on a
    GPU the hot path must run the HIP kernels, never a silent eager fallback."""
    return _native_loader.kernels()
