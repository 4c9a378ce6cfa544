"""Locates the in-tree native extension ``mipipe/_C*.so``.

Two entry points:

* :func:`runtime` -- used by the scheduler for streams / events / peer copies.
  Returns ``None`` when there is no GPU (CPU plumbing runs) so the pure-host
  path keeps working.
* :func:`kernels` -- used by ``mipipe.ops``.  On a machine with a GPU a missing
  or stale extension is a hard error: the hot path must never fall back to
  eager PyTorch silently (set ``MIPIPE_ALLOW_EAGER=1`` to opt in explicitly).
"""
from __future__ import annotations

import importlib
import os
import threading
from types import ModuleType
from typing import Optional

_lock = threading.Lock()
_module: Optional[ModuleType] = None
_load_error: Optional[BaseException] = None
_tried = False


def _load() -> Optional[ModuleType]:
    global _module, _load_error, _tried
    if _tried:
        return _module
    with _lock:
        if _tried:
            return _module
        try:
            import torch  # noqa: F401  (the extension links against libtorch)

            _module = importlib.import_module("mipipe._C")
        except BaseException as exc:  # ImportError, OSError (bad .so), ...
            _module = None
            _load_error = exc
        _tried = True
    return _module


def load_error() -> Optional[BaseException]:
    _load()
    return _load_error


def available() -> bool:
    return _load() is not None


def _gpu_present() -> bool:
    import torch

    return torch.cuda.is_available()


def runtime() -> Optional[ModuleType]:
    """Native runtime when a GPU is present and the extension loaded."""
    if os.environ.get("MIPIPE_DISABLE_NATIVE_RUNTIME") == "1":
        return None
    mod = _load()
    if mod is None or not _gpu_present():
        return None
    return mod


def kernels() -> ModuleType:
    """The kernel module; raises if it is missing."""
    mod = _load()
    if mod is None:
        raise RuntimeError(
            "mipipe native extension (mipipe/_C.so) is not built or failed to load: "
            f"{_load_error!r}. Run `python -m mipipe.build` (or __graft_entry__.build())."
        )
    return mod


def allow_eager() -> bool:
    return os.environ.get("MIPIPE_ALLOW_EAGER") == "1"
