"""Locates the in-tree native extension ``mipipe/_C*.so``.

Two entry points:

* :func:`runtime` -- used by the scheduler for streams / events / peer copies.
  Returns ``None`` when there is no GPU (CPU plumbing runs) so the pure-host
  path keeps working.
* :func:`kernels` -- used by ``mipipe.ops``.  On a machine with a GPU a missing
  or stale extension is a hard error: the hot path must never fall back to
  eager PyTorch silently (set ``MIPIPE_ALLOW_EAGER=1`` to opt in explicitly).

Staleness: ``mipipe.build`` embeds :func:`source_digest` (SHA-256 over every
file under ``csrc/``) into ``_C.so`` as ``_C.source_digest()``.  When the
sources sit next to the package (an in-tree checkout, which is what travels to
a GPU box) the loader recomputes it and REFUSES a binary built from other
sources, so no measurement can come from a ``.so`` that does not match the code
beside it.  ``MIPIPE_ALLOW_STALE=1`` accepts one deliberately (A/B binaries).
"""
from __future__ import annotations

import glob
import hashlib
import importlib
import os
import threading
from types import ModuleType
from typing import Optional

_lock = threading.Lock()
_module: Optional[ModuleType] = None
_load_error: Optional[BaseException] = None
_tried = False

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
_SOURCE_EXTS = (".hip", ".cpp", ".cc", ".h", ".hpp")


class StaleExtensionError(ImportError):
    """``_C.so`` was built from different sources than the ones checked out."""


def source_digest(csrc: str = None) -> str:
    """SHA-256 (hex, 32 chars) over the relative path and bytes of every
    native source under ``csrc`` in sorted order."""
    root = csrc or CSRC
    h = hashlib.sha256()
    paths = [p for p in glob.glob(os.path.join(root, "**", "*"), recursive=True)
             if os.path.isfile(p) and p.endswith(_SOURCE_EXTS)]
    for path in sorted(paths, key=lambda p: os.path.relpath(p, root)):
        h.update(os.path.relpath(path, root).replace(os.sep, "/").encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:32]


def check_digest(mod: ModuleType, csrc: str = None) -> None:
    """Raises :class:`StaleExtensionError` when ``mod`` was not built from the
    sources under ``csrc`` (skipped when the sources are absent, e.g. an
    installed wheel, or with ``MIPIPE_ALLOW_STALE=1``)."""
    root = csrc or CSRC
    if os.environ.get("MIPIPE_ALLOW_STALE") == "1" or not os.path.isdir(root):
        return
    built = mod.source_digest() if hasattr(mod, "source_digest") else "<none>"
    want = source_digest(root)
    if built != want:
        raise StaleExtensionError(
            f"mipipe/_C.so is stale: built from sources {built}, the checkout has {want}. "
            "Rebuild with `python -m mipipe.build` (MIPIPE_ALLOW_STALE=1 accepts it deliberately).")


def _load() -> Optional[ModuleType]:
    global _module, _load_error, _tried
    if _tried:
        return _module
    with _lock:
        if _tried:
            return _module
        try:
            import torch  # noqa: F401  (the extension links against libtorch)

            mod = importlib.import_module("mipipe._C")
            check_digest(mod)
            _module = mod
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
    """Native runtime when a GPU is present (``None`` on CPU-only hosts).  On a
    GPU host a missing or stale extension raises instead of silently running
    the pipeline on torch's own streams."""
    if os.environ.get("MIPIPE_DISABLE_NATIVE_RUNTIME") == "1":
        return None
    if not _gpu_present():
        return None
    return kernels()


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
