"""The loader refuses a ``_C.so`` that was not built from the checked-out
sources: ``mipipe.build`` embeds a digest of ``csrc/``,
``_native_loader`` recomputes it at import."""
import os
import shutil

import pytest

from mipipe import _native_loader as L


def test_digest_tracks_every_source_byte(tmp_path):
    src = tmp_path / "csrc"
    shutil.copytree(L.CSRC, src)
    d0 = L.source_digest(str(src))
    assert d0 == L.source_digest(L.CSRC)
    victim = src / "kernels" / "gemm.hip"
    data = bytearray(victim.read_bytes())
    data[len(data) // 2] ^= 0x01
    victim.write_bytes(bytes(data))
    assert L.source_digest(str(src)) != d0
    victim.write_bytes(bytes(data[: len(data) // 2]) + bytes([data[len(data) // 2] ^ 0x01]) + bytes(data[len(data) // 2 + 1:]))
    assert L.source_digest(str(src)) == d0
    (src / "runtime" / "new.h").write_text("// new file\n")
    assert L.source_digest(str(src)) != d0


class _FakeMod:
    def __init__(self, digest):
        self._d = digest

    def source_digest(self):
        return self._d


def test_loader_refuses_stale_binary(tmp_path, monkeypatch):
    src = tmp_path / "csrc"
    shutil.copytree(L.CSRC, src)
    good = _FakeMod(L.source_digest(str(src)))
    L.check_digest(good, str(src))  # matches: accepted
    victim = src / "bindings.cpp"
    victim.write_bytes(victim.read_bytes() + b" ")
    with pytest.raises(L.StaleExtensionError, match="stale"):
        L.check_digest(good, str(src))
    with pytest.raises(L.StaleExtensionError):
        L.check_digest(object(), str(src))  # a binary without a digest
    monkeypatch.setenv("MIPIPE_ALLOW_STALE", "1")
    L.check_digest(good, str(src))  # deliberate override


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(L.__file__), "_C.so")), reason="not built")
def test_built_extension_matches_checkout():
    """Whatever is on disk: a loaded extension matches the sources, a stale one
    is refused with StaleExtensionError (never loaded)."""
    mod = L._load()
    if mod is None:
        assert isinstance(L.load_error(), L.StaleExtensionError), L.load_error()
    else:
        assert mod.source_digest() == L.source_digest()
