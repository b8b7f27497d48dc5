"""Binary provenance of the native libraries: each carries the hash of the sources it was built from, and the
loader refuses one that does not match the tree (a stale library copied next to newer sources)."""
import shutil

import pytest

from transmogrifai_amd.ops import build as B


def test_built_libraries_carry_the_tree_hash():
    B.build_host()
    assert B.embedded_hash(B.HOST_SO) == B.source_hash("host")
    B.verify(B.HOST_SO, "host")
    if B.HIP_SO.exists():
        assert B.embedded_hash(B.HIP_SO) == B.source_hash("hip")


def test_loaded_host_library_reports_its_hash():
    from transmogrifai_amd.ops import _native
    lib = _native.host()
    _native._check_loaded_hash(lib, "host")


def test_stale_library_is_refused(tmp_path):
    B.build_host()
    stale = tmp_path / "libtmog_host.so"
    data = B.HOST_SO.read_bytes()
    good = B.source_hash("host").encode()
    stale.write_bytes(data.replace(good, b"0" * 64))
    assert B.embedded_hash(stale) == "0" * 64
    assert B._stale(stale, "host")
    with pytest.raises(RuntimeError, match="built from other sources"):
        B.verify(stale, "host")


def test_edited_source_makes_the_library_stale(tmp_path, monkeypatch):
    B.build_host()
    csrc = tmp_path / "csrc"
    shutil.copytree(B.CSRC, csrc)
    monkeypatch.setattr(B, "CSRC", csrc)
    assert not B._stale(B.HOST_SO, "host")          # same bytes in another place: same identity
    src = csrc / "host" / "hashing_cpu.cpp"
    src.write_text(src.read_text() + "\n// edited\n")
    assert B._stale(B.HOST_SO, "host")
    with pytest.raises(RuntimeError):
        B.verify(B.HOST_SO, "host")


def test_library_without_provenance_is_stale(tmp_path):
    so = tmp_path / "libx.so"
    so.write_bytes(b"\x7fELF no hash here")
    assert B.embedded_hash(so) is None
    assert B._stale(so, "host")
    assert B._stale(tmp_path / "missing.so", "hip")
