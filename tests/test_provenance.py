"""Build provenance (_build.py / ops/native.py): the binary carries the hash of the sources it was
built from, and the loader refuses one whose hash does not match the tree."""
import shutil

import pytest

from deconv_api_amd import _build
from deconv_api_amd.ops import native


def test_source_hash_is_content_and_flag_sensitive(tmp_path, monkeypatch):
    h0 = _build.source_hash()
    assert len(h0) == 64 and h0 == _build.source_hash()
    assert _build.source_hash(debug=True) != h0  # flags are part of it
    csrc = tmp_path / "csrc"
    shutil.copytree(_build.CSRC, csrc)
    monkeypatch.setattr(_build, "CSRC", csrc)
    assert _build.source_hash() == h0  # same bytes elsewhere: same hash (no paths, no mtimes)
    f = csrc / "misc.hip"
    f.write_bytes(f.read_bytes() + b"\n// touched\n")
    assert _build.source_hash() != h0


def test_loader_refuses_a_binary_built_from_other_sources(tmp_path, monkeypatch):
    so = tmp_path / "_C.so"
    so.write_bytes(b"\x7fELF...DV_SOURCE_HASH:" + b"ab" * 32 + b"\0...")
    monkeypatch.setattr(_build, "TARGET", so)
    monkeypatch.delenv("DV_SKIP_PROVENANCE", raising=False)
    assert _build.embedded_hash(so) == "ab" * 32
    with pytest.raises(native.StaleBinaryError, match="built from other sources"):
        native.check_provenance()
    so.write_bytes(b"DV_SOURCE_HASH:" + _build.source_hash().encode())
    assert native.check_provenance() == _build.source_hash()


def test_touching_a_kernel_source_makes_the_built_binary_stale(tmp_path, monkeypatch):
    if not _build.TARGET.exists():
        pytest.skip("extension not built")
    if _build.embedded_hash(_build.TARGET) != _build.source_hash():
        pytest.skip("in-tree binary predates the current sources (rebuild)")
    csrc = tmp_path / "csrc"
    shutil.copytree(_build.CSRC, csrc)
    monkeypatch.setattr(_build, "CSRC", csrc)
    monkeypatch.delenv("DV_SKIP_PROVENANCE", raising=False)
    assert native.check_provenance() == _build.embedded_hash(_build.TARGET)
    (csrc / "conv_pw.hip").write_bytes((csrc / "conv_pw.hip").read_bytes() + b"\n")
    with pytest.raises(native.StaleBinaryError):
        native.check_provenance()
