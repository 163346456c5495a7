"""Loader for the in-tree gfx950 extension (``deconv_api_amd/_C*.so``).

GPU tensors always go through the HIP kernels; if the extension is missing on a machine with
a GPU the ops raise instead of silently falling back to PyTorch (the round-end driver checks
which native ``.so`` files the GPU tests actually loaded).
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


class StaleBinaryError(RuntimeError):
    pass


def check_provenance() -> str:
    """The tree's source hash if the built ``_C`` carries the same one; raises StaleBinaryError
    when it was built from other sources / flags (``_build.py``: provenance). A missing binary
    passes here (the import reports it). ``DV_SKIP_PROVENANCE=1`` skips the check (tools that
    load a scratch build on purpose)."""
    from .. import _build

    want = _build.source_hash()
    if os.environ.get("DV_SKIP_PROVENANCE") == "1" or not _build.TARGET.exists():
        return want
    got = _build.embedded_hash(_build.TARGET)
    if got != want:
        raise StaleBinaryError(
            f"deconv_api_amd/_C was built from other sources (embedded hash {got}, tree {want}); rebuild with "
            "`python -m deconv_api_amd._build` (or set DV_AUTOBUILD=1)")
    return want


def load(build_if_missing: bool = False):
    """Import ``deconv_api_amd._C`` after checking that it was built from this tree's sources;
    optionally (re)build it in-tree first."""
    global _mod, _err
    with _lock:
        if _mod is not None:
            return _mod
        autobuild = build_if_missing or os.environ.get("DV_AUTOBUILD", "0") == "1"
        try:
            check_provenance()
        except StaleBinaryError:
            if not autobuild:
                raise
            from .. import _build

            _build.build()
        try:
            _mod = importlib.import_module("deconv_api_amd._C")
        except ImportError as e:  # pragma: no cover - depends on build state
            if autobuild:
                from .. import _build

                _build.build()
                _mod = importlib.import_module("deconv_api_amd._C")
            else:
                _err = e
                raise RuntimeError(
                    "deconv_api_amd native extension (_C) is not built; run "
                    "`python -m deconv_api_amd._build` (hipcc --offload-arch=gfx950)"
                ) from e
        return _mod


def available() -> bool:
    try:
        load()
        return True
    except RuntimeError:
        return False


def lib():
    """The extension module; raises loudly if it is not importable."""
    return _mod if _mod is not None else load()
