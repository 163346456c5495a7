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


def load(build_if_missing: bool = False):
    """Import ``deconv_api_amd._C``; optionally build it in-tree first."""
    global _mod, _err
    with _lock:
        if _mod is not None:
            return _mod
        try:
            _mod = importlib.import_module("deconv_api_amd._C")
        except ImportError as e:  # pragma: no cover - depends on build state
            if build_if_missing or os.environ.get("DV_AUTOBUILD", "0") == "1":
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
