"""roctx ranges around engine stages (visible with ``rocprofv3 --marker-trace``) plus a light
host timer. Loads ``libroctx64.so`` (shipped with torch-ROCm and ROCm) via ctypes; becomes a no-op
when it is absent (CPU-only machines)."""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Dict, Optional

_lib: Optional[ctypes.CDLL] = None
_tried = False
ENABLED = os.environ.get("DV_ROCTX", "1") != "0"


def _load():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    cands = ["libroctx64.so", "/opt/rocm/lib/libroctx64.so"]
    try:
        import torch

        cands.insert(0, os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"))
    except Exception:  # noqa: BLE001
        pass
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            break
        except OSError:
            continue
    return _lib


def push(name: str) -> None:
    if ENABLED and _load() is not None:
        _lib.roctxRangePushA(name.encode())


def pop() -> None:
    if ENABLED and _lib is not None:
        _lib.roctxRangePop()


def mark(name: str) -> None:
    if ENABLED and _load() is not None:
        _lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range_(name: str, timings: Optional[Dict[str, float]] = None):
    """roctx range + optional host wall-time accumulation into ``timings[name]`` (seconds)."""
    push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        pop()
        if timings is not None:
            timings[name] = timings.get(name, 0.0) + time.perf_counter() - t0


def available() -> bool:
    return _load() is not None
