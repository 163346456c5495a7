"""Long-lived per-device copy streams (bench.py's copy-back of each step's mosaics).

Removed after measuring (round 2): CU-masked copy streams (``hipExtStreamCreateWithCUMask``) kept
the D2H blit off most CUs, but every one-wave kernel then waited for its workgroups on the masked
CUs (config 2: 6.1k vs 6.8k img/s, profiles/bench_c2_blit_wg_ab_r2.txt); side-stream branch
execution for InceptionV3 blocks (no gain inside a graph). What bench.py does instead is WHEN it
issues the copy: behind the first MFMA-bound layers of the next step (bench.py:COPY_AT).
"""
from __future__ import annotations

import threading
from typing import Dict

import torch

_lock = threading.Lock()
_copy_streams: Dict[int, torch.cuda.Stream] = {}


def copy_stream(device: torch.device) -> torch.cuda.Stream:
    """The device's long-lived device -> host copy stream (created once)."""
    idx = torch.device(device).index or 0
    with _lock:
        s = _copy_streams.get(idx)
        if s is None:
            s = _copy_streams[idx] = torch.cuda.Stream(device=idx)
        return s
