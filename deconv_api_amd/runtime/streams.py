"""Long-lived per-device copy streams (bench.py's copy-back of each step's mosaics), and streams that
do not share a hardware queue with the compute stream.

HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues per process (4 by default) round-robin in
creation order, and torch hands out its pool streams round-robin too, so two "independent" streams can
land on one queue and execute strictly in order: the serving input stream then waits behind the
previous batch's whole engine (found by tests/test_sharded_streams_gpu.py, which failed only when an
earlier test module had created streams). ``independent_stream`` probes candidates at init.

Removed after measuring (round 2): CU-masked copy streams (``hipExtStreamCreateWithCUMask``) kept
the D2H blit off most CUs, but every one-wave kernel then waited for its workgroups on the masked
CUs (config 2: 6.1k vs 6.8k img/s, profiles/bench_c2_blit_wg_ab_r2.txt); side-stream branch
execution for InceptionV3 blocks (no gain inside a graph). What bench.py does instead is WHEN it
issues the copy: behind the first MFMA-bound layers of the next step (bench.py:COPY_AT).
"""
from __future__ import annotations

import threading
import time
from typing import Dict, Sequence

import torch

from .. import knobs

_lock = threading.Lock()
_copy_streams: Dict[int, torch.cuda.Stream] = {}


def copy_stream(device: torch.device) -> torch.cuda.Stream:
    """The device's long-lived device -> host copy stream (created once, on a hardware queue apart
    from the calling thread's current stream)."""
    idx = torch.device(device).index or 0
    with _lock:
        s = _copy_streams.get(idx)
        if s is None:
            s = _copy_streams[idx] = independent_stream(torch.device("cuda", idx),
                                                        [torch.cuda.current_stream(idx)])
        return s


def _behind(s: torch.cuda.Stream, a: torch.cuda.Stream, spin_cycles: int, timeout_s: float = 2.0) -> bool:
    """True when a marker on ``s`` completes only after a spin kernel on ``a`` (one hardware queue)."""
    with torch.cuda.stream(a):
        torch.cuda._sleep(spin_cycles)
        end = torch.cuda.Event()
        end.record(a)
    mark = torch.cuda.Event()
    mark.record(s)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < timeout_s:
        m = mark.query()  # (marker first: "marker done, spin not" is then a real instant)
        e = end.query()
        if m and not e:
            return False
        if e:
            return True
    return True


def independent_stream(device, avoid: Sequence[torch.cuda.Stream], tries: int = 8,
                       spin_cycles: int = 4_000_000) -> torch.cuda.Stream:
    """A new stream whose work does not queue behind ``avoid``'s on the hardware (probed: a ~2 ms spin
    on each avoided stream must still run when a marker on the candidate completes). Call at init,
    outside graph capture (it synchronizes the device). Falls back to a plain new stream when every
    candidate shares a queue (fewer hardware queues than streams in use)."""
    dev = torch.device(device)
    if knobs.ablation("DV_NO_STREAM_PROBE") == "1":  # A/B: plain pool streams
        return torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    first = None
    for _ in range(max(1, tries)):
        s = torch.cuda.Stream(dev)
        first = first or s
        if not any(_behind(s, a, spin_cycles) for a in avoid):
            torch.cuda.synchronize(dev)
            return s
    torch.cuda.synchronize(dev)
    return first

