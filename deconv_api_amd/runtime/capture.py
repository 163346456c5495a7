"""hipGraph capture that other host threads cannot break.

torch's default capture mode is "global": while ANY thread has a capture open, a
``hipEventQuery`` / ``hipEventSynchronize`` / ``hipStreamSynchronize`` from ANY other thread is
refused and invalidates the capture. Two such threads always exist in this service:

* the RCCL (ProcessGroupNCCL) watchdog, which polls the end events of every collective it still
  tracks — round 3's intermittent SIGABRT of the captured tiled-DeepDream octave was the watchdog
  polling the eager warm-up all-gather while the octave capture was open (the failure rate
  depended on whether its poll fell inside the capture window);
* the deconv service's completion thread, which synchronizes earlier batches' events
  (runtime/staging.py) while a ``/deepdream`` request captures a new octave shape.

Every capture in the package therefore goes through ``capture`` (mode "thread_local": only the
capturing thread's own unsafe calls are refused), and ``drain_collective`` retires an eager
collective (work.wait + device sync) before a capture that follows it.
"""
from __future__ import annotations

import time
from typing import Callable, Optional

import torch


def capture(fn: Callable[[], object], graph: Optional[torch.cuda.CUDAGraph] = None, pool=None):
    """Capture ``fn()`` into ``graph`` (a new CUDAGraph when None) in thread-local mode on a fresh
    side stream (torch's capture context). Returns (graph, fn's result)."""
    g = graph if graph is not None else torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
        out = fn()
    return g, out


def drain_collective(work, device, wait=None, settle: bool = True) -> None:
    """Retire an eager (async_op=True) collective before a capture: wait for its work object
    (``wait(work)`` when given: the caller's polled wait under its failure deadlines), then
    synchronize the device so its end event has completed before the capture opens, and (``settle``,
    once after the last of several) give the process group's watchdog time to drop it (below)."""
    if work is not None:
        if wait is not None:
            wait(work)
        work.wait()
    torch.cuda.synchronize(device)
    if work is not None and settle:
        # ... and let ProcessGroupNCCL's watchdog (which wakes every 100 ms) drop the completed work from its
        # list first: HIP refuses hipEventQuery on an event of a stream that is capturing NOW, even one
        # recorded before the capture, so a watchdog poll of this work's end event once the captured
        # collectives have pulled the NCCL stream into the capture aborts the process (hipErrorCapturedEvent,
        # intermittently in tests/test_deepdream.py::test_gpu_tiled_collective_octave_captured)
        time.sleep(0.3)
