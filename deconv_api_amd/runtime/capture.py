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

from typing import Callable, Optional

import torch


def capture(fn: Callable[[], object], graph: Optional[torch.cuda.CUDAGraph] = None, pool=None):
    """Capture ``fn()`` into ``graph`` (a new CUDAGraph when None) in thread-local mode on a fresh
    side stream (torch's capture context). Returns (graph, fn's result)."""
    g = graph if graph is not None else torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
        out = fn()
    return g, out


def drain_collective(work, device, wait=None) -> None:
    """Retire an eager (async_op=True) collective before a capture: wait for its work object
    (``wait(work)`` when given: the caller's polled wait under its failure deadlines), then
    synchronize the device so its end event has completed before the capture opens (the watchdog
    may still hold the work; with thread-local capture its poll is legal either way, and a
    completed event makes the poll trivially succeed)."""
    if work is not None:
        if wait is not None:
            wait(work)
        work.wait()
    torch.cuda.synchronize(device)
