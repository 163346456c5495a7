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
capturing thread's own unsafe calls are refused). Captured collectives run on their own process
group, connected eagerly and never used eagerly (engine/deepdream.py ``_capture_group``), so the
watchdog never tracks a work whose event lives on a stream a capture pulled in; no sleep, no drain.
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
