"""Per-device HIP stream pool and fork/join execution of independent branches.

A CNN block whose branches are independent (InceptionV3 mixed blocks) launches each branch on its
own stream: small-spatial convs leave most of the 256 CUs idle when run one after another, and
branches on separate streams run concurrently. Inside ``torch.cuda.graph`` capture the fork/join
becomes parallel graph nodes; autograd runs each node's backward on the stream its forward used,
so the backward branches overlap too.
"""
from __future__ import annotations

import threading
from typing import Callable, Dict, List, Sequence

import torch

_lock = threading.Lock()
_pools: Dict[int, List[torch.cuda.Stream]] = {}


def side_streams(device: torch.device, n: int) -> List[torch.cuda.Stream]:
    """``n`` long-lived side streams of ``device`` (created once, reused by every call)."""
    idx = torch.device(device).index or 0
    with _lock:
        pool = _pools.setdefault(idx, [])
        while len(pool) < n:
            pool.append(torch.cuda.Stream(device=idx))
        return pool[:n]


def run_parallel(fns: Sequence[Callable[[torch.Tensor], torch.Tensor]], x: torch.Tensor) -> List[torch.Tensor]:
    """[fn(x) for fn in fns], fn i on side stream i, joined back into the current stream.

    Outputs are ``record_stream``-ed on the current stream so the caching allocator does not hand
    their memory to a side stream while the consumer still reads it."""
    cur = torch.cuda.current_stream(x.device)
    streams = side_streams(x.device, len(fns))
    outs = []
    for fn, s in zip(fns, streams):
        s.wait_stream(cur)
        x.record_stream(s)  # x may be freed on `cur` while a branch still reads it
        with torch.cuda.stream(s):
            outs.append(fn(x))
    for s, o in zip(streams, outs):
        cur.wait_stream(s)
        o.record_stream(cur)
    return outs


_copy_streams: Dict[tuple, torch.cuda.Stream] = {}


def copy_stream(device: torch.device, cus: int | None = None) -> torch.cuda.Stream:
    """Long-lived stream for device -> host copies; with ``cus`` > 0 (``DV_COPY_CUS``) its
    dispatches are confined to that many CUs. Default 0: an ordinary, unmasked stream (CU masking
    was measured slower end to end, profiles/bench_c2_blit_wg_ab_r2.txt; opt-in for A/B only).

    A D2H copy into pinned memory runs as a runtime blit kernel whose waves wait on PCIe writes; on an
    unrestricted stream it fills every CU for the length of the transfer and the compute stream's next
    kernel cannot start (measured in ``bench.py``: the 38 us input kernel stretched to 2.7 ms behind the
    2.8 ms mosaic copy-back, profiles/copyback_overlap_r2.txt). On a CU-masked stream the copy keeps a
    few CUs and overlaps with compute on the rest, but the copy then takes longer than it hides."""
    import os

    idx = torch.device(device).index or 0
    n = int(os.environ.get("DV_COPY_CUS", "0")) if cus is None else int(cus)
    key = (idx, n)
    with _lock:
        s = _copy_streams.get(key)
        if s is None:
            if n > 0:
                from ..ops import native

                total = torch.cuda.get_device_properties(idx).multi_processor_count
                handle = native.lib().cu_masked_stream(idx, min(n, total))
                s = torch.cuda.ExternalStream(handle, device=torch.device("cuda", idx))
            else:
                s = torch.cuda.Stream(device=idx)
            _copy_streams[key] = s
        return s
