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
