#!/usr/bin/env python
"""Summarize a rocprofv3 kernel-trace database (``rocprofv3 --kernel-trace -d DIR -o NAME``
writes DIR/.../NAME_results.db, an SQLite "rocpd" file) into a per-kernel table, optionally
restricted to a time window (e.g. only the timed run after the warmup).

  python tools/kstats.py gpurun_out/prof_c5/c5_results.db [--top 30] [--last-frac 0.5]
"""
from __future__ import annotations

import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*\)$", "", name)
    return name[:110]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--last-frac", type=float, default=1.0,
                    help="only dispatches in the last fraction of the trace's GPU time span")
    ap.add_argument("--gaps", action="store_true", help="also report idle gaps between dispatches")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels").fetchall()
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    cut = t1 - (t1 - t0) * a.last_frac
    agg = defaultdict(lambda: [0, 0.0])
    busy = 0.0
    lo, hi = None, None
    for name, s, e, gx, wx in rows:
        if s < cut:
            continue
        k = agg[short(name)]
        k[0] += 1
        k[1] += (e - s) / 1e3
        busy += (e - s) / 1e3
        lo = s if lo is None else min(lo, s)
        hi = e if hi is None else max(hi, e)
    span = (hi - lo) / 1e3 if lo is not None else 0.0
    # union of dispatch intervals (busy above double-counts kernels that run concurrently)
    ev = sorted((s, e) for _, s, e, _, _ in rows if s >= cut)
    union = 0.0
    cs, ce = (ev[0] if ev else (0, 0))
    for s, e in ev[1:]:
        if s > ce:
            union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union = (union + ce - cs) / 1e3
    print(f"window: {span / 1e3:.1f} ms wall, {busy / 1e3:.1f} ms kernel-busy ({100 * busy / max(span, 1e-9):.0f}%), "
          f"{union / 1e3:.1f} ms with >= 1 kernel in flight (concurrency {busy / max(union, 1e-9):.2f}x)")
    print(f"{'total_ms':>9} {'%':>5} {'calls':>7} {'avg_us':>8}  kernel")
    for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{us / 1e3:9.2f} {100 * us / busy:5.1f} {n:7d} {us / n:8.1f}  {name}")
    if a.gaps:
        gaps(rows, cut, a.top)


def gaps(rows, cut, top):
    """Idle time between consecutive dispatches (GPU timeline, single queue assumed): a histogram
    and the kernels that the largest idle totals FOLLOW (host syncs / launch-bound stretches)."""
    ev = sorted((s, e, short(n)) for n, s, e, _, _ in rows if s >= cut)
    hist = defaultdict(lambda: [0, 0.0])
    after = defaultdict(lambda: [0, 0.0])
    edges = (2, 5, 10, 20, 50, 100, 1000, float("inf"))
    end = ev[0][1] if ev else 0
    prev = ev[0][2] if ev else ""
    for s, e, n in ev[1:]:
        g = (s - end) / 1e3  # us
        if g > 0:
            b = next(x for x in edges if g <= x)
            hist[b][0] += 1
            hist[b][1] += g
            after[prev][0] += 1
            after[prev][1] += g
        if e >= end:
            end, prev = e, n
    print("idle gaps (us bucket <=: count, total ms)")
    for b in edges:
        if b in hist:
            print(f"  <= {b:>6}: {hist[b][0]:7d} {hist[b][1] / 1e3:9.2f}")
    print(f"{'idle_ms':>9} {'gaps':>7} {'avg_us':>8}  preceding kernel")
    for name, (n, us) in sorted(after.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{us / 1e3:9.2f} {n:7d} {us / n:8.1f}  {name}")


if __name__ == "__main__":
    main()
