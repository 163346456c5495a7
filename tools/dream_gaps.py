#!/usr/bin/env python
"""Where a DeepDream batch's GPU idle goes ("kernel-busy 64 % of the profiled window").

Reads a rocprofv3 kernel-trace database and reports, over the trace (or its last fraction):
  * per queue: kernels, busy time, and the gaps between consecutive kernels ON THAT QUEUE, bucketed by size;
  * the whole device: the union of kernel intervals (busy), and every interval in which NO kernel runs on
    ANY queue (true idle), bucketed by size and by the kernel that ends it (an octave_resize / copy ends
    an octave boundary; a conv ends an intra-step gap);
  * the concurrency actually recorded (sum of kernel time / union).

  python tools/dream_gaps.py gpurun_out/prof_c3/c3_results.db [--last-frac 0.5]
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import Counter, defaultdict

BUCKETS = [(0, 2), (2, 5), (5, 20), (20, 100), (100, 1000), (1000, 1e12)]  # microseconds


def bucket(us: float) -> str:
    for lo, hi in BUCKETS:
        if lo <= us < hi:
            return f"{lo}-{hi if hi < 1e12 else 'inf'} us"
    return "?"


def family(name: str) -> str:
    import re

    name = name.replace("void ", "")
    name = re.sub(r"\(.*\)$", "", name)
    return re.sub(r"<.*", "", name)[:60]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last-frac", type=float, default=1.0)
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    cols = [d[0] for d in c.execute("select * from kernels limit 1").description]
    qcol = next((k for k in ("stream_id", "queue_id", "stream", "queue") if k in cols), None)
    rows = c.execute(f"select name, start, end{', ' + qcol if qcol else ''} from kernels order by start").fetchall()
    t0, t1 = rows[0][1], max(r[2] for r in rows)
    cut = t1 - (t1 - t0) * a.last_frac
    rows = [r for r in rows if r[1] >= cut]
    span = (max(r[2] for r in rows) - rows[0][1]) / 1e3
    ksum = sum(r[2] - r[1] for r in rows) / 1e3
    print(f"window {span / 1e3:.1f} ms, {len(rows)} kernels, sum of kernel time {ksum / 1e3:.1f} ms")
    # per queue
    byq = defaultdict(list)
    for r in rows:
        byq[r[3] if qcol else 0].append(r)
    for q, rs in sorted(byq.items()):
        gaps = Counter()
        gsum = Counter()
        for p, n in zip(rs, rs[1:]):
            g = max(0.0, (n[1] - p[2]) / 1e3)
            gaps[bucket(g)] += 1
            gsum[bucket(g)] += g
        busy = sum(r[2] - r[1] for r in rs) / 1e3
        print(f"queue {q}: {len(rs)} kernels, busy {busy / 1e3:.1f} ms; gaps between its kernels:")
        for lo, hi in BUCKETS:
            k = f"{lo}-{hi if hi < 1e12 else 'inf'} us"
            if gaps[k]:
                print(f"    {k:>14}: {gaps[k]:>7} gaps, {gsum[k] / 1e3:8.2f} ms")
    # device-wide idle: intervals with no kernel in flight on any queue
    ev = sorted((r[1], r[2], r[0]) for r in rows)
    union = 0.0
    idle = Counter()
    idle_sum = Counter()
    idle_by_next = Counter()
    cs, ce = ev[0][0], ev[0][1]
    for s, e, name in ev[1:]:
        if s > ce:
            union += ce - cs
            g = (s - ce) / 1e3
            idle[bucket(g)] += 1
            idle_sum[bucket(g)] += g
            idle_by_next[family(name)] += g
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union = (union + ce - cs) / 1e3
    print(f"device: busy (union) {union / 1e3:.1f} ms = {100 * union / span:.0f} % of the window; "
          f"recorded concurrency {ksum / max(union, 1e-9):.2f}x")
    print("device idle (no kernel on any queue), by size:")
    for lo, hi in BUCKETS:
        k = f"{lo}-{hi if hi < 1e12 else 'inf'} us"
        if idle[k]:
            print(f"    {k:>14}: {idle[k]:>7} intervals, {idle_sum[k] / 1e3:8.2f} ms")
    print("device idle by the kernel family that ends it (top 12):")
    for k, v in idle_by_next.most_common(12):
        print(f"    {k:<60} {v / 1e3:8.2f} ms")


if __name__ == "__main__":
    main()
