#!/usr/bin/env python
"""Print the ordered kernel sequence of ONE iteration from a rocprofv3 kernel-trace database:
the dispatches between the Nth and (N+1)th occurrence of a marker kernel (e.g. DeepDream's
``dream_update_kernel``, one per gradient step), per queue/stream when the trace has one, with
each kernel's duration, grid, and the idle gap since the previous dispatch on the same queue.
A summary counts launches by kernel family — the launch-count budget of a latency-bound step.

  python tools/kseq.py gpurun_out/prof_c3/x_results.db --marker dream_update --nth 40
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import Counter, defaultdict

from kstats import short


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="dream_update")
    ap.add_argument("--nth", type=int, default=-2, help="which marker occurrence starts the window (per queue)")
    ap.add_argument("--quiet", action="store_true", help="summary only")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    cols = [d[0] for d in c.execute("select * from kernels limit 1").description]
    qcol = next((k for k in ("stream_id", "queue_id", "stream", "queue") if k in cols), None)
    sel = f"select name, start, end, grid_x, workgroup_x{', ' + qcol if qcol else ''} from kernels order by start"
    rows = c.execute(sel).fetchall()
    byq = defaultdict(list)
    for r in rows:
        byq[r[5] if qcol else 0].append(r)
    for q, rs in byq.items():
        marks = [i for i, r in enumerate(rs) if a.marker in r[0]]
        if len(marks) < 2:
            continue
        i0 = marks[max(-len(marks), min(a.nth, len(marks) - 1))]
        nxt = [m for m in marks if m > i0]
        if not nxt:
            i0, nxt = marks[-2], marks[-1:]
        win = rs[i0 + 1: nxt[0] + 1]
        span = (win[-1][2] - rs[i0][2]) / 1e3
        busy = sum(r[2] - r[1] for r in win) / 1e3
        print(f"== queue {q}: {len(win)} launches, {span:.1f} us span, {busy:.1f} us kernel-busy")
        fam = Counter()
        gap_tot = 0.0
        prev_end = rs[i0][2]
        for r in win:
            g = (r[1] - prev_end) / 1e3
            gap_tot += max(g, 0.0)
            prev_end = max(prev_end, r[2])
            nm = short(r[0])
            fam[nm.split("<")[0]] += 1
            if not a.quiet:
                print(f"  {(r[2] - r[1]) / 1e3:8.1f} us  gap {g:7.1f}  grid {r[3] // max(r[4], 1):6d}x{r[4]:<4d} {nm[:90]}")
        print(f"  idle gaps total {gap_tot:.1f} us; launches by family:")
        for k, n in fam.most_common():
            print(f"    {n:4d}  {k}")


if __name__ == "__main__":
    main()
