#!/usr/bin/env python
"""Compare per-kernel VGPR spills / scratch between two sets of ``-Rpass-analysis=kernel-resource-usage``
remark files (e.g. the current tree against a git worktree of the previous commit), so a change to a shared
device helper (common.h) that pushes some instantiation over its register budget is caught before a GPU run.

  python tools/spill_diff.py /tmp/o_{unit}.txt /tmp/n_{unit}.txt conv_dma conv_pw ...
"""
import re
import sys


def load(path):
    d, cur = {}, None
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            d[cur] = {"sp": 0, "sc": 0, "vgpr": 0}
            continue
        for key, pat in (("sp", r"VGPRs Spill: (\d+)"), ("sc", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("vgpr", r"remark:\s+VGPRs: (\d+)")):
            m = re.search(r"remark:\s+" + pat if key != "vgpr" else pat, line)
            if m and cur:
                d[cur][key] = int(m.group(1))
    return d


def main():
    old_pat, new_pat, units = sys.argv[1], sys.argv[2], sys.argv[3:]
    bad = 0
    for u in units:
        o, n = load(old_pat.format(unit=u)), load(new_pat.format(unit=u))
        worse = [k for k in n if k in o and (n[k]["sp"] > o[k]["sp"] or n[k]["sc"] > o[k]["sc"])]
        better = [k for k in n if k in o and (n[k]["sp"] < o[k]["sp"] or n[k]["sc"] < o[k]["sc"])]
        print(f"{u}: {len(n)} kernels, worse {len(worse)}, better {len(better)}")
        for k in worse[:5]:
            print(f"  worse  {k[:100]} {o[k]} -> {n[k]}")
        for k in better[:5]:
            print(f"  better {k[:100]} {o[k]} -> {n[k]}")
        bad += len(worse)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
