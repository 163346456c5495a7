#!/usr/bin/env python
"""Per-kernel sums of rocprofv3 PMC counters from *counter_collection.csv files (one or more
passes) or rocpd SQLite databases (*.db: rocprofv3's default output in ROCm 7), with the derived
stall fractions used in docs/KERNELS.md:
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMDs... reported raw)
  wait_any / wave_cycles, wait_inst_any / wave_cycles, lds_bank_conflict / lds_idx_active.
  python tools/pmc_summary.py DIR [--top 12]"""
import argparse
import collections
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = re.sub(r"\(.*\)$", "", row.get("Kernel_Name", "?").replace("void ", ""))[:90]
            tot[name][row["Counter_Name"]] += float(row["Counter_Value"])
            if "End_Timestamp" in row and "Start_Timestamp" in row:
                dur[name] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
    import sqlite3

    for f in glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True) + ([a.dir] if a.dir.endswith(".db") else []):
        seen = set()
        for kname, cname, val, disp, d in sqlite3.connect(f).execute(
                "select kernel_name, counter_name, value, dispatch_id, duration from counters_collection"):
            name = re.sub(r"\(.*\)$", "", kname.replace("void ", "").replace("(anonymous namespace)::", ""))[:90]
            tot[name][cname] += float(val)
            if (name, disp) not in seen:
                seen.add((name, disp))
                dur[name] += d / 1e3
    names = sorted(tot, key=lambda n: -dur.get(n, 0.0))
    for n in names[: a.top]:
        c = tot[n]
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        out = {k: f"{v:.3g}" for k, v in sorted(c.items())}
        der = []
        if "SQ_WAIT_ANY" in c:
            der.append(f"wait_any {c['SQ_WAIT_ANY'] / wc:.2f}")
        if "SQ_WAIT_INST_ANY" in c:
            der.append(f"wait_inst {c['SQ_WAIT_INST_ANY'] / wc:.2f}")
        if "SQ_ACTIVE_INST_ANY" in c:
            der.append(f"active {c['SQ_ACTIVE_INST_ANY'] / wc:.2f}")
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            der.append(f"lds_conflict/active {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("SQ_BUSY_CYCLES"):
            der.append(f"mfma_busy/busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / c['SQ_BUSY_CYCLES']:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
            # MFMA pipe busy per SIMD over the kernel's active GPU cycles (GRBM_GUI_ACTIVE sums the
            # 8 XCDs; 32 CUs x 4 SIMDs per XCD)
            der.append(f"mfma_util {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['GRBM_GUI_ACTIVE'] / 8 * 1024):.2f}")
        if "FETCH_SIZE" in c and dur.get(n):
            # FETCH_SIZE (KB) reads 1/2 of wide coalesced streaming bytes on gfx950 (MI355X_MICROARCH.md)
            der.append(f"fetch {2 * c['FETCH_SIZE'] / 1e6:.2f} GB ({2 * c['FETCH_SIZE'] * 1e-3 / dur[n]:.2f} TB/s x2-corrected)")
        if dur.get(n):
            der.append(f"dur {dur[n] / 1e3:.2f} ms")
        print(f"== {n}\n   {'; '.join(der)}\n   {out}")


if __name__ == "__main__":
    main()
