#!/usr/bin/env python
"""Summarize ``hipcc -Rpass-analysis=kernel-resource-usage`` remarks (VGPRs, AGPRs, spills, occupancy,
LDS) per demangled kernel, optionally filtered by a substring of the demangled name.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -c deconv_api_amd/csrc/conv_dma_bf16_fwd.hip \\
      -o /tmp/x.o -Rpass-analysis=kernel-resource-usage 2> /tmp/ru.txt
  python tools/resource_usage.py /tmp/ru.txt --filter conv_dma_kw3
"""
import argparse
import re
import subprocess

KEYS = ("VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
        "LDS Size [bytes/block]")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("remarks")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    recs, cur = [], None
    for line in open(a.remarks):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            recs.append(cur)
            continue
        for k in KEYS:
            m = re.search(r"remark:\s+" + re.escape(k) + r": (\d+)", line)
            if m and cur is not None:
                cur[k] = int(m.group(1))
    dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in recs), capture_output=True,
                         text=True).stdout.splitlines()
    for r, d in zip(recs, dem):
        if a.filter in d:
            print(d.split("(")[0], {k: v for k, v in r.items() if k != "name"})


if __name__ == "__main__":
    main()
