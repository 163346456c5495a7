#!/usr/bin/env python
"""Bandwidth of large-M 1x1 convs (ResNet-50 stage-2 shapes of config 5) on the persistent
pointwise kernel vs the one-tile-per-workgroup LDS-DMA kernel, against a plain device copy of the
same bytes (the HBM ceiling this box reaches). Timed as hipGraph replays (no launch overhead).

  python tools/pw_bench.py [--m 524288]
"""
from __future__ import annotations

import argparse
import json
import os

os.environ.setdefault("DV_ABLATIONS", "1")  # this tool A/Bs switches of deconv_api_amd/knobs.py ABLATION
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.ops.conv import ConvWeights  # noqa: E402


def graph_us(fn, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=524288)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = ops.native.load()
    dt = torch.float16
    M = a.m
    side = int(M ** 0.5)
    src = torch.empty(M * 256, device=dev, dtype=dt)
    dst = torch.empty_like(src)
    us = graph_us(lambda: dst.copy_(src))
    print(json.dumps({"op": "copy 256ch", "us": round(us, 1), "TB/s": round(2 * src.numel() * 2 / us * 1e-6, 2)}),
          flush=True)
    for C, OC, mode in [(64, 256, "plain"), (64, 256, "res"), (256, 64, "plain"), (64, 256, "res_emask"),
                        (256, 64, "emask")]:
        x = torch.randn(1, side, M // side, C, device=dev).to(dt)
        cw = ConvWeights(torch.randn(OC, C, 1, 1) / C ** 0.5, torch.zeros(OC), "fwd").to_device(dev, dt)
        res = torch.randn(1, side, M // side, OC, device=dev).to(dt)
        kw = {"plain": dict(relu=True), "res": dict(relu=True, res=res), "emask": dict(relu=False, emask=res),
              "res_emask": dict(relu=True, res=res, emask=res)}[mode]
        mm = side * (M // side)
        nbytes = mm * (C + OC) * 2 + mm * OC * 2 * (("res" in mode) + ("emask" in mode))
        row = {"op": f"1x1 {C}->{OC} {mode}", "GB": round(nbytes / 1e9, 3)}
        for name, env, cfg in [("pw", None, 0), ("dma", "1", 0)]:
            if env:
                os.environ["DV_NO_PW"] = env
            lib.dma_tune(3 if OC > 64 else 5, 1) if env else None
            try:
                t = graph_us(lambda: ops.conv2d(x, cw, pad=0, **kw))
            finally:
                lib.dma_tune(0, 0)
            row[name + "_us"] = round(t, 1)
            row[name + "_TB/s"] = round(nbytes / t * 1e-6, 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
