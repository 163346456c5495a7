#!/usr/bin/env python
"""Per-launch GPU time of small convs inside a hipGraph (the regime of DeepDream's small octaves):
for each (M, N, K) a graph of `--reps` back-to-back dependent launches is replayed and timed, so
host launch cost is excluded and the number is the kernel's own latency floor plus the
inter-kernel gap. Also times an empty elementwise kernel (torch add_) as the floor reference.

  python tools/small_conv_latency.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.ops.conv import ConvWeights  # noqa: E402


def graph_time(fn, reps=50, iters=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
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
    for _ in range(iters):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


# (tile config, split-K) pairs: 0/0 = the shipped policy; configs in csrc/conv_dma_impl.h:dma_forced
# (8: 64x64 4 waves 3 stages, 16: 64x64 8 waves, 17: 8 waves 4 stages, 12: 4 waves 6 stages,
#  7: 128x64 4 waves)
SWEEP = [(0, 0), (8, 1), (16, 1), (17, 1), (12, 1), (7, 1), (8, 4), (16, 4)]


def main():
    dev = torch.device("cuda", 0)
    ops.native.load()
    t = torch.zeros(1024, device=dev)
    print(json.dumps({"kernel": "torch add_ (1024 floats)", "us": round(graph_time(lambda: t.add_(1.0)), 2)}), flush=True)
    for (M_img, hw, C, OC, k) in [(64, 5, 64, 64, 1), (64, 5, 192, 160, 1), (64, 5, 160, 160, 3), (64, 5, 768, 192, 1),
                                 (64, 8, 288, 96, 3), (64, 17, 768, 192, 1), (64, 17, 160, 160, 3)]:
        x = torch.randn(M_img, hw, hw, C, device=dev).to(torch.bfloat16)
        cw = ConvWeights(torch.randn(OC, C, k, k) / (C * k * k) ** 0.5, torch.zeros(OC), "fwd").to_device(dev)
        out = torch.empty(M_img, hw, hw, OC, device=dev, dtype=torch.bfloat16)
        M, K = M_img * hw * hw, C * k * k
        lib = ops.native.lib()
        res = {}
        for cfg, ks in SWEEP:
            lib.dma_tune(cfg, ks)
            try:
                res[f"{cfg}/{ks}"] = round(graph_time(lambda: ops.conv2d(x, cw, relu=True, out=out)), 2)
            except RuntimeError as e:  # config not valid for this shape
                res[f"{cfg}/{ks}"] = None
            lib.dma_tune(0, 0)
        print(json.dumps({"kernel": "conv_dma", "M": M, "N": OC, "K": K, "us(cfg/ks)": res}), flush=True)


if __name__ == "__main__":
    main()
