#!/usr/bin/env python
"""Per-shape conv kernel benchmark: time, TFLOP/s and effective HBM GB/s (minimum bytes: read x,
weights, optional mask/residual/emask once, write the output once) for the shapes of a model.

  python tools/bench_conv.py --set resnet512 [--dtype fp16] [--impl auto]
  python tools/bench_conv.py --shape 32,128,128,64,256,1,1 --mask --res

A shape is N,H,W,C,OC,k,stride (pad = k//2).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops
from deconv_api_amd.ops.conv import ConvWeights, set_policy

SETS = {
    # ResNet-50 trunk at 512x512 tiles, 32 tiles per batch (config 5, 1 GPU): fwd and dgrad shapes
    "resnet512": [
        (32, 128, 128, 64, 64, 1, 1), (32, 128, 128, 64, 64, 3, 1), (32, 128, 128, 64, 256, 1, 1),
        (32, 128, 128, 256, 64, 1, 1), (32, 64, 64, 128, 128, 3, 1), (32, 64, 64, 128, 512, 1, 1),
        (32, 64, 64, 512, 128, 1, 1), (32, 32, 32, 256, 256, 3, 1), (32, 32, 32, 256, 1024, 1, 1),
        (32, 32, 32, 1024, 256, 1, 1), (32, 256, 256, 64, 147, 1, 1),
    ],
    # VGG16 block5_conv3 deconvnet at B=256 (flagship bench)
    "vgg256": [
        (256, 224, 224, 64, 64, 3, 1), (256, 112, 112, 128, 128, 3, 1), (256, 56, 56, 256, 256, 3, 1),
        (256, 28, 28, 512, 512, 3, 1), (256, 14, 14, 512, 512, 3, 1),
    ],
}


def bench_one(shape, dt, mask, res, iters, warm):
    N, H, W, C, OC, k, s = shape
    dev = "cuda"
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, W, C, generator=g).to(dt).to(dev)
    cw = ConvWeights(torch.randn(OC, C, k, k, generator=g) / (C * k * k) ** 0.5, torch.zeros(OC), "fwd")
    cwd = cw.to_device(dev, dt)
    OH, OW = (H + 2 * (k // 2) - k) // s + 1, (W + 2 * (k // 2) - k) // s + 1
    m = x.clone() if mask else None
    r = torch.randn(N, OH, OW, OC, generator=g).to(dt).to(dev) if res else None
    out = torch.empty(N, OH, OW, OC, dtype=dt, device=dev)
    kw = dict(stride=s, relu=True, mask=m, out=out, res=r, emask=(r if res else None))

    def run():
        ops.conv2d(x, cwd, **kw)

    for _ in range(warm):
        run()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(iters):
        run()
    t1.record()
    torch.cuda.synchronize()
    us = t0.elapsed_time(t1) * 1e3 / iters
    flops = 2.0 * N * OH * OW * OC * C * k * k
    el = 2
    byts = el * (N * H * W * C * (2 if mask else 1) + OC * C * k * k + N * OH * OW * OC * (3 if res else 1))
    return {"shape": list(shape), "mask": mask, "res": res, "us": round(us, 1),
            "tflops": round(flops / us / 1e6, 1), "gbps": round(byts / us / 1e3, 1)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default=None, choices=sorted(SETS))
    ap.add_argument("--shape", action="append", default=[])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--mask", action="store_true")
    ap.add_argument("--res", action="store_true")
    ap.add_argument("--impl", default="auto")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args(argv)
    ops.native.load()
    set_policy(impl=a.impl)
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    shapes = list(SETS[a.set]) if a.set else []
    shapes += [tuple(int(v) for v in s.split(",")) for s in a.shape]
    for sh in shapes:
        variants = [(a.mask, a.res)] if (a.mask or a.res or not a.set) else [(False, False), (True, False)]
        if a.set == "resnet512" and sh[5] == 1 and sh[6] == 1 and not (a.mask or a.res):
            variants.append((True, True))
        for mk, rs in variants:
            print(json.dumps(bench_one(sh, dt, mk, rs, a.iters, a.warmup)), flush=True)


if __name__ == "__main__":
    main()
