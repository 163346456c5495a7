#!/usr/bin/env python
"""Time the fused VGG16 stem (ops.stem_pool: block1_conv1 -> block1_conv2 -> pool in one launch) against
the two launches it replaces, at the config-2 shape (256 x 224^2), and check they agree bit for bit.

  python tools/stem_ab.py [--batch 256] [--reps 20]
"""
import argparse
import json
import os

os.environ.setdefault("DV_ABLATIONS", "1")  # this tool A/Bs switches of deconv_api_amd/knobs.py ABLATION
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.models.vgg16 import VGG16  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    rt = VGG16.random(0, include_top=False).build("cuda")
    c1, c2 = rt.convs["block1_conv1"].fwd, rt.convs["block1_conv2"].fwd
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.zeros(a.batch, 224, 224, 8, device="cuda")
    x[..., :3] = torch.randn(a.batch, 224, 224, 3, device="cuda", generator=g) * 60
    x = x.to(torch.bfloat16).contiguous()

    def fused():
        return ops.stem_pool(x, c1, c2)

    def unfused():
        return ops.conv2d(ops.conv2d(x, c1, relu=True), c2, relu=True, epilogue="pool")

    f, u = fused(), unfused()
    same = bool(torch.equal(f[0], u[0]) and torch.equal(f[1], u[1]))
    res = {"same": same}
    for name, fn in (("fused", fused), ("unfused", unfused)) * 2:
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(name + "_ms", []).append(round(e0.elapsed_time(e1) / a.reps, 4))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
