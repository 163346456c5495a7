#!/usr/bin/env python
"""Per-octave wall time of the graphed DeepDream step (config 3 by default): for every octave shape,
replay each sub-batch's whole-octave hipGraph on its own stream (as DeepDream.run does) and time
the octave alone. Tells which octaves are launch-latency bound (small) vs MFMA/HBM bound (large).

  python tools/dream_octave_times.py --model inception_v3 --batch 64 --size 299 [--split 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.engine import deepdream as ddm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=299)
    ap.add_argument("--split", type=int, default=ddm.SPLIT)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops.native.load()
    if a.model == "inception_v3":
        from deconv_api_amd.models.inception_v3 import InceptionV3
        net = InceptionV3(0).build(dev, torch.bfloat16)
        s = ddm.DreamSettings()
    else:
        from deconv_api_amd.models.resnet50 import ResNet50
        net = ResNet50(0).build(dev, torch.float16)
        s = ddm.DreamSettings(layers=dict(ddm.RESNET_LAYERS))
    dd = ddm.DeepDream(net, s)
    dd.split = a.split
    x = torch.rand(a.batch, a.size, a.size, 3, device=dev) * 2 - 1
    dd.run(x)  # capture every octave graph of every sub-batch
    torch.cuda.synchronize()
    n = a.split
    streams = [torch.cuda.Stream(dev) for _ in range(n)]
    rows = []
    for hw in dd.octave_shapes(a.size, a.size):
        sts = []
        for i in range(n):
            key = (a.batch // n, tuple(hw), s.iterations if ddm.OCTAVE_GRAPH else 1, i)
            sts.append(dd._graphs[key])
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for st, sm in zip(sts, streams):
                with torch.cuda.stream(sm):
                    for _ in range(s.iterations // st.steps):
                        st.graph.replay()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        rows.append({"octave": list(hw), "ms": round(best * 1e3, 2), "ms_per_step": round(best * 1e3 / s.iterations, 3)})
        print(json.dumps(rows[-1]), flush=True)
    tot = sum(r["ms"] for r in rows)
    print(json.dumps({"total_ms": round(tot, 2), "img_per_s_octaves_only": round(a.batch / tot * 1e3, 1),
                      "split": n}), flush=True)


if __name__ == "__main__":
    main()
