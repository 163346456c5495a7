"""Where a tiled DeepDream batch's host time goes (config 5: host_enqueue_s ~0.22 of a ~0.25 s batch):
per-call host time of every hipGraph replay and of the rest of TiledDeepDream.run, after warm-up.

    python tools/dream_host_probe.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.engine.deepdream import RESNET_LAYERS, DreamSettings, TiledDeepDream  # noqa: E402
from deconv_api_amd.models.resnet50 import ResNet50  # noqa: E402
from deconv_api_amd.parallel import dist as pdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--runs", type=int, default=2)
    a = ap.parse_args()
    info = pdist.init()
    dev = info.device
    ops.native.load()
    net = ResNet50(0).build(dev, torch.float16)
    dd = TiledDeepDream(net, DreamSettings(layers=dict(RESNET_LAYERS)), tile=a.tile, info=info)
    g = torch.Generator(device=dev).manual_seed(7)
    img = torch.randint(0, 256, (a.batch, a.size, a.size, 3), dtype=torch.uint8, device=dev, generator=g)
    from deconv_api_amd.engine.deepdream import inception_preprocess

    x = inception_preprocess(img)
    dd.run(x)
    torch.cuda.synchronize()
    calls = []
    orig = torch.cuda.CUDAGraph.replay

    def timed(self):
        t0 = time.perf_counter()
        orig(self)
        calls.append(time.perf_counter() - t0)

    torch.cuda.CUDAGraph.replay = timed
    for r in range(a.runs):
        calls.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dd.run(x)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        print(json.dumps({"run": r, "host_s": round(t_host, 4), "wall_s": round(t_all, 4),
                          "replays": len(calls), "replay_host_s": [round(c, 4) for c in calls],
                          "other_host_s": round(t_host - sum(calls), 4)}), flush=True)
    torch.cuda.CUDAGraph.replay = orig
    # GPU-only time of the octave graphs: replay each captured octave graph alone, host waits after
    states = list(dd._tgraphs.values())
    for st in states:
        gph = getattr(st, "graph", None)
        if gph is None:
            continue
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gph.replay()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        print(json.dumps({"octave_state": list(st.x.shape), "replay_host_s": round(th, 4),
                          "replay_wall_s": round(time.perf_counter() - t0, 4)}), flush=True)


if __name__ == "__main__":
    main()
