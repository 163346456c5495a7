"""List every ATen (non-HIP-extension) op one DeepDream step dispatches on the GPU, with shapes
and the innermost framework frame that issued it, to find the at::native glue kernels in the
kstats tables. Usage (GPU box):

    python tools/aten_trace.py --model resnet50 --batch 8 --size 1024 --tile 512 --dtype fp16
    python tools/aten_trace.py --model inception_v3 --batch 64 --size 299
"""
import argparse
import os
import sys
import traceback
from collections import Counter

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd.engine.deepdream import RESNET_LAYERS, DeepDream, DreamSettings, TiledDeepDream  # noqa: E402

# metadata-only ops: no kernel
SKIP = {"aten.view", "aten._unsafe_view", "aten.as_strided", "aten.detach", "aten.t", "aten.expand",
        "aten.permute", "aten.slice", "aten.select", "aten.empty", "aten.empty_strided", "aten.empty_like",
        "aten.alias", "aten.unsqueeze", "aten.squeeze", "aten.reshape", "aten.lift_fresh", "aten.split",
        "aten.unbind", "aten.is_same_size"}


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func.overloadpacket)
        if name not in SKIP:
            shapes = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))[:3]
            where = "autograd engine"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if "deconv_api_amd" in fr.filename:
                    where = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}"
                    break
            self.rows[(name, shapes, where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=["inception_v3", "resnet50"])
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--tile", type=int, default=512)
    ap.add_argument("--dtype", default="fp16", choices=["bf16", "fp16"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    if a.model == "resnet50":
        from deconv_api_amd.models.resnet50 import ResNet50

        net = ResNet50(0).build(dev, dt)
        s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=1, iterations=2)
        dd = TiledDeepDream(net, s, tile=a.tile, use_graphs=False)
    else:
        from deconv_api_amd.models.inception_v3 import InceptionV3

        net = InceptionV3(0).build(dev, dt)
        s = DreamSettings(octaves=1, iterations=2)
        dd = DeepDream(net, s, use_graphs=False)
    x = torch.rand(a.batch, a.size, a.size, 3, device=dev) * 2 - 1
    dd.gradient_ascent(x)  # warm: states, plans, lazily-built weights
    torch.cuda.synchronize()
    log = Log()
    with log:
        dd.gradient_ascent(x)
    torch.cuda.synchronize()
    print(f"{'count':>5s}  {'op':32s} {'shapes':60s} where")
    for (name, shapes, where), n in sorted(log.rows.items(), key=lambda kv: -kv[1]):
        print(f"{n:5d}  {name:32s} {str(shapes)[:60]:60s} {where}")


if __name__ == "__main__":
    main()
