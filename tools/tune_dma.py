"""Sweep the LDS-DMA conv kernel's tile configs x split-K factors on every conv launch of one
DeepDream step (or any engine step) and report the automatic choice against the best one.

Each conv2d call of the step is intercepted while its inputs are live and re-run under every
forced (tile config, split-K) pair (``_C.dma_tune``; configs in csrc/conv_dma.hip:dma_forced),
timed over ``--reps`` back-to-back launches with HIP events. Usage (GPU box):

    python tools/tune_dma.py --model inception_v3 --batch 64 --size 299 --octaves 4
    python tools/tune_dma.py --model resnet50 --batch 32 --size 512 --octaves 1 --dtype fp16
"""
import argparse
import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.engine.deepdream import RESNET_LAYERS, DeepDream, DreamSettings  # noqa: E402
from deconv_api_amd.ops import autograd as ag  # noqa: E402

CFG_NAMES = {0: "auto", 1: "256x256", 2: "128x256", 3: "128x128", 4: "256x128", 5: "256x64", 6: "512x64",
             7: "128x64w4", 8: "64x64w4", 9: "128x128w4", 10: "64x128w4", 11: "256x64w4",
             12: "64x64w4s6", 13: "64x64w4s8", 14: "128x64w4s6", 15: "64x128w4s6"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=299)
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cfgs", default="0,1,2,3,4,5,6,7,8,9,10,11,12,13,14,15")
    ap.add_argument("--ks", default="0,1,2,4,8")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = ops.native.lib()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    if a.model == "inception_v3":
        from deconv_api_amd.models.inception_v3 import InceptionV3

        net = InceptionV3(0).build(dev, dt)
        s = DreamSettings(octaves=a.octaves)
    else:
        from deconv_api_amd.models.resnet50 import ResNet50

        net = ResNet50(0).build(dev, dt)
        s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=a.octaves)
    names = {}
    for n, u in net.units.items():
        names[id(u.fwd)] = f"{n}.fwd"
        names[id(u.bwd)] = f"{n}.bwd"
        for i, (_, _, cw, _) in enumerate(getattr(u, "bwd_sub", []) or []):
            if cw is not None:
                names[id(cw)] = f"{n}.sub{i}"
        if getattr(u, "col_w", None) is not None:
            names[id(u.col_w)] = f"{n}.col"
    cfgs = [int(c) for c in a.cfgs.split(",")]
    kss = [int(k) for k in a.ks.split(",")]
    dd = DeepDream(net, s, use_graphs=False)
    real = ag.conv2d
    results = []

    def time_call(xx, cw, kw):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        real(xx, cw, **kw)  # warm
        st.record()
        for _ in range(a.reps):
            real(xx, cw, **kw)
        en.record()
        en.synchronize()
        return st.elapsed_time(en) / a.reps

    def tuned(xx, cw, **kw):
        y = real(xx, cw, **kw)
        out = y[0] if isinstance(y, tuple) else y
        M = xx.shape[0] * out.shape[1] * out.shape[2]
        fl = 2.0 * M * cw.cout * cw.KH * cw.KW * cw.cin
        row = {"unit": names.get(id(cw), "?"), "M": M, "N": cw.cout, "K": cw.K, "KH": cw.KH, "KW": cw.KW,
               "res": kw.get("res") is not None, "emask": kw.get("emask") is not None,
               "mask": kw.get("mask") is not None, "acc": bool(kw.get("accumulate")), "flop": fl, "t": {}}
        for c in cfgs:
            for k in kss:
                if c == 0 and k != 0:
                    continue
                lib.dma_tune(c, k)
                try:
                    row["t"][f"{c}/{k}"] = time_call(xx, cw, kw)
                except RuntimeError:
                    pass
        lib.dma_tune(0, 0)
        results.append(row)
        return y

    ag.conv2d = tuned
    for hw in dd.octave_shapes(a.size, a.size):
        x = torch.rand(a.batch, *hw, 3, device=dev) * 2 - 1
        dd.loss_and_grad(x)
        torch.cuda.synchronize()
    ag.conv2d = real
    tot_auto = tot_best = 0.0
    wins = defaultdict(int)
    print(f"{'unit':24s} {'M':>8s} {'N':>5s} {'K':>5s} {'auto_us':>8s} {'best_us':>8s} best_cfg")
    for r in results:
        ta = r["t"].get("0/0")
        if ta is None or not r["t"]:
            continue
        bk, bt = min(r["t"].items(), key=lambda kv: kv[1])
        tot_auto += ta
        tot_best += bt
        c, k = bk.split("/")
        wins[(CFG_NAMES[int(c)], k)] += 1
        print(f"{r['unit']:24s} {r['M']:8d} {r['N']:5d} {r['K']:5d} {ta * 1e3:8.1f} {bt * 1e3:8.1f} "
              f"{CFG_NAMES[int(c)]}/ks{k}")
    print(f"total auto {tot_auto:.3f} ms, best {tot_best:.3f} ms ({tot_auto / max(tot_best, 1e-9):.2f}x)")
    print("wins:", dict(sorted(wins.items(), key=lambda kv: -kv[1])))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(results, f)


if __name__ == "__main__":
    main()
