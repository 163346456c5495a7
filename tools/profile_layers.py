"""Per-conv-launch timing of the deconvnet step (forward + backward) with HIP events.

Prints, for every conv2d call the engine makes, its GEMM shape, time and achieved TFLOP/s, so
kernel work can be aimed at the launches that dominate. Usage (GPU box):
    python tools/profile_layers.py [--batch 256] [--layer block5_conv3] [--reps 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.engine.deconvnet import DeconvNet  # noqa: E402
from deconv_api_amd.models.vgg16 import VGG16  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--layer", default="block5_conv3")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    eng = DeconvNet(VGG16.random(0, include_top=False).build(dev, torch.bfloat16))
    img = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device=dev)
    x = torch.empty(a.batch, 224, 224, 8, dtype=torch.bfloat16, device=dev)
    ops.resize_preprocess(img, x)
    real = ops.conv2d
    records = []

    def timed(xx, cw, **kw):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = real(xx, cw, **kw)
        e.record()
        out = r[0] if isinstance(r, tuple) else r
        N = xx.shape[0]
        OH, OW = out.shape[1], out.shape[2]
        if kw.get("epilogue") == "pool":
            OH, OW = OH * 2, OW * 2
        if kw.get("unpool_out") is not None:  # the output was max-unpooled in the epilogue
            OH, OW = OH // 2, OW // 2
        M = N * OH * OW
        flops = 2.0 * M * cw.cout * cw.KH * cw.KW * cw.cin
        mode = "unpoolo" if kw.get("unpool_out") is not None else kw.get("in_mode", "plain")
        records.append((mode, kw.get("epilogue", "bf16"), M, cw.cout, cw.K, flops, s, e))
        return r

    ops.conv2d = timed
    for rep in range(a.reps):
        records.clear()
        st = eng.forward(x, a.layer)
        idx, _ = eng.select_filters(st.out, 4)
        eng.backward(st, idx)
        torch.cuda.synchronize()
    tot_t = tot_f = 0.0
    print(f"{'mode':8s} {'epi':5s} {'M':>10s} {'N':>5s} {'K':>6s} {'ms':>8s} {'TF/s':>8s}")
    for mode, epi, M, N, K, fl, s, e in records:
        ms = s.elapsed_time(e)
        tot_t += ms
        tot_f += fl
        print(f"{mode:8s} {epi:5s} {M:10d} {N:5d} {K:6d} {ms:8.3f} {fl / ms / 1e9:8.1f}")
    print(f"total conv {tot_t:.2f} ms, {tot_f / 1e12:.2f} TFLOP, {tot_f / tot_t / 1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
