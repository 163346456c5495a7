"""A/B of ResNet-50's conv1 forward: the tap-paired MFMA kernel (csrc/conv_stem7.hip) vs the generic
implicit GEMM (DV_STEM7=0 path), on config 5's tile shapes (fp16, 512^2 tiles, chunks of 4 / 16).

    python tools/stem7_ab.py [--batch 4 16] [--size 512] [--reps 50]
"""
from __future__ import annotations

import argparse
import os

os.environ.setdefault("DV_ABLATIONS", "1")  # this tool A/Bs switches of deconv_api_amd/knobs.py ABLATION
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deconv_api_amd.ops import autograd as AG  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[4, 16])
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16"])
    a = ap.parse_args(argv)
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    g = torch.Generator().manual_seed(0)
    w = torch.randn(64, 3, 7, 7, generator=g) / (3 * 49) ** 0.5
    b = torch.randn(64, generator=g) * 0.1
    unit = AG.ConvUnit("conv1", w, b, 2, (3, 3), relu=True).build("cuda", dt)
    for n in a.batch:
        x = torch.nn.functional.pad(torch.randn(n, a.size, a.size, 3, generator=g), (0, 5)).to(dt).cuda()
        res = {}
        for path in ("stem7", "gemm"):
            AG.STEM7 = path == "stem7"
            fn = (lambda: AG._stem_fwd(x, unit)) if path == "stem7" else (lambda: unit(x))
            y = fn()
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            res[path] = (us, y.float())
        AG.STEM7 = True
        # the fused input gradient (csrc/conv_stem_dgrad.hip) on the same shapes, premasked (mask None)
        gy = torch.randn(*res["stem7"][1].shape, generator=g).to(dt).cuda()
        fd = lambda: AG._col2im_dgrad(gy, None, unit, (a.size, a.size))  # noqa: E731
        for _ in range(5):
            fd()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fd()
        e1.record()
        torch.cuda.synchronize()
        dus = e0.elapsed_time(e1) * 1e3 / a.reps
        print(f"N={n} stem dgrad (fused): {dus:.1f} us ({(gy.numel() + x.numel()) * 2 / dus / 1e6:.2f} TB/s)", flush=True)
        by = x.numel() * 2 + res["stem7"][1].numel() * 2
        diff = float((res["stem7"][1] - res["gemm"][1]).abs().max())
        print(f"N={n} {a.size}^2 {a.dtype}: stem7 {res['stem7'][0]:.1f} us ({by / res['stem7'][0] / 1e6:.2f} TB/s)"
              f"  gemm {res['gemm'][0]:.1f} us ({by / res['gemm'][0] / 1e6:.2f} TB/s)"
              f"  speedup {res['gemm'][0] / res['stem7'][0]:.2f}x  max|diff| {diff:.3g}", flush=True)


if __name__ == "__main__":
    main()
