"""Run one conv layer shape repeatedly (for rocprofv3 counter collection / A-B of kernel choices).

    python tools/bench_layer.py --case b1c2down --impl auto --reps 5
Cases mirror the deconvnet's hottest launches at B*K = 1024 (VGG16 block5_conv3 backward).
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.ops.conv import ConvWeights, set_policy  # noqa: E402

CASES = {
    # name: (N, H, W, C, OC, unpool, epilogue)
    "b1c2down": (1024, 224, 224, 64, 64, True, "bf16"),
    "b1c1down": (1024, 224, 224, 64, 3, False, "f32"),
    "b2c1down": (1024, 112, 112, 128, 64, False, "bf16"),
    "b4c2down": (1024, 28, 28, 512, 512, False, "bf16"),
    "b3c2down": (1024, 56, 56, 256, 256, False, "bf16"),
    "b5c2down": (1024, 14, 14, 512, 512, False, "bf16"),
    "b3c2fwd": (256, 56, 56, 256, 256, False, "bf16"),
    "b1c2fwd": (256, 224, 224, 64, 64, False, "pool"),
    "b1c1fwd": (256, 224, 224, 8, 64, False, "bf16"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="b1c2down", choices=sorted(CASES))
    ap.add_argument("--impl", default="auto")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=0, help="override N")
    a = ap.parse_args()
    N, H, W, C, OC, unpool, epi = CASES[a.case]
    N = a.batch or N
    set_policy(impl=a.impl)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    w = torch.randn(OC, C, 3, 3) / (3 * C ** 0.5)
    cw = ConvWeights(w, None, "fwd").to_device(dev)
    if unpool:
        x = torch.randn(N, H // 2, W // 2, C, device=dev, generator=g).to(torch.bfloat16)
        code = torch.randint(0, 4, (N // 4, H // 2, W // 2, C), device=dev, generator=g, dtype=torch.uint8)
        kw = dict(in_mode="unpool", code=code, code_div=4)
    else:
        x = torch.randn(N, H, W, C, device=dev, generator=g).to(torch.bfloat16)
        kw = {}
    run = lambda: ops.conv2d(x, cw, relu=True, relu_in="down" in a.case, epilogue=epi, use_bias=False, **kw)  # noqa: E731
    run()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / a.reps
    fl = 2.0 * N * H * W * OC * 9 * C
    print(f"{a.case} impl={a.impl} N={N}: {dt * 1e3:.3f} ms  {fl / dt / 1e12:.1f} TF/s")


if __name__ == "__main__":
    main()
