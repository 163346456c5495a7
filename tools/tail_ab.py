"""Timing of the fused deconvnet tail (ops.deconv_tail: conv3x3_unpool_c64_v2_kernel<ZOUT> + zsum3x3) at the
config-2 shape (1024 signals, 112^2 pooled -> 224^2) for DV_TAIL_V schedules / ablations, interleaved in ONE
process. Ablation bits (timing only, WRONG outputs; DV_ALLOW_WRONG_ABLATION=1 is set here): 4 = no Z GEMM /
stores, 8 = no halo expansion (csrc/conv_smalln.hip). Times include the zsum3x3 launch (~0.72 ms).

    python tools/tail_ab.py --vars 0,3,7,11,15 --rounds 5 --reps 10
"""
import argparse
import json
import os

os.environ.setdefault("DV_ABLATIONS", "1")  # this tool A/Bs switches of deconv_api_amd/knobs.py ABLATION
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.ops.conv import ConvWeights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vars", default="0,3,7,11,15")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    os.environ["DV_ALLOW_WRONG_ABLATION"] = "1"
    ops.native.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    N, H, W, div = a.n, 224, 224, 4
    p = (torch.randn(N, H // 2, W // 2, 64, device=dev, generator=g)).to(torch.bfloat16)
    code = torch.randint(0, 4, (N // div, H // 2, W // 2, 64), device=dev, dtype=torch.uint8, generator=g)
    mid = ConvWeights(torch.randn(64, 64, 3, 3) / 24, None, "fwd").to_device(dev)
    last = ConvWeights(torch.randn(3, 64, 3, 3) / 24, None, "fwd").to_device(dev)
    variants = [int(v) for v in a.vars.split(",")]

    def run(v):
        os.environ["DV_TAIL_V"] = str(v)
        return ops.deconv_tail(p, code, div, mid, last)

    ref = run(3).clone()
    for v in variants:
        out = run(v)
        if v in (0, 1, 2, 3):  # exact schedules: bit-identical to the shipped one
            print(json.dumps({"tail_v": v, "bit_identical_to_3": bool(torch.equal(out, ref))}), flush=True)
    torch.cuda.synchronize()
    times = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run(v)
            e1.record()
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.reps)
    os.environ.pop("DV_TAIL_V", None)
    for v in variants:
        print(json.dumps({"tail_v": v, "ms_median": round(statistics.median(times[v]), 4),
                          "ms_min": round(min(times[v]), 4)}), flush=True)


if __name__ == "__main__":
    main()
