"""A/B of the KW3 conv main-loop variants (csrc/conv_dma_impl.h, conv_dma_kw3_kernel / conv_dma_kw3p_kernel) on the
config-2 launch shapes, interleaved in ONE process (cdna_hip_programming.md §5.4 rule 24).

    python tools/kw3_ab.py --vars 0,2,8,9 --rounds 5 --reps 20

VAR 0 (KW3) / 2 (persistent KW3P, the default) are real kernels (their outputs are compared bit for bit: the
accumulation order is the same); 8 (no epilogue stores) and 9 (no K loop) are ablations that price the epilogue and the
prologue + epilogue of a tile. Prints one JSON line per (case, variant) with the median and min
time over rounds and the conv TF/s.
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

# config-2 KW3 launches (VGG16 block5_conv3 deconvnet, B = 256 images x K = 4 signals): name ->
# (N, H, W, C, OC)
CASES = {
    "b5down": (1024, 14, 14, 512, 512),     # block5_conv{2,3}.down (x2 per step) and conv1.down (unpool-out)
    "b4down": (1024, 28, 28, 512, 512),     # block4_conv{2,3}.down
    "b4c1down": (1024, 28, 28, 512, 256),   # block4_conv1.down: 512 -> 256
    "b3down": (1024, 56, 56, 256, 256),     # block3_conv{2,3}.down
    "b3c1down": (1024, 56, 56, 256, 128),   # block3_conv1.down: 512 x 128 KW3 tile
    "b4fwd": (256, 28, 28, 512, 512),       # block4_conv{2,3} forward
    "b3fwd": (256, 56, 56, 256, 256),       # block3_conv{2,3} forward
    "b5fwd": (256, 14, 14, 512, 512),       # block5 forward (tail-split KW3)
    # unpool-out conv-downs (suffix "unp": max-unpooled output, switch codes shared by 4 signals)
    "b5c1unp": (1024, 14, 14, 512, 512),    # block5_conv1.down -> 28^2
    "b4c1unp": (1024, 28, 28, 512, 256),    # block4_conv1.down -> 56^2
    "b3c1unp": (1024, 56, 56, 256, 128),    # block3_conv1.down -> 112^2 (512 x 128 tile)
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vars", default="0,2,8,9")
    ap.add_argument("--cases", default=",".join(CASES))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    os.environ.setdefault("DV_ALLOW_WRONG_ABLATION", "1")  # VAR 8 / 9 are wrong-output timing ablations
    ops.native.load()
    dev = torch.device("cuda", 0)
    variants = [int(v) for v in a.vars.split(",")]
    g = torch.Generator(device=dev).manual_seed(0)
    for case in a.cases.split(","):
        N, H, W, C, OC = CASES[case]
        w = torch.randn(OC, C, 3, 3) / (3 * C ** 0.5)
        cw = ConvWeights(w, None, "fwd").to_device(dev)
        x = (torch.rand(N, H, W, C, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        out = {v: torch.empty(N, H, W, OC, dtype=torch.bfloat16, device=dev) for v in variants}
        unp = case.endswith("unp")
        code = torch.randint(0, 4, (N // 4, H, W, OC), device=dev, dtype=torch.uint8, generator=g) if unp else None

        def run(v):
            # 2: KW3P as selected (stream-K where it applies, step-1 DMA ahead of the epilogue stores);
            # 12: whole tiles (DV_NO_KW3_SK=1); 13: whole tiles without the early DMA (+ DV_KW3P_NO_PRE=1);
            # 14: stream-K without the early DMA; 15: whole tiles with the register-transposed 8-B store epilogue;
            # 16: stream-K on every eligible grid (DV_KW3_SK=all); 20 / 21: KW3P ablations without any DMA after
            # the first step / without the weight DMA (WRONG outputs: how much of a launch waits on staging)
            os.environ["DV_KW3_VAR"] = str(2 if v in (12, 13, 14, 15, 16, 22) else v)
            for k, on in (("DV_NO_KW3_SK", v in (12, 13, 15)), ("DV_KW3P_NO_PRE", v in (13, 14))):
                if on:
                    os.environ[k] = "1"
                else:
                    os.environ.pop(k, None)
            if v == 15:
                os.environ["DV_KW3P_EPI"] = "reg"
            else:
                os.environ.pop("DV_KW3P_EPI", None)
            if v == 16:
                os.environ["DV_KW3_SK"] = "all"
            else:
                os.environ.pop("DV_KW3_SK", None)
            if v == 22:  # the 512 x 128 KW3P tile on 256 / 512-channel outputs
                os.environ["DV_KW3_TILE"] = "512x128"
            else:
                os.environ.pop("DV_KW3_TILE", None)
            if unp:  # a fresh unpooled output per call (as the engine does)
                out[v] = ops.conv2d(x, cw, relu=True, use_bias=False, unpool_out=code, unpool_div=4)
                return out[v]
            return ops.conv2d(x, cw, relu=True, use_bias=False, out=out[v])

        for v in variants:  # warm up every variant (and check the real ones agree)
            run(v)
        torch.cuda.synchronize()
        real = [v for v in variants if v < 8 or v in (11, 12, 13, 14, 15, 16, 22)]
        for v in real[1:]:
            same = torch.equal(out[v], out[real[0]])
            if not same:  # stream-K vs whole tiles: split tiles round differently
                d = (out[v].float() - out[real[0]].float()).abs()
                same = float(d.max()) <= 2 ** -6 * float(out[real[0]].float().abs().max())
            if not same:
                d = (out[v].float() - out[real[0]].float()).abs().max().item()
                print(json.dumps({"case": case, "var": v, "equal_to": real[0], "equal": False, "maxdiff": d}),
                      flush=True)
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
        fl = 2.0 * N * H * W * OC * 9 * C
        for v in variants:
            med = statistics.median(times[v])
            print(json.dumps({"case": case, "var": v, "ms_median": round(med, 4), "ms_min": round(min(times[v]), 4),
                              "tflops": round(fl / med / 1e9, 1)}), flush=True)
    os.environ.pop("DV_KW3_VAR", None)


if __name__ == "__main__":
    main()
