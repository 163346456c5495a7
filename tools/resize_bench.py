"""Time the fused resize + preprocess kernel (csrc/misc.hip) on the bench / serving shapes:
B images uint8 [Hs, Ws, 3] -> bf16 [224, 224, 8]; reports us per batch and effective GB/s."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deconv_api_amd import ops  # noqa: E402


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    ops.native.load()
    B = a.batch
    out = torch.empty(B, 224, 224, 8, dtype=torch.bfloat16, device="cuda")
    res = {}
    for hs, ws in ((224, 224), (448, 448), (375, 500), (480, 640)):
        img = torch.randint(0, 256, (B, hs, ws, 3), dtype=torch.uint8, device="cuda")
        us = t(lambda: ops.resize_preprocess(img, out))
        gb = (img.numel() + out.numel() * 2) / 1e9
        res[f"{hs}x{ws}"] = {"us": round(us, 1), "GB_per_s": round(gb / (us * 1e-6), 1)}
    src = torch.empty(out.numel() * 2 // 4, dtype=torch.int32, device="cuda")
    dst = torch.empty_like(src)
    res["copy_same_bytes_us"] = round(t(lambda: dst.copy_(src)), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
