"""Time the fused deconvnet tail (ops.deconv_tail: conv_unpool_z + zsum3x3) alone at the config-2
shape (B*K = 1024 signals, pooled 112^2 x 64 input, 224^2 output), with HIP events per kernel.

    python tools/bench_tail.py [--n 1024] [--reps 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.ops import native  # noqa: E402
from deconv_api_amd.ops.conv import ConvWeights, tail_w2  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--k", type=int, default=4, help="signals per image (code_div)")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    N, PH = a.n, 112
    x = torch.randn(N, PH, PH, 64, device=dev, generator=g).relu_().to(torch.bfloat16)
    code = torch.randint(0, 4, (N // a.k, PH, PH, 64), device=dev, generator=g, dtype=torch.uint8)
    cg = torch.Generator().manual_seed(1)
    mid = ConvWeights(torch.randn(64, 64, 3, 3, generator=cg) * 0.05, None).to_device(dev)
    last = ConvWeights(torch.randn(3, 64, 3, 3, generator=cg) * 0.05, None).to_device(dev)
    lib = native.lib()
    z = torch.empty(N, 2 * PH, 2 * PH, 32, dtype=torch.bfloat16, device=dev)
    out = torch.empty(N, 2 * PH, 2 * PH, 3, dtype=torch.float32, device=dev)
    w2 = tail_w2(last)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tz, ts = [], []
    for r in range(a.reps + 2):
        ev[0].record()
        assert lib.conv_unpool_z(x, code, a.k, mid.w_gemm, w2, z)
        ev[1].record()
        lib.zsum3x3(z, out, None, 1)
        ev[2].record()
        torch.cuda.synchronize()
        if r >= 2:
            tz.append(ev[0].elapsed_time(ev[1]))
            ts.append(ev[1].elapsed_time(ev[2]))
    flops = 2.0 * N * (2 * PH) ** 2 * 64 * 576
    tz.sort()
    ts.sort()
    mz, ms = tz[len(tz) // 2], ts[len(ts) // 2]
    print(f"conv_unpool_z {mz:.3f} ms ({flops / mz / 1e9:.0f} TF/s), zsum3x3 {ms:.3f} ms, total {mz + ms:.3f} ms")
    # numerics against the same-rounding fp32 oracle on a slice
    ref = ops.deconv_tail_ref(x[:8], code[: 8 // a.k], a.k, mid, last)
    got = out[:8].cpu()
    err = ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
    print(f"max rel err vs oracle (8 signals): {err:.2e}")


if __name__ == "__main__":
    main()
