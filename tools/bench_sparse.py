"""A/B of the 2:4 sparse-MFMA unpool conv-down against the dense path (unpooled map + DMA conv) on
the flagship's unpool-fed conv-down shapes (B*K = 1024, VGG16 block5_conv3 backward).

    python tools/bench_sparse.py --reps 10
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.ops import sparse_unpool as su  # noqa: E402
from deconv_api_amd.ops.conv import ConvWeights  # noqa: E402

CASES = {  # name: (NB, PH, PW, C (unpooled channels), Ci (conv-down outputs))
    "b4c3down": (1024, 14, 14, 512, 512),
    "b3c3down": (1024, 28, 28, 256, 256),
    "b2c2down": (1024, 56, 56, 128, 128),
}


def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cases", default=",".join(CASES))
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name in a.cases.split(","):
        NB, PH, PW, C, Ci = CASES[name]
        g = torch.Generator(device=dev).manual_seed(0)
        v = torch.randn(NB, PH, PW, C, device=dev, generator=g).to(torch.bfloat16)
        code = torch.randint(0, 4, (NB // 4, PH, PW, C), device=dev, generator=g, dtype=torch.uint8)
        w = torch.randn(C, Ci, 3, 3) / (3 * C ** 0.5)
        wt = su.pack_for_kernel(w, dev)
        u = ops.unpool2x2(v, code, 4, relu=True)
        # dense path: conv over the (3/4 zero) unpooled map with the conv-down's correlation kernel
        wd = su.corr_weights(w).permute(3, 2, 0, 1).contiguous()  # [Ci, C, 3, 3] as a forward conv
        cw = ConvWeights(wd, None, "fwd").to_device(dev)
        out_s = torch.empty(NB, 2 * PH, 2 * PW, Ci, dtype=torch.bfloat16, device=dev)
        t_dense = _time(lambda: ops.conv2d(u, cw, relu=True, use_bias=False), a.reps)
        t_sparse = _time(lambda: su.sparse_unpool_conv(v, code, wt, 4, out=out_s), a.reps)
        ref = ops.conv2d(u, cw, relu=True, use_bias=False).float()
        got = su.sparse_unpool_conv(v, code, wt, 4).float()
        rel = ((got - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * NB * 4 * PH * PW * Ci * 9 * C
        print(f"{name}: dense {t_dense:.3f} ms ({fl / t_dense / 1e9:.0f} TF/s)  sparse {t_sparse:.3f} ms "
              f"({fl / t_sparse / 1e9:.0f} dense-equiv TF/s)  speedup {t_dense / t_sparse:.2f}x  max rel diff {rel:.2e}",
              flush=True)


if __name__ == "__main__":
    main()
