"""Per-conv-launch timing of one DeepDream gradient step (forward + input-gradient backward).

For each octave shape of the config it prints every conv2d launch (which unit, fwd/bwd, GEMM
M x N x K, ms, TF/s), the conv total against the whole (eager) step, and a per-unit summary, so
kernel work can be aimed at the launches that dominate. Usage (GPU box):

    python tools/profile_dream.py --model inception_v3 --batch 64 --size 299
    python tools/profile_dream.py --model resnet50 --batch 8 --size 512 --dtype fp16
"""
import argparse
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.engine.deepdream import RESNET_LAYERS, DeepDream, DreamSettings  # noqa: E402
from deconv_api_amd.ops import autograd as ag  # noqa: E402
from deconv_api_amd.ops import inception as inc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--size", type=int, default=299)
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops.native.load()
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
        names[id(u.fwd)] = (n, "fwd")
        names[id(u.bwd)] = (n, "bwd")
        for i, (_, _, cw, _) in enumerate(getattr(u, "bwd_sub", []) or []):
            if cw is not None:
                names[id(cw)] = (n, f"bwd.sub{i}")
        if getattr(u, "col_w", None) is not None:
            names[id(u.col_w)] = (n, "bwd.col")
    dd = DeepDream(net, s, use_graphs=False)
    real = ag.conv2d
    records = []

    def timed(xx, cw, **kw):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        r = real(xx, cw, **kw)
        en.record()
        out = kw.get("out")
        y = r[0] if isinstance(r, tuple) else r
        oh, ow = (y.shape[1], y.shape[2]) if out is None else (out.shape[1], out.shape[2])
        M = xx.shape[0] * oh * ow
        fl = 2.0 * M * cw.cout * cw.KH * cw.KW * cw.cin
        # compulsory HBM bytes: input + output (+ residual / output-mask / accumulate reads)
        by = xx.numel() * xx.element_size() + M * cw.cout * y.element_size()
        for k in ("res", "emask"):
            if kw.get(k) is not None:
                by += kw[k].numel() * kw[k].element_size()
        if kw.get("accumulate"):
            by += M * cw.cout * y.element_size()
        records.append((names.get(id(cw), ("?", "?")), M, cw.cout, cw.K, fl, by, st, en))
        return r

    ag.conv2d = timed
    inc.conv2d = timed
    for blk in getattr(net, "iblocks", []):  # merged head GEMMs
        if blk.merge is not None:
            names[id(blk.merge[0])] = (blk.name + ".heads", "fwd")
            names[id(blk.merge[1])] = (blk.name + ".heads", "bwd")
    per_unit = defaultdict(lambda: [0.0, 0.0])
    grand_t = grand_f = grand_step = 0.0
    for hw in dd.octave_shapes(a.size, a.size):
        x = torch.rand(a.batch, *hw, 3, device=dev) * 2 - 1
        for rep in range(a.reps):
            records.clear()
            torch.cuda.synchronize()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            dd.loss_and_grad(x)
            s1.record()
            torch.cuda.synchronize()
        step_ms = s0.elapsed_time(s1)
        tot_t = tot_f = 0.0
        rows = []
        for (n, kind), M, N, K, fl, by, st, en in records:
            ms = st.elapsed_time(en)
            tot_t += ms
            tot_f += fl
            rows.append((ms, n, kind, M, N, K, fl, by))
            per_unit[(n, kind)][0] += ms
            per_unit[(n, kind)][1] += fl
        grand_t += tot_t
        grand_f += tot_f
        grand_step += step_ms
        print(f"=== octave {hw[0]}x{hw[1]}  batch {a.batch}: step {step_ms:.2f} ms (eager), conv {tot_t:.2f} ms "
              f"in {len(rows)} launches, {tot_f / 1e12:.3f} TFLOP, {tot_f / tot_t / 1e9:.0f} TF/s on conv time, "
              f"{tot_f / step_ms / 1e9:.0f} TF/s on step time")
        rows.sort(reverse=True)
        print(f"  {'unit':22s} {'kind':9s} {'M':>9s} {'N':>5s} {'K':>6s} {'ms':>7s} {'TF/s':>7s} {'GB/s':>7s}")
        for ms, n, kind, M, N, K, fl, by in rows[: a.top]:
            print(f"  {n:22s} {kind:9s} {M:9d} {N:5d} {K:6d} {ms:7.3f} {fl / ms / 1e9:7.0f} {by / ms / 1e6:7.0f}")
    print(f"=== all octaves: step {grand_step:.2f} ms, conv {grand_t:.2f} ms, {grand_f / 1e12:.3f} TFLOP "
          f"({grand_f / grand_step / 1e9:.0f} TF/s on step time)")
    print("per unit (summed over octaves):")
    for (n, kind), (ms, fl) in sorted(per_unit.items(), key=lambda kv: -kv[1][0])[: a.top * 2]:
        print(f"  {n:22s} {kind:9s} {ms:7.3f} ms {fl / ms / 1e9:7.0f} TF/s")


if __name__ == "__main__":
    main()
