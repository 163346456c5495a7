#!/usr/bin/env python
"""Flagship benchmark: VGG16 block5_conv3 deconvnet, 256 synthetic 224x224 images per GPU, bf16.

One timed step = what the reference's ``POST /`` computes for a batch of images (app/main.py:
45-78), minus only the host JPEG encode: preprocess (uint8 -> caffe bf16 NHWC), VGG16 forward to
the target with fused pool+switch, per-image top-4 filter selection, 4 deconv chains per image
to the input (unpool fused into the conv-down gather), 2x2 mosaic + deprocess to uint8, and with
N > 1 an RCCL all-gather of every rank's uint8 mosaics over xGMI (weak scaling: 256 img/GPU).

Run: ``python bench.py [--gpus N --steps K --warmup W]``; for N > 1 under
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N``.
Rank 0 prints ONE JSON line. Weights: seeded random-init VGG16 (no network for ImageNet
weights); data: synthetic uint8 images.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

from deconv_api_amd import ops
from deconv_api_amd.engine.deconvnet import DeconvNet
from deconv_api_amd.models.vgg16 import VGG16
from deconv_api_amd.parallel import dist as pdist

# the reference's implied end-to-end rate for layer=block5_conv3 is ~0.03-0.04 img/s
# (CPU, one request at a time; a lower bound on its cost). We divide by the favourable 0.04.
REF_IMG_PER_S = 0.04
METRIC = "images/sec, VGG16 deconv 224px (block5_conv3 deconvnet, top-4 mosaic)"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--layer", default="block5_conv3")
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--breakdown", action="store_true", help="per-phase timing to stderr (extra syncs)")
    return ap.parse_args(argv)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main(argv=None):
    args = parse(argv)
    info = pdist.init()
    if info.world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={info.world}; using WORLD_SIZE")
    dev = info.device
    if dev.type != "cuda":
        raise SystemExit("bench.py needs a GPU (MI355X)")
    ops.native.load()

    # ---- weights: built on rank 0, broadcast once over RCCL ----
    t0 = time.time()
    model = VGG16.random(args.seed) if info.is_main else VGG16.random(args.seed + 12345)
    if info.world > 1:
        sd = pdist.broadcast_state(model.state_dict(), info)
        model = VGG16.from_state_dict(sd)
    rt = model.build(dev, torch.bfloat16)
    eng = DeconvNet(rt)
    log(f"[rank {info.rank}] weights ready in {time.time() - t0:.1f}s ({model.num_params() / 1e6:.1f}M params)")

    B = args.batch
    g = torch.Generator(device=dev).manual_seed(1000 + info.rank)
    images = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev, generator=g)
    xbuf = torch.empty(B, 224, 224, 8, dtype=torch.bfloat16, device=dev)
    gathered = torch.empty(info.world * B, 448, 448, 3, dtype=torch.uint8, device=dev) if info.world > 1 else None

    def step():
        ops.resize_preprocess(images, xbuf)
        res = eng.run(xbuf, args.layer, k=args.k)
        out = pdist.all_gather_rows(res.mosaic, info, gathered)
        return res, out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    if args.breakdown and info.is_main:
        _breakdown(eng, images, xbuf, args)

    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    pdist.barrier(info)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    evs[0].record()
    for i in range(args.steps):
        step()
        evs[i + 1].record()
    torch.cuda.synchronize()
    pdist.barrier(info)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    elapsed = pdist.all_reduce_max(elapsed, info)
    per_step = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    p50 = per_step[len(per_step) // 2]
    p50 = pdist.all_reduce_max(p50, info)

    ms = elapsed / args.steps * 1e3
    total_imgs = B * info.world * args.steps
    value = total_imgs / elapsed
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": info.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "p50_batch_latency_ms": round(p50, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / REF_IMG_PER_S, 1),
        "baseline_img_per_s": REF_IMG_PER_S,
        "dtype": "bf16",
        "data": "synthetic uint8 224x224 images, seeded random-init VGG16 weights",
        "config": {"model": f"vgg16_deconvnet_{args.layer}", "global_batch": B * info.world, "seq_len": 224,
                   "image_size": 224, "filters_per_image": args.k, "parallelism": f"dp{info.world}"},
    }
    if info.is_main:
        print(json.dumps(line), flush=True)
    pdist.shutdown()


def _breakdown(eng, images, xbuf, args):
    """Per-phase wall time with syncs (diagnostic only, not the reported number)."""
    def t(fn):
        torch.cuda.synchronize()
        a = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return r, (time.perf_counter() - a) * 1e3

    _, tp = t(lambda: ops.resize_preprocess(images, xbuf))
    st, tf = t(lambda: eng.forward(xbuf, args.layer))
    (idx, _), ts = t(lambda: eng.select_filters(st.out, args.k))
    rec, tb = t(lambda: eng.backward(st, idx))
    B = rec.shape[0]
    _, td = t(lambda: ops.deprocess_mosaic(rec.reshape(B * args.k, *rec.shape[2:]).contiguous()))
    log(f"breakdown ms: preprocess {tp:.2f} forward {tf:.2f} select {ts:.2f} backward {tb:.2f} deprocess {td:.2f}")


if __name__ == "__main__":
    main()
