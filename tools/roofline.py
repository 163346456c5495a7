#!/usr/bin/env python
"""Roofline accounting for the BASELINE configs (SURVEY §5.1 "rocprof counters shown").

FLOPs are COUNTED, not hand-written: the framework's own fp32 CPU path (the same engine code, ops on the
torch oracle) runs one unit of work under a dispatch mode that prices every aten convolution / matmul
with torch's flop formulas (torch.utils.flop_counter), and the unit is scaled to the config:

  config 2  VGG16 block5_conv3 deconvnet step: forward of 256 images + the K = 4 deconvolution signals
            per image (1024 backward passes); unit = one image (x 256)
  config 3  InceptionV3 DeepDream batch: 4 octaves x 20 gradient steps (forward + input gradient) of 64
            images at 299^2; unit = one image, one step, per octave (x 20 x 64)
  config 5  ResNet-50 tiled DeepDream batch at 1024^2, tile 512, fp16: per octave the tile plan of
            TiledDeepDream (equal tiles, (tile, image) units); unit = one tile (x units x 20 steps)

With a measured rate (``--img-per-s``, the bench's ``value``) it prints the achieved PFLOP/s and % of the
dense MFMA peak (2.5 PF/s bf16 / fp16; AMD's headline figures with 2:1 sparsity are never used). With a
rocprofv3 kernel-trace database (``--db``, ``rocprofv3 --kernel-trace -d DIR -o NAME``) it also prints each
kernel family's time per unit of work and share, and the conv families' aggregate PF/s.

  python tools/roofline.py --config 2 --img-per-s 7400 [--db gpurun_out/prof/x_results.db --db-units 3]
"""
from __future__ import annotations

import argparse
import os
import re
import sqlite3
import sys
from collections import defaultdict

import torch
from torch.utils import flop_counter as fc
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PEAK_PF = 2.5  # dense bf16 / fp16 MFMA, MI355X
HBM_TBS = 8.0


class FlopLog(TorchDispatchMode):
    """Every priced aten op in call order: (op name, flops)."""

    def __init__(self):
        super().__init__()
        self.calls = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        pk = func._overloadpacket
        if pk in fc.flop_registry:
            self.calls.append((str(pk).split(".")[-1], int(fc.flop_registry[pk](*args, **kwargs, out_val=out))))
        return out

    @property
    def total(self) -> int:
        return sum(f for _, f in self.calls)


def config2():
    """GFLOP per deconvnet step (256 images, K = 4) -> (total, [(label, flops)])."""
    from deconv_api_amd.engine.deconvnet import DeconvNet
    from deconv_api_amd.models.vgg16 import VGG16

    eng = DeconvNet(VGG16.random(0, include_top=False).build(torch.device("cpu"), torch.float32))
    x = torch.rand(1, 224, 224, 8) * 255
    with torch.no_grad(), FlopLog() as fl:
        eng.run(x, "block5_conv3", k=4, mode="all")
    return 256 * fl.total, [("per image", fl.total)], 256


def _dream_net(model):
    if model == "inception_v3":
        from deconv_api_amd.models.inception_v3 import InceptionV3

        return InceptionV3(0).build(torch.device("cpu"), torch.float32)
    from deconv_api_amd.models.resnet50 import ResNet50

    return ResNet50(0).build(torch.device("cpu"), torch.float32)


def _step_flops(dd, hw):
    x = torch.rand(1, hw[0], hw[1], 3) * 2 - 1
    with FlopLog() as fl:
        dd.loss_and_grad(x)
    return fl.total


def config3(batch=64, size=299, octaves=4, steps=20):
    from deconv_api_amd.engine.deepdream import DeepDream, DreamSettings

    dd = DeepDream(_dream_net("inception_v3"), DreamSettings(octaves=octaves, iterations=steps), use_graphs=False)
    rows = []
    for hw in dd.octave_shapes(size, size):
        f = _step_flops(dd, hw)
        rows.append((f"octave {hw[0]}x{hw[1]}: {f / 1e9:.1f} GFLOP/img/step", f * steps * batch))
    return sum(f for _, f in rows), rows, batch


def config5(batch=8, size=1024, tile=512, octaves=4, steps=20):
    from deconv_api_amd.engine.deepdream import RESNET_LAYERS, DreamSettings, TiledDeepDream

    s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=octaves, iterations=steps)
    dd = TiledDeepDream(_dream_net("resnet50"), s, tile=tile, use_graphs=False)
    rows = []
    for hw in dd.octave_shapes(size, size):
        Th, Tw, tiles = dd._tiles(*hw)
        f = _step_flops(dd, (Th, Tw))
        rows.append((f"octave {hw[0]}x{hw[1]}: {len(tiles)} tiles of {Th}x{Tw}, {f / 1e9:.1f} GFLOP/tile/step",
                     f * len(tiles) * batch * steps))
    return sum(f for _, f in rows), rows, batch


def family(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*\)$", "", name)
    return re.sub(r"<.*", "", name)


def db_families(db: str, last_frac: float, marker: str = "", last_units: int = 0):
    """Per-family (launches, ms) over the window; with ``marker`` the window is from the first to the last
    launch of that kernel family in the trace's last fraction, i.e. exactly (markers - 1) units of work."""
    c = sqlite3.connect(db)
    rows = sorted(c.execute("select name, start, end from kernels").fetchall(), key=lambda r: r[1])
    t0, t1 = min(r[1] for r in rows), max(r[2] for r in rows)
    cut = t1 - (t1 - t0) * last_frac
    end = None
    units = None
    if marker:
        ms = [r[1] for r in rows if r[1] >= cut and marker in r[0]]
        if last_units > 0:
            ms = ms[-(last_units + 1):]
        if len(ms) >= 2:
            cut, end, units = ms[0], ms[-1], len(ms) - 1
    agg = defaultdict(lambda: [0, 0.0])
    lo = hi = None
    for n, s, e in rows:
        if s < cut or (end is not None and s >= end):
            continue
        a = agg[family(n)]
        a[0] += 1
        a[1] += (e - s) / 1e6  # ms
        lo = s if lo is None else min(lo, s)
        hi = e if hi is None else max(hi, e)
    span = (end - cut) / 1e6 if end is not None else (hi - lo) / 1e6
    return agg, span, units


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, choices=[2, 3, 5], required=True)
    ap.add_argument("--img-per-s", type=float, default=0.0, help="measured rate (bench JSON value)")
    ap.add_argument("--db", default="", help="rocprofv3 kernel-trace results db")
    ap.add_argument("--last-units", type=int, default=0, help="db + --unit-marker: only the last N units")
    ap.add_argument("--marker-per-unit", type=float, default=1.0,
                    help="db: marker launches per unit (config 3: 160 dream_update per batch; 5: 80 tile_update)")
    ap.add_argument("--db-units", type=float, default=1.0,
                    help="units of work (config-2 steps / dream batches) in the db window")
    ap.add_argument("--last-frac", type=float, default=1.0, help="db: only the last fraction of the trace")
    ap.add_argument("--unit-marker", default="",
                    help="db: a kernel launched once per unit of work (config 2: resize_preprocess; 3 / 5: "
                         "dream_update / tile_update x steps): the window spans whole units between its launches")
    a = ap.parse_args(argv)
    total, rows, imgs = {2: config2, 3: config3, 5: config5}[a.config]()
    unit = {2: "step (256 images, K = 4)", 3: "dream batch (64 images)", 5: "dream batch (8 images)"}[a.config]
    print(f"config {a.config}: {total / 1e12:.2f} TFLOP of conv/matmul per {unit}")
    for lab, f in rows:
        print(f"  {lab}: {f / 1e12:.2f} TFLOP per {unit.split(' (')[0]}")
    ideal_ms = total / (PEAK_PF * 1e15) * 1e3
    print(f"  at the {PEAK_PF} PF/s dense peak: {ideal_ms:.2f} ms per {unit.split(' (')[0]} "
          f"= {imgs / ideal_ms * 1e3:.0f} img/s")
    if a.img_per_s > 0:
        ms = imgs / a.img_per_s * 1e3
        pf = total / (ms / 1e3) / 1e15
        print(f"measured {a.img_per_s:.1f} img/s = {ms:.2f} ms per unit: {pf:.3f} PF/s = "
              f"{100 * pf / PEAK_PF:.1f} % of the dense MFMA peak")
    if a.db:
        agg, span, units = db_families(a.db, a.last_frac, a.unit_marker, a.last_units)
        busy = sum(v[1] for v in agg.values())
        per = units / a.marker_per_unit if units else a.db_units
        print(f"db: {span:.1f} ms window, {busy:.1f} ms kernel-busy ({100 * busy / max(span, 1e-9):.0f} %), "
              f"{per:g} units -> {span / per:.2f} ms wall / {busy / per:.2f} ms busy per unit")
        conv_ms = sum(v[1] for k, v in agg.items() if "conv" in k) / per
        print(f"  conv kernels: {conv_ms:.2f} ms per unit -> {total / (conv_ms / 1e3) / 1e15:.3f} PF/s "
              f"({100 * total / (conv_ms / 1e3) / 1e15 / PEAK_PF:.1f} % of peak while a conv runs)")
        print(f"  {'family':<44} {'launches/unit':>14} {'ms/unit':>9} {'share':>7}")
        for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
            print(f"  {k[:44]:<44} {n / per:>14.1f} {ms / per:>9.3f} {100 * ms / busy:>6.1f}%")


if __name__ == "__main__":
    main()
