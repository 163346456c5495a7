"""Command line for files on disk: the service's computations without HTTP.

    python -m deconv_api_amd.cli deconv photo.jpg [more.png ...] --layer block5_conv3 [--out-dir out/]
    python -m deconv_api_amd.cli dream photo.jpg --model inception_v3 --octaves 4 --steps 20 [--out-dir out/]
    python -m deconv_api_amd.cli layers

``deconv`` writes ``<stem>_<layer>.jpg``: the 2x2 mosaic of the top-4 deconvnet reconstructions, the same
image ``POST /`` returns as a data URL (reference: app/main.py:45-78), all files as one batch on the device.
``dream`` writes ``<stem>_dream_<model>.jpg`` (``POST /deepdream``). Configuration as the server's
(``DV_*`` variables, config.py) with ``--device`` / ``--dtype`` / ``--weights`` overrides.
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import List

import numpy as np


def _read(paths: List[str]) -> List[np.ndarray]:
    from .codec import decode_image

    out = []
    for p in paths:
        with open(p, "rb") as f:
            out.append(decode_image(f.read()))
    return out


def _stem(p: str) -> str:
    return os.path.splitext(os.path.basename(p))[0]


def cmd_deconv(a, cfg) -> int:
    from .codec import encode_jpeg
    from .serve.service import DeconvService

    imgs = _read(a.images)
    svc = DeconvService(cfg)
    try:
        svc.engine._check_layer(a.layer)  # an unknown layer fails before any compute
        mos = svc.run_batch(a.layer, imgs)
    finally:
        svc.close()
    os.makedirs(a.out_dir, exist_ok=True)
    from .runtime.staging import GpuScans

    for b, p in enumerate(a.images):
        if isinstance(mos, GpuScans):  # GPU service: the mosaics arrive JPEG-encoded on the device
            from .codec.image import gpu_jpeg_bytes

            jpeg = gpu_jpeg_bytes(mos.packed, mos.off, b, mos.H, mos.W, cfg.jpeg_quality)
        else:
            jpeg = encode_jpeg(np.ascontiguousarray(mos[b]), cfg.jpeg_quality)
        dst = os.path.join(a.out_dir, f"{_stem(p)}_{a.layer}.jpg")
        with open(dst, "wb") as f:
            f.write(jpeg)
        print(dst)
    return 0


def cmd_dream(a, cfg) -> int:
    from .codec import encode_jpeg
    from .serve.dream_service import DreamService

    imgs = _read(a.images)
    ds = DreamService(cfg)
    try:
        outs = [ds.run_batch([ds.prepare(img, a.octaves)], a.model, a.octaves, a.steps)[0] for img in imgs]
    finally:
        ds.close()
    os.makedirs(a.out_dir, exist_ok=True)
    for p, o in zip(a.images, outs):
        dst = os.path.join(a.out_dir, f"{_stem(p)}_dream_{a.model}.jpg")
        with open(dst, "wb") as f:
            f.write(encode_jpeg(np.ascontiguousarray(o), cfg.jpeg_quality))
        print(dst)
    return 0


def cmd_layers(a, cfg) -> int:
    from .models.vgg16 import VGG16_LAYER_NAMES

    print("\n".join(n for n in VGG16_LAYER_NAMES if n != "input_1"))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m deconv_api_amd.cli")
    ap.add_argument("--device", default=None, help="auto | cuda | cpu (DV_DEVICE)")
    ap.add_argument("--dtype", default=None, help="bf16 | fp16 on a GPU (DV_DTYPE)")
    ap.add_argument("--weights", default=None, help="VGG16 weights (DV_WEIGHTS): .safetensors / .pt / Keras .h5")
    sub = ap.add_subparsers(dest="cmd", required=True)
    d = sub.add_parser("deconv", help="deconvnet mosaic of each image")
    d.add_argument("images", nargs="+")
    d.add_argument("--layer", default="block5_conv3")
    d.add_argument("--mode", default=None, help="all | max (DV_MODE)")
    d.add_argument("--out-dir", default=".")
    r = sub.add_parser("dream", help="DeepDream of each image")
    r.add_argument("images", nargs="+")
    r.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    r.add_argument("--octaves", type=int, default=4)
    r.add_argument("--steps", type=int, default=20)
    r.add_argument("--out-dir", default=".")
    sub.add_parser("layers", help="the VGG16 layer names POST / accepts")
    a = ap.parse_args(argv)

    from .config import Config

    over = {k: v for k, v in (("device", a.device), ("dtype", a.dtype), ("weights", a.weights),
                              ("mode", getattr(a, "mode", None))) if v is not None}
    cfg = Config.from_env(**over)
    from .codec import ImageDecodeError
    from .engine.deconvnet import UnknownLayerError

    try:
        return {"deconv": cmd_deconv, "dream": cmd_dream, "layers": cmd_layers}[a.cmd](a, cfg)
    except (UnknownLayerError, ImageDecodeError, ValueError, OSError) as e:  # the HTTP routes' 400s
        print(f"error: {str(e).strip(chr(34))}", file=sys.stderr)
        return 2


if __name__ == "__main__":
    sys.exit(main())
