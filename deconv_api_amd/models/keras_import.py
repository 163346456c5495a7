"""Keras -> PyTorch weight import for the reference's model.

The reference loads ``keras.applications.vgg16.VGG16(weights='imagenet')`` (app/main.py:17),
i.e. ``vgg16_weights_tf_dim_ordering_tf_kernels.h5``: one HDF5 group per layer whose
``weight_names`` attribute lists ``<layer>/kernel:0`` and ``<layer>/bias:0``. Keras layouts are
kept as-is (conv kernels HWIO, dense kernels [in, out]; fc1's rows are already in the (h, w, c)
order our NHWC flatten produces), so the import is a pure name mapping; the device packing in
models/vgg16.py does every transpose.

``h5py`` is not installed in this environment; the reader is duck-typed over any mapping with the
h5py interface (``f[name]``, ``.attrs``, ``np.asarray(dataset)``), and ``load_keras_vgg16_h5``
opens the file with h5py when it is importable and with the framework's own dependency-free HDF5
reader (``models/h5lite.py``) otherwise, so ``VGG16.load("x.h5")`` works in the shipped container.
``python -m deconv_api_amd.models.keras_import in.h5 out.safetensors`` converts once.
"""
from __future__ import annotations

import sys
from typing import Dict, Mapping

import numpy as np
import torch

from .vgg16 import VGG16, VGG16_SPECS


def _names(attrs, key):
    v = attrs.get(key) if hasattr(attrs, "get") else attrs[key]
    return [n.decode("utf8") if isinstance(n, bytes) else str(n) for n in v]


def keras_state_from_h5_like(f: Mapping) -> Dict[str, torch.Tensor]:
    sd: Dict[str, torch.Tensor] = {}
    layer_names = _names(f.attrs, "layer_names") if "layer_names" in getattr(f, "attrs", {}) else list(f.keys())
    wanted = {s.name: s for s in VGG16_SPECS if s.kind in ("conv", "dense")}
    for lname in layer_names:
        if lname not in wanted:
            continue
        g = f[lname]
        wn = _names(g.attrs, "weight_names")
        if len(wn) != 2:
            raise ValueError(f"{lname}: expected kernel and bias, got {wn}")
        arrs = []
        for n in wn:
            node = g
            for part in n.split("/"):
                if part in node:
                    node = node[part]
                elif f"{lname}/{part}" in node:
                    node = node[f"{lname}/{part}"]
            arrs.append(np.asarray(node, dtype=np.float32))
        k, b = arrs
        s = wanted[lname]
        exp_k = (3, 3, s.cin, s.cout) if s.kind == "conv" else (s.cin, s.cout)
        if tuple(k.shape) != exp_k or tuple(b.shape) != (s.cout,):
            raise ValueError(f"{lname}: kernel {k.shape} / bias {b.shape} do not match VGG16 {exp_k}")
        sd[f"{lname}.kernel"] = torch.from_numpy(k)
        sd[f"{lname}.bias"] = torch.from_numpy(b)
    missing = [n for n, s in wanted.items() if f"{n}.kernel" not in sd and s.kind == "conv"]
    if missing:
        raise ValueError(f"weights file lacks conv layers: {missing}")
    return sd


def load_keras_vgg16_h5(path: str) -> VGG16:
    from .h5lite import open_h5

    with open_h5(path) as f:
        sd = keras_state_from_h5_like(f)
    return VGG16.from_state_dict(sd)


def main(argv=None):
    argv = argv or sys.argv[1:]
    if len(argv) != 2:
        print("usage: python -m deconv_api_amd.models.keras_import in.h5 out.safetensors")
        return 2
    load_keras_vgg16_h5(argv[0]).save(argv[1])
    print(f"wrote {argv[1]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
