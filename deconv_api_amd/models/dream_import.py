"""Keras -> framework weight import for the DeepDream models (InceptionV3, ResNet-50).

Not in the reference (its DeepDream networks are an extension); this gives them the
same import path VGG16 has (models/keras_import.py), so DeepDream can run on the ImageNet weights
of ``keras.applications.inception_v3.InceptionV3`` / ``resnet50.ResNet50`` instead of seeded
random init.

Keras HDF5 layouts handled (duck-typed over the h5py interface, so testable without h5py):

* InceptionV3: every ``conv2d_bn`` is a bias-free ``conv2d[_N]`` (kernel HWIO) followed by
  ``batch_normalization[_N]`` with ``scale=False`` (beta, moving_mean, moving_variance;
  eps 1e-3). Keras numbers the layers in creation order, which is the order our model defines its
  ``conv2d_{i}`` units (models/inception_v3.py), so the i-th conv / BN of the file (sorted by
  numeric suffix; no suffix = first, as TF2 names it) maps to unit ``conv2d_{i+1}``.
* ResNet-50 (Keras >= 2.3 names): ``convS_blockB_K_conv`` (kernel, bias) + ``..._bn`` (gamma,
  beta, moving_mean, moving_variance; eps 1.001e-5), stem ``conv1_conv`` / ``conv1_bn``: the unit
  names of models/resnet50.py.

Each BN is folded into its conv (``fold_bn``) and stored as the unit's OIHW kernel and bias. The
folded state saves/loads as safetensors (``{unit}.w``, ``{unit}.b``):

    python -m deconv_api_amd.models.dream_import inception_v3 in.h5 out.safetensors
"""
from __future__ import annotations

import re
import sys
from typing import Dict, List, Mapping

import numpy as np
import torch

from .inception_v3 import fold_bn

INCEPTION_BN_EPS = 1e-3
RESNET_BN_EPS = 1.001e-5


def _names(attrs, key) -> List[str]:
    v = attrs.get(key) if hasattr(attrs, "get") else attrs[key]
    return [n.decode("utf8") if isinstance(n, bytes) else str(n) for n in v]


def layer_names(f: Mapping) -> List[str]:
    attrs = getattr(f, "attrs", {})
    return _names(attrs, "layer_names") if "layer_names" in attrs else list(f.keys())


def layer_arrays(f: Mapping, lname: str) -> List[np.ndarray]:
    """The weight arrays of one Keras layer group, in its ``weight_names`` order."""
    g = f[lname]
    out = []
    for n in _names(g.attrs, "weight_names"):
        node = g
        for part in n.split("/"):
            if part in node:
                node = node[part]
            elif f"{lname}/{part}" in node:
                node = node[f"{lname}/{part}"]
        out.append(np.asarray(node, dtype=np.float32))
    return out


def _ordered(names: List[str], prefix: str) -> List[str]:
    pat = re.compile(rf"^{prefix}(?:_(\d+))?$")
    hits = [(int(m.group(1) or 0), n) for n in names for m in [pat.match(n)] if m]
    return [n for _, n in sorted(hits)]


def _hwio_to_oihw(k: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(k.transpose(3, 2, 0, 1)))


def _check(unit, w: torch.Tensor, src: str) -> None:
    if tuple(w.shape) != tuple(unit.w.shape):
        raise ValueError(f"{src} -> {unit.name}: kernel {tuple(w.shape)} does not match {tuple(unit.w.shape)}")


def inception_state_from_h5_like(f: Mapping, model) -> Dict[str, torch.Tensor]:
    names = layer_names(f)
    convs, bns = _ordered(names, "conv2d"), _ordered(names, "batch_normalization")
    units = [model.units[f"conv2d_{i + 1}"] for i in range(len(model.units))]
    if len(convs) != len(units) or len(bns) != len(units):
        raise ValueError(f"expected {len(units)} conv2d / batch_normalization layers, found {len(convs)} / {len(bns)}")
    sd: Dict[str, torch.Tensor] = {}
    for u, cn, bn in zip(units, convs, bns):
        ka = layer_arrays(f, cn)
        w = _hwio_to_oihw(ka[0])
        _check(u, w, cn)
        ba = [torch.from_numpy(a) for a in layer_arrays(f, bn)]
        if len(ba) == 3:  # scale=False: beta, moving_mean, moving_variance
            gamma, (beta, mean, var) = None, ba
        elif len(ba) == 4:
            gamma, beta, mean, var = ba
        else:
            raise ValueError(f"{bn}: expected 3 or 4 BatchNorm arrays, got {len(ba)}")
        bias = torch.from_numpy(ka[1]) if len(ka) > 1 else None
        sd[f"{u.name}.w"], sd[f"{u.name}.b"] = fold_bn(w, gamma, beta, mean, var, INCEPTION_BN_EPS, bias)
    return sd


def resnet50_state_from_h5_like(f: Mapping, model) -> Dict[str, torch.Tensor]:
    names = set(layer_names(f))
    sd: Dict[str, torch.Tensor] = {}
    for name, u in model.units.items():
        bn = name[: -len("_conv")] + "_bn"
        if name not in names or bn not in names:
            raise ValueError(f"weights file lacks {name} / {bn}")
        ka = layer_arrays(f, name)
        w = _hwio_to_oihw(ka[0])
        _check(u, w, name)
        ba = [torch.from_numpy(a) for a in layer_arrays(f, bn)]
        if len(ba) != 4:
            raise ValueError(f"{bn}: expected gamma, beta, moving_mean, moving_variance")
        bias = torch.from_numpy(ka[1]) if len(ka) > 1 else None
        sd[f"{name}.w"], sd[f"{name}.b"] = fold_bn(w, *ba, RESNET_BN_EPS, bias)
    return sd


def state_from_h5_like(f: Mapping, model) -> Dict[str, torch.Tensor]:
    from .inception_v3 import InceptionV3

    if isinstance(model, InceptionV3):
        return inception_state_from_h5_like(f, model)
    return resnet50_state_from_h5_like(f, model)


def apply_state(model, sd: Dict[str, torch.Tensor]):
    """Install folded kernels/biases into an UNBUILT model (call ``model.build`` afterwards)."""
    missing = [n for n in model.units if f"{n}.w" not in sd]
    if missing:
        raise ValueError(f"state lacks units: {missing[:5]}{'...' if len(missing) > 5 else ''}")
    for n, u in model.units.items():
        w, b = sd[f"{n}.w"].float(), sd[f"{n}.b"].float()
        _check(u, w, n)
        if tuple(b.shape) != (u.cout,):
            raise ValueError(f"{n}: bias {tuple(b.shape)} != ({u.cout},)")
        u.w, u.b = w.contiguous(), b.contiguous()
    return model


def state_dict(model) -> Dict[str, torch.Tensor]:
    sd = {}
    for n, u in model.units.items():
        sd[f"{n}.w"], sd[f"{n}.b"] = u.w.contiguous(), u.b.contiguous()
    return sd


def save(model, path: str) -> None:
    from safetensors.torch import save_file

    save_file(state_dict(model), path)


def load_weights(model, path: str):
    """``path``: folded ``.safetensors`` (this module's format) or a Keras ``.h5`` (h5py when importable,
    else the dependency-free ``models/h5lite.py`` reader)."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file

        return apply_state(model, load_file(path))
    from .h5lite import open_h5

    with open_h5(path) as f:
        return apply_state(model, state_from_h5_like(f, model))


def new_model(name: str, seed: int = 0):
    if name == "inception_v3":
        from .inception_v3 import InceptionV3

        return InceptionV3(seed)
    if name == "resnet50":
        from .resnet50 import ResNet50

        return ResNet50(seed)
    raise ValueError("model must be inception_v3 or resnet50")


def main(argv=None):
    argv = argv or sys.argv[1:]
    if len(argv) != 3:
        print("usage: python -m deconv_api_amd.models.dream_import {inception_v3|resnet50} in.h5 out.safetensors")
        return 2
    m = load_weights(new_model(argv[0]), argv[1])
    save(m, argv[2])
    print(f"wrote {argv[2]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
