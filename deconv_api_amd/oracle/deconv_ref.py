"""Float64 CPU oracle of the reference deconvnet (ground truth for every other path).

Written from the behaviour of app/deepdream.py, structured like it: a stack
of D-layers with ``up``/``down`` built while walking the model's layers, a forward chain, then
for each visualized layer and each selected filter a ``down`` chain to the input.

  DInput      identity both ways                                  (app/deepdream.py:13-50)
  DConv       up: ReLU(conv 'same' + b); down: ReLU(conv 'same' with
              flip(W) in/out-swapped, zero bias)                     (:53-111)
  DPooling    up: 2x2 max + one-hot first-max switch; down: the
              pooled signal upsampled and masked by the switch       (:114-209)
  DActivation same activation up and down (ReLU / softmax)           (:212-261)
  DDense      up: act(xW + b); down: y W^T (linear, zero bias)        (:264-321)
  DFlatten    up: reshape (h, w, c order); down: reshape back        (:324-366)
  find_top_filters: sums over every axis but the last (batch too), keep > 0, stable sort
              descending, first ``top``                              (:369-380)
Tensors are NHWC float64; the model is a ``models.vgg16.VGG16`` (Keras-layout weights).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch
import torch.nn.functional as F

DT = torch.float64


class DInput:
    def __init__(self, name):
        self.name = name

    def up(self, x):
        self.up_data = x
        return x

    def down(self, y):
        self.down_data = y
        return y


class DConv:
    def __init__(self, name, kernel, bias):
        self.name = name
        self.w = kernel.to(DT).permute(3, 2, 0, 1)  # OIHW
        self.b = bias.to(DT)
        # down kernel: Keras W.transpose(0,1,3,2)[::-1, ::-1] as a conv -> OIHW flip+swap
        self.wd = self.w.flip(2, 3).transpose(0, 1).contiguous()

    def up(self, x):
        y = F.conv2d(x.permute(0, 3, 1, 2), self.w, self.b, padding=1).relu()
        self.up_data = y.permute(0, 2, 3, 1)
        return self.up_data

    def down(self, y):
        x = F.conv2d(y.permute(0, 3, 1, 2), self.wd, None, padding=1).relu()
        self.down_data = x.permute(0, 2, 3, 1)
        return self.down_data


class DPooling:
    def __init__(self, name):
        self.name = name

    def up(self, x):
        N, H, W, C = x.shape
        win = x.reshape(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, C, 4)
        m = win.max(dim=-1).values
        first = (win == m.unsqueeze(-1)).to(torch.int64).argmax(dim=-1)  # first max, row-major
        onehot = F.one_hot(first, 4).to(DT)  # [N, PH, PW, C, 4]
        self.switch = onehot.reshape(N, H // 2, W // 2, C, 2, 2).permute(0, 1, 4, 2, 5, 3).reshape(N, H, W, C)
        self.up_data = m
        return m

    def down(self, y):
        up = y.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)  # np.kron(y, ones(2,2))
        self.down_data = up * self.switch
        return self.down_data


class DActivation:
    def __init__(self, name, kind):
        self.name = name
        self.kind = kind

    def _f(self, x):
        return x.relu() if self.kind == "relu" else torch.softmax(x, dim=-1)

    def up(self, x):
        self.up_data = self._f(x)
        return self.up_data

    def down(self, y):
        self.down_data = self._f(y)
        return self.down_data


class DDense:
    def __init__(self, name, kernel, bias, act):
        self.name = name
        self.w = kernel.to(DT)
        self.b = bias.to(DT)
        self.act = act

    def up(self, x):
        y = x @ self.w + self.b
        self.up_data = y.relu() if self.act == "relu" else torch.softmax(y, dim=-1)
        return self.up_data

    def down(self, y):
        self.down_data = y @ self.w.t()
        return self.down_data


class DFlatten:
    def __init__(self, name, shape):
        self.name = name
        self.shape = shape

    def up(self, x):
        self.up_data = x.reshape(x.shape[0], -1)
        return self.up_data

    def down(self, y):
        self.down_data = y.reshape(y.shape[0], *self.shape)
        return self.down_data


def build_stack(model, layer_name: str):
    """D-layer stack up to and including ``layer_name`` (append, then break)."""
    stack = []
    prev_hw, prev_c = None, None
    for s in model.specs:
        if s.kind == "input":
            stack.append(DInput(s.name))
        elif s.kind == "conv":
            k, b = model.params[s.name]
            stack.append(DConv(s.name, k, b))
            stack.append(DActivation(s.name + "_activation", "relu"))
            prev_c = s.cout
        elif s.kind == "pool":
            stack.append(DPooling(s.name))
            prev_hw = s.out_hw
        elif s.kind == "flatten":
            stack.append(DFlatten(s.name, (prev_hw, prev_hw, prev_c)))
        elif s.kind == "dense":
            k, b = model.params[s.name]
            stack.append(DDense(s.name, k, b, s.activation))
            stack.append(DActivation(s.name + "_activation", s.activation))
        if s.name == layer_name:
            break
    return stack


def find_top_filters(output: torch.Tensor, top: int = 8):
    sums = []
    for f in range(output.shape[-1]):
        v = float(output[..., f].sum())
        if v > 0:
            sums.append((f, v))
    sums.sort(key=lambda t: t[1], reverse=True)  # Python sort is stable
    return sums[:top]


def visualize_all_layers(model, data, layer_name: str = "predictions", visualize_mode: str = "all",
                         top: int = 8, only_target: bool = False) -> Dict[str, List[np.ndarray]]:
    """data: preprocessed NHWC [N, H, W, 3]. Returns {layer: [squeezed recon float64 ndarray]}."""
    if visualize_mode not in ("all", "max"):
        raise ValueError("Illegal visualize mode")
    x = torch.as_tensor(np.asarray(data), dtype=DT)
    stack = build_stack(model, layer_name)
    stack[0].up(x)
    for i in range(1, len(stack)):
        stack[i].up(stack[i - 1].up_data)
    names = {s.name for s in model.specs}
    idxs = [i for i, d in enumerate(stack) if d.name in names]
    idxs.reverse()
    idxs.pop()  # the input layer
    if only_target:
        idxs = [i for i in idxs if stack[i].name == layer_name]
    out: Dict[str, List[np.ndarray]] = {}
    for i in idxs:
        output = stack[i].up_data
        recs = []
        for f, _ in find_top_filters(output, top):
            fmap = output[..., f]
            if visualize_mode == "max":
                fmap = fmap * (fmap == fmap.max())
            seed = torch.zeros_like(output)
            seed[..., f] = fmap
            stack[i].down(seed)
            for j in range(i - 1, -1, -1):
                stack[j].down(stack[j + 1].down_data)
            recs.append(stack[0].down_data.squeeze().numpy())
        out[stack[i].name] = recs
    return out


def deprocess_image(x: np.ndarray) -> np.ndarray:
    """Keras filter-visualization post-processing in float32 (app/deepdream.py:483-498)."""
    x = np.array(x, dtype=np.float32, copy=True)
    x -= x.mean()
    x /= (x.std() + 1e-7)
    x *= 0.1
    x += 0.5
    x = np.clip(x, 0, 1)
    x *= 255
    return np.clip(x, 0, 255).astype("uint8")


def mosaic(recs: List[np.ndarray]) -> np.ndarray:
    """2x2 mosaic of the first four reconstructions (app/main.py:67-69)."""
    top = np.concatenate((recs[0], recs[1]), axis=1)
    bottom = np.concatenate((recs[2], recs[3]), axis=1)
    return np.concatenate((top, bottom), axis=0)
