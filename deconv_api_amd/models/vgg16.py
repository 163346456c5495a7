"""VGG16 (Keras ``keras.applications.vgg16.VGG16(include_top=True)`` topology, channels_last).

The reference instantiates this model with ImageNet weights at app/main.py:16-17 and walks
``model.layers`` at app/deepdream.py:401-423. Layer names, order and shapes are identical here.
Weights are kept in Keras layout on the host (conv kernel HWIO ``[3,3,Cin,Cout]``, dense kernel
``[in,out]``) so a Keras ``.h5`` imports without transposition (models/keras_import.py), and
are packed once per device into the GEMM layouts the gfx950 kernels stream (ops/conv.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from ..ops.conv import ConvWeights, deconv_weights, pad_channels_oihw

IMAGE_SIZE = 224
INPUT_CPAD = 8  # RGB padded to 8 channels so every conv sees a 16-byte channel vector


@dataclass(frozen=True)
class LayerSpec:
    name: str
    kind: str  # input | conv | pool | flatten | dense
    cin: int = 0
    cout: int = 0
    activation: str = ""  # relu | softmax (conv / dense)
    out_hw: int = 0  # spatial size of the output (conv / pool)


def vgg16_specs(width_div: int = 1, image_size: int = IMAGE_SIZE, fc: int = 4096,
                classes: int = 1000) -> List[LayerSpec]:
    """Layer list of Keras VGG16. ``width_div``/``image_size``/``fc``/``classes`` build the same
    topology at a reduced size (used by the float64 oracle tests)."""
    specs = [LayerSpec("input_1", "input", out_hw=image_size)]
    cfg = [(1, 2, 64 // width_div), (2, 2, 128 // width_div), (3, 3, 256 // width_div),
           (4, 3, 512 // width_div), (5, 3, 512 // width_div)]
    cin, hw = 3, image_size
    for b, n, c in cfg:
        for i in range(1, n + 1):
            specs.append(LayerSpec(f"block{b}_conv{i}", "conv", cin, c, "relu", hw))
            cin = c
        hw //= 2
        specs.append(LayerSpec(f"block{b}_pool", "pool", c, c, out_hw=hw))
    specs.append(LayerSpec("flatten", "flatten", cin, cin * hw * hw, out_hw=hw))
    specs.append(LayerSpec("fc1", "dense", cin * hw * hw, fc, "relu"))
    specs.append(LayerSpec("fc2", "dense", fc, fc, "relu"))
    specs.append(LayerSpec("predictions", "dense", fc, classes, "softmax"))
    return specs


VGG16_SPECS: List[LayerSpec] = vgg16_specs()
VGG16_LAYER_NAMES: List[str] = [s.name for s in VGG16_SPECS]
SPEC_BY_NAME: Dict[str, LayerSpec] = {s.name: s for s in VGG16_SPECS}


@dataclass
class ConvLayer:
    spec: LayerSpec
    fwd: ConvWeights  # up: conv + bias (+ReLU applied by the op flag)
    dec: ConvWeights  # down: flipped / transposed kernel, zero bias
    seed_wt: torch.Tensor  # [Cout, 3, 3, Cin_pad8] first-step weights (wt[f,kh,kw,ci] = W[2-kh,2-kw,ci,f])


@dataclass
class DenseLayer:
    spec: LayerSpec
    w: torch.Tensor  # [in, out]
    b: torch.Tensor  # [out] fp32
    wt: Optional[torch.Tensor] = None  # [out, in] contiguous copy for the down GEMM on device
    # GPU: the dense layer as a 1x1 conv on the MFMA kernel ([B, 1, 1, in] NHWC rows; fused bias +
    # ReLU epilogue, split-K for small batches): up = x . W + b, down = y . W^T
    up: Optional[ConvWeights] = None
    down: Optional[ConvWeights] = None


@dataclass
class VGG16:
    """Host-side Keras-layout weights: ``params[name] = (kernel, bias)`` fp32 CPU tensors."""

    params: Dict[str, Tuple[torch.Tensor, torch.Tensor]]
    specs: List[LayerSpec] = field(default_factory=lambda: list(VGG16_SPECS))

    # ---------------------------------------------------------------- construction
    @classmethod
    def random(cls, seed: int = 0, include_top: bool = True, specs: Optional[List[LayerSpec]] = None) -> "VGG16":
        """Seeded random init: He-normal kernels (keeps activation scale through 13 ReLU convs,
        so the bf16 path is exercised at realistic magnitudes) and small normal biases."""
        specs = specs or list(VGG16_SPECS)
        g = torch.Generator().manual_seed(seed)
        params = {}
        for s in specs:
            if s.kind == "conv":
                std = math.sqrt(2.0 / (9 * s.cin))
                k = torch.randn(3, 3, s.cin, s.cout, generator=g) * std
                b = torch.randn(s.cout, generator=g) * 0.05
                params[s.name] = (k, b)
            elif s.kind == "dense" and include_top:
                std = math.sqrt(2.0 / s.cin)
                if s.activation == "softmax":
                    # un-normalized caffe-mode inputs (~+-128) keep activations large through the
                    # He-scaled stack; shrink the classifier so softmax is not saturated
                    std *= 1e-3
                k = torch.randn(s.cin, s.cout, generator=g) * std
                b = torch.randn(s.cout, generator=g) * 0.05
                params[s.name] = (k, b)
        return cls(params, list(specs))

    @classmethod
    def from_state_dict(cls, sd: Dict[str, torch.Tensor], specs: Optional[List[LayerSpec]] = None) -> "VGG16":
        specs = specs or list(VGG16_SPECS)
        params = {}
        for s in specs:
            if s.kind in ("conv", "dense") and f"{s.name}.kernel" in sd:
                params[s.name] = (sd[f"{s.name}.kernel"].float(), sd[f"{s.name}.bias"].float())
        return cls(params, list(specs))

    def state_dict(self) -> Dict[str, torch.Tensor]:
        sd = {}
        for name, (k, b) in self.params.items():
            sd[f"{name}.kernel"] = k
            sd[f"{name}.bias"] = b
        return sd

    def save(self, path: str) -> None:
        from safetensors.torch import save_file

        save_file({k: v.contiguous() for k, v in self.state_dict().items()}, path)

    @classmethod
    def load(cls, path: str) -> "VGG16":
        if path.endswith(".safetensors"):
            from safetensors.torch import load_file

            return cls.from_state_dict(load_file(path))
        if path.endswith((".h5", ".hdf5")):  # Keras weights (app/main.py:17's ImageNet file)
            from .keras_import import load_keras_vgg16_h5

            return load_keras_vgg16_h5(path)
        return cls.from_state_dict(torch.load(path, map_location="cpu", weights_only=True))

    @property
    def image_size(self) -> int:
        return self.specs[0].out_hw

    @property
    def has_top(self) -> bool:
        return "fc1" in self.params

    def num_params(self) -> int:
        return sum(k.numel() + b.numel() for k, b in self.params.values())

    # ---------------------------------------------------------------- device packing
    def build(self, device="cpu", dtype=torch.bfloat16) -> "VGG16Runtime":
        return VGG16Runtime(self, torch.device(device), dtype)


class VGG16Runtime:
    """Weights packed for one device: per conv the forward GEMM matrix, the deconv GEMM matrix
    and the seeded-first-step weights; per dense layer 16-bit (device) kernels. ``dtype``: the
    device storage dtype, bf16 or fp16 (Config.dtype); CPU weights stay fp32."""

    def __init__(self, model: VGG16, device: torch.device, dtype: torch.dtype):
        self.model = model
        self.device = device
        self.dtype = dtype
        self.specs = model.specs
        self.convs: Dict[str, ConvLayer] = {}
        self.dense: Dict[str, DenseLayer] = {}
        for s in self.specs:
            if s.kind == "conv":
                k, b = model.params[s.name]
                w_oihw = pad_channels_oihw(k.permute(3, 2, 0, 1).contiguous())  # [Cout, Cin8, 3, 3]
                fwd = ConvWeights(w_oihw, b.clone(), "fwd")
                dec = deconv_weights(ConvWeights(k.permute(3, 2, 0, 1).contiguous(), None, "fwd"))
                cin8 = w_oihw.shape[1]
                seed = torch.zeros(s.cout, 3, 3, cin8)
                seed[..., : s.cin] = k.flip(0, 1).permute(3, 0, 1, 2)  # [f, kh, kw, ci] = W[2-kh, 2-kw, ci, f]
                self.convs[s.name] = ConvLayer(s, fwd.to_device(device, dtype), dec.to_device(device, dtype),
                                               seed.to(device=device, dtype=dtype).contiguous())
            elif s.kind == "dense" and s.name in model.params:
                k, b = model.params[s.name]
                wdt = dtype if device.type == "cuda" else torch.float32
                w = k.to(device=device, dtype=wdt).contiguous()
                dl = DenseLayer(s, w, b.to(device=device, dtype=torch.float32),
                                k.t().contiguous().to(device=device, dtype=wdt))
                kin, kout = k.shape  # Keras kernel [in, out]
                if device.type == "cuda" and kin % 8 == 0:  # the kernel's K gather is 8-channel granular
                    dl.up = ConvWeights(k.t().reshape(kout, kin, 1, 1).contiguous(), b.clone(), "fwd").to_device(
                        device, dtype)
                if device.type == "cuda" and kout % 8 == 0:
                    dl.down = ConvWeights(k.reshape(kin, kout, 1, 1).contiguous(), None, "fwd").to_device(device, dtype)
                self.dense[s.name] = dl

    def layer_index(self, name: str) -> int:
        for i, s in enumerate(self.specs):
            if s.name == name:
                return i
        raise KeyError(name)
