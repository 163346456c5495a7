"""ResNet-50 (Keras ``keras.applications.resnet50.ResNet50(include_top=False)`` topology), NHWC,
BatchNorm folded into conv bias, for DeepDream at 1024x1024 (BASELINE config 5; not part of the
reference). Block output names follow Keras >= 2.3 (``conv{stage}_block{i}_out``).

Bottleneck block: 1x1 (stride s) -> 3x3 -> 1x1 (no ReLU) + shortcut (1x1 stride s projection in
the first block of a stage), then ReLU(sum). The stem's ZeroPadding(3) + 7x7/2 'valid' conv is a
7x7/2 conv with pad 3; ZeroPadding(1) + 3x3/2 max-pool equals a padded max-pool on the
non-negative post-ReLU map.
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List

import torch

from ..ops.autograd import ConvUnit, bottleneck, max_pool

STAGES = [(2, 3, 64, 1), (3, 4, 128, 2), (4, 6, 256, 2), (5, 3, 512, 2)]  # (stage, blocks, width, stride)


class ResNet50:
    def __init__(self, seed: int = 0):
        self.g = torch.Generator().manual_seed(seed)
        self.units: Dict[str, ConvUnit] = {}
        self.device = torch.device("cpu")
        self._conv("conv1_conv", 3, 64, 7, 2, 3, relu=True)
        self.blocks: List[tuple] = []
        cin = 64
        for stage, nblocks, w, stride in STAGES:
            for b in range(1, nblocks + 1):
                s = stride if b == 1 else 1
                pre = f"conv{stage}_block{b}"
                short = None
                if b == 1:
                    short = self._conv(f"{pre}_0_conv", cin, 4 * w, 1, s, 0, relu=False, gain=0.5)
                c1 = self._conv(f"{pre}_1_conv", cin, w, 1, s, 0)
                c2 = self._conv(f"{pre}_2_conv", w, w, 3, 1, 1)
                c3 = self._conv(f"{pre}_3_conv", w, 4 * w, 1, 1, 0, relu=False, gain=0.5)
                self.blocks.append((f"{pre}_out", short, (c1, c2, c3)))
                cin = 4 * w

    def _conv(self, name, cin, cout, k, stride, pad, relu=True, gain=1.0) -> str:
        std = gain * math.sqrt(2.0 / (cin * k * k))
        w = torch.randn(cout, cin, k, k, generator=self.g) * std
        b = torch.randn(cout, generator=self.g) * 0.02
        self.units[name] = ConvUnit(name, w, b, stride, (pad, pad), relu=relu)
        return name

    @property
    def block_names(self) -> List[str]:
        return [b[0] for b in self.blocks]

    def build(self, device, dtype=torch.bfloat16) -> "ResNet50":
        """Pack weights for ``device``; ``dtype`` is the GPU storage dtype (bf16 or fp16)."""
        self.device = torch.device(device)
        self.dtype = dtype
        for u in self.units.values():
            u.build(self.device, dtype)
        return self

    def num_params(self) -> int:
        return sum(u.w.numel() + u.b.numel() for u in self.units.values())

    def forward(self, x: torch.Tensor, outputs: Iterable[str] = ("conv5_block3_out",),
                tap=None) -> Dict[str, torch.Tensor]:
        """``tap(name, t)`` (optional) replaces every requested output except the deepest before
        deeper blocks use it (the DeepDream loss taps)."""
        want = set(outputs)
        names = self.block_names
        last = max(names.index(o) for o in want)
        x = self.units["conv1_conv"](x)
        x = max_pool(x, 3, 2, 1)
        out = {}
        for i, (name, short, (c1, c2, c3)) in enumerate(self.blocks):
            if i > last:
                break
            u = self.units
            # GPU: one autograd node per block (residual add + ReLU in the conv3 epilogue, no
            # elementwise kernels in the backward; see ops.autograd._BottleneckFn)
            x = bottleneck(x, u[c1], u[c2], u[c3], u[short] if short is not None else None)
            if name in want:
                if tap is not None and i < last:
                    x = tap(name, x)
                out[name] = x
        return out
