"""InceptionV3 (Keras ``keras.applications.inception_v3.InceptionV3(include_top=False)``
topology), NHWC, for DeepDream (BASELINE config 3; not part of the reference).

Every Keras ``conv2d_bn`` (conv without bias -> BatchNorm(scale=False) -> ReLU) is one ConvUnit
with the BN folded into the conv kernel and bias (``fold_bn``). Branch outputs are concatenated
along channels in Keras order, and the ``mixedN`` names match Keras so DeepDream's layer
settings (mixed2..mixed5) address the same tensors. ``forward(x, outputs)`` stops at the
deepest requested layer (DeepDream's loss never reaches mixed6..mixed10).
"""
from __future__ import annotations

import math
from typing import Dict, Iterable, List

import torch

from .. import knobs
from ..ops.autograd import ConvUnit, avg_pool, cat_channels, max_pool
from ..ops.inception import InceptionBlock

# DV_INCEPTION_FUSED=0: per-op autograd units + torch.cat instead of the one-node blocks of
# ops/inception.py (the oracle-shaped path; GPU tests compare the two). Removed after measuring:
# branches on side streams (no gain in a graph, profiles/kstats_c3_r2_branch_streams.txt) and
# conv2d_4/5 padded to 96 channels (neutral, profiles/dream_c3_r2_padstem.txt).
FUSED_BLOCKS = knobs.ablation("DV_INCEPTION_FUSED", "1") != "0"

MIXED = [f"mixed{i}" for i in range(11)]


def fold_bn(w_oihw, gamma, beta, mean, var, eps: float = 1e-3, bias=None):
    """Fold an inference BatchNorm into the preceding conv (Keras BN eps = 1e-3)."""
    scale = (gamma if gamma is not None else torch.ones_like(var)) / torch.sqrt(var + eps)
    w = w_oihw * scale.view(-1, 1, 1, 1)
    b = beta - mean * scale + (0 if bias is None else bias * scale)
    return w, b


class InceptionV3:
    def __init__(self, seed: int = 0):
        self.g = torch.Generator().manual_seed(seed)
        self.units: Dict[str, ConvUnit] = {}
        self._n = 0
        self.device = torch.device("cpu")
        self._define()
        self.iblocks = [InceptionBlock(name, order, br, self.units) for name, order, br in self.blocks]

    # ----------------------------------------------------------------- definition
    def _conv(self, cin, cout, kh, kw, stride=1, padding="same") -> str:
        self._n += 1
        name = f"conv2d_{self._n}"
        std = math.sqrt(2.0 / (cin * kh * kw))
        w = torch.randn(cout, cin, kh, kw, generator=self.g) * std
        b = torch.randn(cout, generator=self.g) * 0.05
        pad = ((kh - 1) // 2, (kw - 1) // 2) if padding == "same" else (0, 0)
        self.units[name] = ConvUnit(name, w, b, stride, pad, relu=True)
        return name

    def _define(self):
        c = self._conv
        self.stem = [c(3, 32, 3, 3, 2, "valid"), c(32, 32, 3, 3, 1, "valid"), c(32, 64, 3, 3), "pool",
                     c(64, 80, 1, 1, 1, "valid"), c(80, 192, 3, 3, 1, "valid"), "pool"]
        self.blocks: List[tuple] = []
        cin = 192
        for i, pool_ch in enumerate((32, 64, 64)):  # mixed0-2 (35x35)
            br = {"b1": [c(cin, 64, 1, 1)], "b5": [c(cin, 48, 1, 1), c(48, 64, 5, 5)],
                  "b3": [c(cin, 64, 1, 1), c(64, 96, 3, 3), c(96, 96, 3, 3)], "pool": ["avg", c(cin, pool_ch, 1, 1)]}
            self.blocks.append((f"mixed{i}", ["b1", "b5", "b3", "pool"], br))
            cin = 64 + 64 + 96 + pool_ch
        br = {"b3": [c(cin, 384, 3, 3, 2, "valid")],
              "b3d": [c(cin, 64, 1, 1), c(64, 96, 3, 3), c(96, 96, 3, 3, 2, "valid")], "pool": ["max"]}
        self.blocks.append(("mixed3", ["b3", "b3d", "pool"], br))
        cin = 384 + 96 + cin
        for i, m in zip(range(4, 8), (128, 160, 160, 192)):  # mixed4-7 (17x17)
            br = {"b1": [c(cin, 192, 1, 1)],
                  "b7": [c(cin, m, 1, 1), c(m, m, 1, 7), c(m, 192, 7, 1)],
                  "b7d": [c(cin, m, 1, 1), c(m, m, 7, 1), c(m, m, 1, 7), c(m, m, 7, 1), c(m, 192, 1, 7)],
                  "pool": ["avg", c(cin, 192, 1, 1)]}
            self.blocks.append((f"mixed{i}", ["b1", "b7", "b7d", "pool"], br))
            cin = 768
        br = {"b3": [c(cin, 192, 1, 1), c(192, 320, 3, 3, 2, "valid")],
              "b7x3": [c(cin, 192, 1, 1), c(192, 192, 1, 7), c(192, 192, 7, 1), c(192, 192, 3, 3, 2, "valid")],
              "pool": ["max"]}
        self.blocks.append(("mixed8", ["b3", "b7x3", "pool"], br))
        cin = 320 + 192 + 768
        for i in (9, 10):  # mixed9, mixed10 (8x8), with 1x3 / 3x1 splits
            br = {"b1": [c(cin, 320, 1, 1)],
                  "b3": [c(cin, 384, 1, 1), ("split", c(384, 384, 1, 3), c(384, 384, 3, 1))],
                  "b3d": [c(cin, 448, 1, 1), c(448, 384, 3, 3), ("split", c(384, 384, 1, 3), c(384, 384, 3, 1))],
                  "pool": ["avg", c(cin, 192, 1, 1)]}
            self.blocks.append((f"mixed{i}", ["b1", "b3", "b3d", "pool"], br))
            cin = 2048

    # ----------------------------------------------------------------- runtime
    def build(self, device, dtype=torch.bfloat16) -> "InceptionV3":
        """Pack weights for ``device``; ``dtype`` is the GPU storage dtype (bf16 or fp16)."""
        self.device = torch.device(device)
        self.dtype = dtype
        for u in self.units.values():
            u.build(self.device, dtype)
        for blk in self.iblocks:  # merged head GEMMs (GPU)
            blk.build(self.device, dtype)
        return self

    def num_params(self) -> int:
        """Keras parameter count."""
        return sum(u.w.numel() + u.b.numel() for u in self.units.values())

    def _branch(self, x, ops_):
        for op in ops_:
            if op == "avg":
                x = avg_pool(x, 3, 1, 1)
            elif op == "max":
                x = max_pool(x, 3, 2, 0)
            elif isinstance(op, tuple):  # ("split", a, b): concat of two convs of the same input
                x = cat_channels([self.units[op[1]](x), self.units[op[2]](x)])
            else:
                x = self.units[op](x)
        return x

    def forward(self, x: torch.Tensor, outputs: Iterable[str] = ("mixed10",), tap=None) -> Dict[str, torch.Tensor]:
        """x: [N, H, W, 8] (RGB in slots 0..2, inception preprocessing x/127.5 - 1). ``tap(name, t)``
        (optional) replaces every requested output except the deepest before deeper layers use it."""
        want = set(outputs)
        last = max(MIXED.index(o) for o in want)
        for op in self.stem:
            x = max_pool(x, 3, 2, 0) if op == "pool" else self.units[op](x)
        out = {}
        for bi, (name, order, br) in enumerate(self.blocks):
            if bi > last:
                break
            if x.is_cuda and FUSED_BLOCKS:
                x = self.iblocks[bi](x)
            else:
                x = cat_channels([self._branch(x, br[k]) for k in order])
            if name in want:
                if tap is not None and bi < last:
                    x = tap(name, x)
                out[name] = x
        return out
