"""Differentiable conv / pool units for DeepDream (input-gradient only: weights are frozen, so
no weight-gradient kernels exist or are needed).

On GPU every unit is a torch.autograd.Function whose forward and backward are HIP kernels:
  conv (+folded-BN bias, +ReLU)  fwd: MFMA implicit-GEMM conv, ReLU in the epilogue
                                 bwd: dgrad = conv over dy with the flipped/transposed kernel
                                      (stride 1) or the transposed-gather kernel (stride > 1),
                                      ReLU'(y) applied as a mask in the A-operand prologue
  max/avg pool k x k             fwd/bwd: csrc/pool.hip (argmax bytes, gather-form backward)
On CPU the same units are plain torch functional ops (autograd), which doubles as the oracle.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from . import native
from .conv import ConvWeights, conv2d, pad_channels_oihw, transpose_subpixel

# DV_SUBPIXEL=0 falls back to the direct transposed gather for strided dgrads (A/B testing)
SUBPIXEL = os.environ.get("DV_SUBPIXEL", "1") != "0"


class ConvUnit:
    """conv KHxKW / stride / symmetric pad (+ bias) (+ ReLU); OIHW fp32 weights on the host."""

    def __init__(self, name: str, w_oihw: torch.Tensor, bias: Optional[torch.Tensor], stride: int = 1,
                 pad: Tuple[int, int] = (0, 0), relu: bool = True):
        self.name = name
        self.w = w_oihw.float()
        self.b = None if bias is None else bias.float()
        self.stride = stride
        self.pad = tuple(pad)
        self.relu = relu
        self.device = torch.device("cpu")

    @property
    def cin(self):
        return self.w.shape[1]

    @property
    def cout(self):
        return self.w.shape[0]

    def build(self, device, dtype=torch.bfloat16) -> "ConvUnit":
        """``dtype``: 16-bit storage/MFMA dtype of the GPU path (bf16, or fp16 for config 5)."""
        self.device = torch.device(device)
        self.dtype = dtype
        w8 = pad_channels_oihw(self.w)
        self.w_dev = w8.to(self.device)
        self.b_dev = None if self.b is None else self.b.to(self.device)
        if self.device.type == "cuda":
            self.fwd = ConvWeights(w8, self.b, "fwd").to_device(self.device, dtype)
            kh, kw = self.w.shape[2:]
            if self.stride == 1:
                wd = pad_channels_oihw(w8.flip(2, 3).transpose(0, 1).contiguous())
                self.bwd = ConvWeights(wd, None, "fwd").to_device(self.device, dtype)
                self.bwd_pad = (kh - 1 - self.pad[0], kw - 1 - self.pad[1])
            else:
                self.bwd = ConvWeights(w8, None, "transpose").to_device(self.device, dtype)
                # sub-pixel classes: s^2 stride-1 convs instead of one s^2-times-wasteful gather
                self.bwd_sub = []
                for rh, rw, ws, pd in transpose_subpixel(w8, self.stride, self.pad):
                    cw = None if ws is None else ConvWeights(pad_channels_oihw(ws), None, "fwd").to_device(
                        self.device, dtype)
                    self.bwd_sub.append((rh, rw, cw, pd))
        return self

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return _ConvFn.apply(x, self)
        y = F.conv2d(x.permute(0, 3, 1, 2), self.w_dev[:, : x.shape[3]] if x.shape[3] < self.w_dev.shape[1]
                     else self.w_dev, self.b_dev, stride=self.stride, padding=self.pad).permute(0, 2, 3, 1)
        return y.relu() if self.relu else y


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, unit: ConvUnit):
        y = conv2d(x, unit.fwd, stride=unit.stride, pad=unit.pad, relu=unit.relu)
        ctx.unit = unit
        ctx.in_hw = (x.shape[1], x.shape[2])
        if unit.relu:
            ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        unit: ConvUnit = ctx.unit
        mask = ctx.saved_tensors[0] if unit.relu else None
        gy = gy.contiguous() if gy.stride(-1) != 1 else gy
        if mask is not None and gy.stride() != mask.stride():
            gy = gy.contiguous()
        if unit.stride == 1:
            gx = conv2d(gy, unit.bwd, stride=1, pad=unit.bwd_pad, relu=False, mask=mask, use_bias=False)
        elif SUBPIXEL:
            gx = _subpixel_dgrad(gy, mask, unit, ctx.in_hw)
        else:
            gx = conv2d(gy, unit.bwd, stride=unit.stride, pad=unit.pad, relu=False, mask=mask, in_mode="transpose",
                        out_hw=ctx.in_hw, use_bias=False)
        return gx, None


def _subpixel_dgrad(gy, mask, unit: ConvUnit, in_hw):
    """dx of a strided conv as s^2 stride-1 convs (ops.conv.transpose_subpixel), each written to its
    parity class of dx."""
    s = unit.stride
    H, W = in_hw
    N = gy.shape[0]
    C = unit.fwd.cin
    gx = torch.empty(N, H, W, C, dtype=gy.dtype, device=gy.device)
    for rh, rw, cw, pd in unit.bwd_sub:
        hc, wc = len(range(rh, H, s)), len(range(rw, W, s))
        if hc == 0 or wc == 0:
            continue
        if cw is None:
            gx[:, rh::s, rw::s] = 0
            continue
        part = conv2d(gy, cw, stride=1, pad=pd, relu=False, mask=mask, out_hw=(hc, wc), use_bias=False)
        gx[:, rh::s, rw::s] = part[..., :C]
    return gx


def _pool_out(L, k, s, p):
    return (L + 2 * p - k) // s + 1


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, H, W, C = x.shape
        OH, OW = _pool_out(H, k, s, p), _pool_out(W, k, s, p)
        x = x.contiguous()
        y = torch.empty(N, OH, OW, C, dtype=x.dtype, device=x.device)
        idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=x.device)
        native.lib().pool(x, y, idx, 0, 0, [N, H, W, C, OH, OW, k, s, p])
        ctx.save_for_backward(idx)
        ctx.geom = [N, H, W, C, OH, OW, k, s, p]
        return y

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        g = ctx.geom
        gx = torch.empty(g[0], g[1], g[2], g[3], dtype=gy.dtype, device=gy.device)
        native.lib().pool(gy.contiguous(), gx, idx, 0, 1, g)
        return gx, None, None, None


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, H, W, C = x.shape
        OH, OW = _pool_out(H, k, s, p), _pool_out(W, k, s, p)
        y = torch.empty(N, OH, OW, C, dtype=x.dtype, device=x.device)
        native.lib().pool(x.contiguous(), y, None, 1, 0, [N, H, W, C, OH, OW, k, s, p])
        ctx.geom = [N, H, W, C, OH, OW, k, s, p]
        return y

    @staticmethod
    def backward(ctx, gy):
        g = ctx.geom
        gx = torch.empty(g[0], g[1], g[2], g[3], dtype=gy.dtype, device=gy.device)
        native.lib().pool(gy.contiguous(), gx, None, 1, 1, g)
        return gx, None, None, None


def max_pool(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    if x.is_cuda:
        return _MaxPoolFn.apply(x, k, s, p)
    return F.max_pool2d(x.permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1)


def avg_pool(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    if x.is_cuda:
        return _AvgPoolFn.apply(x, k, s, p)
    return F.avg_pool2d(x.permute(0, 3, 1, 2), k, s, p, count_include_pad=False).permute(0, 2, 3, 1)


class _ConvResReluFn(torch.autograd.Function):
    """y = ReLU(conv(x) + bias + sc): the ResNet block tail in one kernel (residual add and ReLU in
    the conv epilogue). Backward: gm = gy * (y > 0) is materialized once (it is also the shortcut's
    gradient), then the conv's dgrad runs on it without a mask."""

    @staticmethod
    def forward(ctx, x, sc, unit: ConvUnit):
        assert not unit.relu and unit.stride == 1, "conv_res_relu: the unit must be a linear stride-1 conv"
        y = conv2d(x, unit.fwd, stride=1, pad=unit.pad, relu=True, res=sc.contiguous())
        ctx.unit = unit
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        unit: ConvUnit = ctx.unit
        gm = torch.ops.aten.threshold_backward(gy.contiguous(), y, 0)
        gx = conv2d(gm, unit.bwd, stride=1, pad=unit.bwd_pad, relu=False, use_bias=False)
        return gx, gm, None


def conv_res_relu(x: torch.Tensor, sc: torch.Tensor, unit: ConvUnit) -> torch.Tensor:
    """ReLU(unit(x) + sc) for a linear (no-ReLU) stride-1 conv unit."""
    if x.is_cuda:
        return _ConvResReluFn.apply(x, sc, unit)
    return torch.relu(unit(x) + sc)


class _SumSqCoreFn(torch.autograd.Function):
    """Per-image sum of x^2 over x[:, b:H-b, b:W-b, :] (fp32), HIP forward and backward."""

    @staticmethod
    def forward(ctx, x, b: int):
        x = x.contiguous()
        N = x.shape[0]
        core = (x.shape[1] - 2 * b) * (x.shape[2] - 2 * b) * x.shape[3]
        parts = max(1, min(64, core // (256 * 8 * 8)))
        part = torch.empty(N, parts, dtype=torch.float32, device=x.device)
        native.lib().sumsq_core(x, part, b)
        ctx.b = b
        ctx.save_for_backward(x)
        return part.sum(dim=1)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        gx = torch.empty_like(x)
        native.lib().sumsq_core_bwd(x, g.float().contiguous(), gx, ctx.b)
        return gx, None


def sumsq_core(x: torch.Tensor, b: int) -> torch.Tensor:
    """sum(x[:, b:-b, b:-b, :]^2) per image, fp32 [N] (the DeepDream activation loss term)."""
    if x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.shape[3] % 8 == 0:
        return _SumSqCoreFn.apply(x, b)
    core = x[:, b:x.shape[1] - b, b:x.shape[2] - b, :].float()
    return (core * core).sum(dim=(1, 2, 3))
