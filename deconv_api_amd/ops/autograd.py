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

import contextlib
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .. import knobs
from . import native
from .conv import ConvWeights, bits_flags, conv2d, pad_channels_oihw, transpose_subpixel

# DV_RELU_BITS=0: bottleneck outputs keep no 1-bit ReLU masks (the next block's input-gradient epilogue
# reads the 16-bit activation as its mask again; A/B)
RELU_BITS = knobs.ablation("DV_RELU_BITS", "1") != "0"
# DV_SUBPIXEL=0 falls back to the direct transposed gather for strided dgrads (A/B testing)
SUBPIXEL = knobs.ablation("DV_SUBPIXEL", "1") != "0"
# DV_COL2IM=0 disables the GEMM + col2im input gradient of few-channel strided convs (A/B testing)
COL2IM = knobs.ablation("DV_COL2IM", "1") != "0"
# DV_STEM_DIRECT=0: InceptionV3's conv2d_1 (3 -> 32, 3x3 / 2) on the GEMM (+ col2im) path (A/B)
STEM_DIRECT = knobs.ablation("DV_STEM_DIRECT", "1") != "0"
# DV_STEM_FUSED=0: ResNet-50 conv1's input gradient as GEMM (cols to HBM) + col2im (A/B)
STEM_FUSED = knobs.ablation("DV_STEM_FUSED", "1") != "0"
# DV_STEM7=0: ResNet-50 conv1's forward on the generic implicit GEMM instead of the tap-paired MFMA
# kernel (csrc/conv_stem7.hip) (A/B)
STEM7 = knobs.ablation("DV_STEM7", "1") != "0"


_PREMASKED = [False]


@contextlib.contextmanager
def premasked_grads():
    """Forward passes run inside this context record the *premasked-gradient contract*: every
    gradient that will reach a ReLU output is already zero where that output is zero. It holds
    when all consumers of ReLU outputs are the ops of this module (each masks the gradient it
    returns by its input's positivity, in its dgrad epilogue) and the loss gradient vanishes where
    the activation does (DeepDream's sum of squares). ReLU units then skip their own mask pass: the
    ReLU-masked A-operand (2x slower LDS-bound dgrad) becomes an `emask` on the producer's epilogue.
    """
    old = _PREMASKED[0]
    _PREMASKED[0] = True
    try:
        yield
    finally:
        _PREMASKED[0] = old


def _is_relu_out(t: torch.Tensor) -> bool:
    """Tag set on tensors that are ReLU outputs (or max/avg pools / concats of them): >= 0, and
    zero where every upstream ReLU output is zero."""
    return bool(getattr(t, "_dv_relu", False))


def _tag(t: torch.Tensor, relu: bool) -> torch.Tensor:
    t._dv_relu = relu
    return t


def tag_relu_output(t: torch.Tensor, relu: bool = True) -> torch.Tensor:
    """Mark a tensor built from ReLU outputs outside this module (e.g. torch.cat of branches)."""
    return _tag(t, relu)


def cat_channels(parts) -> torch.Tensor:
    """torch.cat along channels (NHWC); the result is a ReLU output iff every part is."""
    return _tag(torch.cat(parts, dim=3), all(_is_relu_out(p) for p in parts))


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
                # few input channels (RGB stem): dx = col2im(dy @ W) -- a GEMM that reads dy once
                cr = self.w.shape[1]
                self.col_w = None
                if cr <= 8 and kh * kw * cr <= 256:
                    wc = self.w.permute(2, 3, 1, 0).reshape(kh * kw * cr, self.cout, 1, 1)  # [(kh,kw,c), oc]
                    self.col_w = ConvWeights(wc.contiguous(), None, "fwd").to_device(self.device, dtype)
                    self.col_ld = -(-kh * kw * cr // 8) * 8
                # few-channel strided stem conv (InceptionV3 conv2d_1): direct VALU kernels for the
                # forward and the input gradient (csrc/conv_stem.hip), fp32 [kh][kw][c][co] weights.
                # (ResNet-50's 7x7 conv1 measured slower there, 2352 FMAs per pixel: its gradient is
                # the fused MFMA GEMM + col2im kernel, csrc/conv_stem_dgrad.hip)
                self.stem_w = None
                if STEM_DIRECT and cr == 3 and self.stride == 2 and w8.shape[1] == 8 and kh == kw == 3 and \
                        self.cout == 32:
                    self.stem_w = self.w.permute(2, 3, 1, 0).contiguous().to(self.device)
                # ResNet-50 conv1 (3 -> 64, 7x7 / 2, pad 3) forward: [64][kh][kw 0..7][c 0..3] weights
                # (kw = 7 and c = 3 zero) for the tap-paired MFMA kernel (csrc/conv_stem7.hip)
                self.stem7_w = None
                if cr == 3 and kh == kw == 7 and self.stride == 2 and tuple(self.pad) == (3, 3) and self.cout == 64:
                    w4 = torch.zeros(64, 7, 8, 4)
                    w4[:, :, :7, :3] = self.w.permute(0, 2, 3, 1).float()
                    self.stem7_w = w4.reshape(64, 224).to(self.device, dtype).contiguous()
                # sub-pixel classes: s^2 stride-1 convs instead of one s^2-times-wasteful gather
                self.bwd_sub = []
                for rh, rw, ws, pd in transpose_subpixel(w8, self.stride, self.pad):
                    cw = None if ws is None else ConvWeights(pad_channels_oihw(ws), None, "fwd").to_device(
                        self.device, dtype)
                    self.bwd_sub.append((rh, rw, cw, pd))
        return self

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return _tag(_ConvFn.apply(x, self), self.relu)
        y = F.conv2d(x.permute(0, 3, 1, 2), self.w_dev[:, : x.shape[3]] if x.shape[3] < self.w_dev.shape[1]
                     else self.w_dev, self.b_dev, stride=self.stride, padding=self.pad).permute(0, 2, 3, 1)
        return y.relu() if self.relu else y


def _stem_fwd(x, unit: ConvUnit):
    """Strided few-channel stem conv on its own kernel, or None (geometry not covered): ResNet-50's
    conv1 on the tap-paired MFMA kernel, conv2d_1-style 3x3 convs on the direct VALU kernel."""
    w7 = getattr(unit, "stem7_w", None)
    if STEM7 and w7 is not None and x.shape[3] == 8 and x.is_contiguous():
        N, H, W, _ = x.shape
        y = torch.empty(N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, 64, dtype=x.dtype, device=x.device)
        if native.lib().stem7_fwd(x, w7, unit.fwd.bias_pad, y, int(unit.relu)):
            return y
    if getattr(unit, "stem_w", None) is None or unit.pad[0] != unit.pad[1] or unit.w.shape[2] != 3:
        return None
    N, H, W, C = x.shape
    OH = (H + 2 * unit.pad[0] - 3) // unit.stride + 1
    OW = (W + 2 * unit.pad[1] - 3) // unit.stride + 1
    y = torch.empty(N, OH, OW, unit.cout, dtype=x.dtype, device=x.device)
    g = [N, H, W, OH, OW, C, 3, unit.cout, 3, unit.stride, unit.pad[0], int(unit.relu)]
    return y if native.lib().stem_conv(x, unit.stem_w, unit.fwd.bias_pad, y, g, 0) else None


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, unit: ConvUnit):
        y = _stem_fwd(x, unit)
        if y is None:
            y = conv2d(x, unit.fwd, stride=unit.stride, pad=unit.pad, relu=unit.relu)
        ctx.unit = unit
        ctx.in_hw = (x.shape[1], x.shape[2])
        ctx.premasked = _PREMASKED[0]
        # premasked: the incoming gradient needs no ReLU mask, and the returned one is masked by
        # x > 0 (x a ReLU output) in the dgrad epilogue
        ctx.emask = ctx.premasked and _is_relu_out(x)
        saved = [y if (unit.relu and not ctx.premasked) else None, x if ctx.emask else None]
        ctx.save_for_backward(*saved)
        return y

    @staticmethod
    def backward(ctx, gy):
        unit: ConvUnit = ctx.unit
        mask, x = ctx.saved_tensors
        gy = gy.contiguous() if gy.stride(-1) != 1 else gy
        if mask is not None and gy.stride() != mask.stride():
            gy = gy.contiguous()
        emask = x if (x is not None and x.is_contiguous()) else None
        gx = _dgrad(unit, gy, mask, ctx.in_hw, emask)
        if x is not None and emask is None:
            gx = torch.ops.aten.threshold_backward(gx, x, 0)
        return gx, None


def _dgrad(unit: ConvUnit, gy, mask, in_hw, emask=None, ebits=None):
    """Input gradient of one conv unit: A-operand ReLU mask ``mask`` (its output, or None) and
    output mask ``emask`` (its input, when a ReLU output; applied in the epilogue when possible;
    ``ebits``: its 1-bit form, read instead where the kernel supports it)."""
    if unit.stride == 1:
        return conv2d(gy, unit.bwd, stride=1, pad=unit.bwd_pad, relu=False, mask=mask, use_bias=False, emask=emask,
                      ebits=ebits if emask is not None else None)
    gx = _dgrad_strided(unit, gy, mask, in_hw)
    return gx if emask is None else torch.ops.aten.threshold_backward(gx, emask, 0)


# strided-conv input gradients below this many (full transposed-GEMM) FLOPs run as ONE transposed
# conv written straight into its destination (accumulate / x-mask epilogue) instead of s^2
# sub-pixel GEMMs + copies: small maps are launch-latency bound, not MFMA bound
STRIDED_DIRECT_FLOPS = float(knobs.ablation("DV_STRIDED_DIRECT_GFLOP", "60")) * 1e9


def strided_direct(unit: ConvUnit, gy, in_hw) -> bool:
    kh, kw = unit.w.shape[2:]
    fl = 2.0 * gy.shape[0] * in_hw[0] * in_hw[1] * unit.cin * unit.cout * kh * kw
    return unit.col_w is None and fl <= STRIDED_DIRECT_FLOPS


def dgrad_strided_into(unit: ConvUnit, gy, in_hw, out: torch.Tensor, accumulate: bool = False,
                       emask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``out`` (=|+=) input gradient of a strided conv, zeroed where ``emask`` <= 0: one transposed
    conv on the LDS-DMA kernel when small (``strided_direct``), else the sub-pixel / col2im path
    plus one elementwise pass."""
    if strided_direct(unit, gy, in_hw):
        return conv2d(gy, unit.bwd, stride=unit.stride, pad=unit.pad, relu=False, in_mode="transpose",
                      out_hw=in_hw, use_bias=False, out=out, accumulate=accumulate, emask=emask)
    if out.is_cuda and SUBPIXEL and _subpixel_ok(unit, out):
        # parity-class GEMMs merged straight into ``out`` with the accumulate and the mask in the same pass
        return _subpixel_dgrad(gy, None, unit, in_hw, out=out, accumulate=accumulate, emask=emask)
    r = _dgrad_strided(unit, gy, None, in_hw)
    if emask is not None:
        r = torch.ops.aten.threshold_backward(r, emask, 0)
    return out.add_(r) if accumulate else out.copy_(r)


def _dgrad_strided(unit: ConvUnit, gy, mask, in_hw):
    if mask is None and getattr(unit, "stem_w", None) is not None and unit.pad[0] == unit.pad[1]:
        N, OH, OW, _ = gy.shape
        H, W = in_hw
        gx = torch.empty(N, H, W, unit.fwd.cin, dtype=gy.dtype, device=gy.device)
        g = [N, H, W, OH, OW, unit.fwd.cin, 3, unit.cout, unit.w.shape[2], unit.stride, unit.pad[0], 0]
        if native.lib().stem_conv(gy.contiguous(), unit.stem_w, None, gx, g, 1):
            return gx
    if unit.col_w is not None and COL2IM:
        return _col2im_dgrad(gy, mask, unit, in_hw)
    if SUBPIXEL:
        return _subpixel_dgrad(gy, mask, unit, in_hw)
    return conv2d(gy, unit.bwd, stride=unit.stride, pad=unit.pad, relu=False, mask=mask, in_mode="transpose",
                      out_hw=in_hw, use_bias=False)


def _col2im_dgrad(gy, mask, unit: ConvUnit, in_hw):
    """dx of a strided conv with <= 8 input channels: cols = (dy*mask) @ W^T as a 1x1 conv on the
    LDS-DMA kernel, then the col2im gather kernel; for ResNet-50's conv1 geometry both in ONE kernel
    (csrc/conv_stem_dgrad.hip: the cols tile never leaves LDS)."""
    N, OH, OW, _ = gy.shape
    H, W = in_hw
    kh, kw = unit.w.shape[2:]
    if STEM_FUSED and unit.fwd.cin == 8 and unit.pad[0] == unit.pad[1]:
        gx = torch.empty(N, H, W, 8, dtype=gy.dtype, device=gy.device)
        m = None if mask is None else mask.contiguous()
        if native.lib().stem_dgrad_fused(gy.contiguous(), m, unit.col_w.w_gemm, gx,
                                         [kh, kw, unit.stride, unit.pad[0], unit.w.shape[1]]):
            return gx
    J = unit.col_w.cout
    cols = torch.empty(N, OH, OW, unit.col_ld, dtype=gy.dtype, device=gy.device)
    conv2d(gy, unit.col_w, stride=1, pad=0, relu=False, mask=mask, use_bias=False, out=cols[..., :J])
    assert unit.fwd.cin == 8, "col2im path writes 8-channel input gradients"
    gx = torch.empty(N, H, W, 8, dtype=gy.dtype, device=gy.device)
    native.lib().col2im(cols, gx, [kh, kw, unit.stride, unit.pad[0], unit.pad[1], unit.w.shape[1]])
    return gx


def _subpixel_ok(unit: ConvUnit, out: Optional[torch.Tensor] = None) -> bool:
    """The native merge takes it: stride <= 2, the classes in (rh, rw) row-major order, 8-channel rows."""
    C = unit.fwd.cin
    return (unit.stride <= 2 and C % 8 == 0 and len(unit.bwd_sub) == unit.stride ** 2 and
            all((rh, rw) == (k // unit.stride, k % unit.stride) for k, (rh, rw, _, _) in enumerate(unit.bwd_sub)) and
            (out is None or (out.is_contiguous() and out.shape[3] == C)))


def _subpixel_dgrad(gy, mask, unit: ConvUnit, in_hw, out=None, accumulate: bool = False, emask=None):
    """dx of a strided conv as s^2 stride-1 convs (ops.conv.transpose_subpixel), each its parity class
    of dx. GPU: the class outputs are merged by ONE kernel (csrc/pool.hip subpixel_merge: interleave,
    optional accumulate into ``out`` and ``emask``) instead of s^2 strided copies (+ add, + mask)."""
    s = unit.stride
    H, W = in_hw
    N = gy.shape[0]
    C = unit.fwd.cin
    native_merge = gy.is_cuda and _subpixel_ok(unit, out)
    parts = []
    for rh, rw, cw, pd in unit.bwd_sub:
        hc, wc = len(range(rh, H, s)), len(range(rw, W, s))
        if hc == 0 or wc == 0 or cw is None:
            parts.append(None)
            continue
        parts.append(conv2d(gy, cw, stride=1, pad=pd, relu=False, mask=mask, out_hw=(hc, wc), use_bias=False))
    if native_merge:
        gx = out if out is not None else torch.empty(N, H, W, C, dtype=gy.dtype, device=gy.device)
        native.lib().subpixel_merge(parts, emask, gx, s, bool(accumulate and out is not None))
        return gx
    assert out is None and emask is None and not accumulate
    empty_class = any(p is None for p in parts)
    gx = (torch.zeros if empty_class else torch.empty)(N, H, W, C, dtype=gy.dtype, device=gy.device)
    for (rh, rw, _, _), part in zip(unit.bwd_sub, parts):
        if part is not None:
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
        # premasked: a max over ReLU outputs is 0 exactly when the chosen input is, so routing the
        # (already masked) output gradient to the argmax keeps the input gradient masked
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
        # premasked: an average spreads its gradient over zero inputs too -> mask by x > 0
        ctx.save_for_backward(x if (_PREMASKED[0] and _is_relu_out(x)) else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        g = ctx.geom
        (x,) = ctx.saved_tensors
        gx = torch.empty(g[0], g[1], g[2], g[3], dtype=gy.dtype, device=gy.device)
        native.lib().pool(gy.contiguous(), gx, None, 1, 1, g)
        if x is not None:
            gx = torch.ops.aten.threshold_backward(gx, x, 0)
        return gx, None, None, None


def max_pool(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    if x.is_cuda:
        return _tag(_MaxPoolFn.apply(x, k, s, p), _is_relu_out(x))
    return F.max_pool2d(x.permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1)


def avg_pool(x: torch.Tensor, k: int, s: int, p: int = 0) -> torch.Tensor:
    if x.is_cuda:
        return _tag(_AvgPoolFn.apply(x, k, s, p), _is_relu_out(x))
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


class _LossTapFn(torch.autograd.Function):
    """Identity on an intermediate DeepDream loss layer whose output also feeds deeper layers. Its
    backward adds the layer's own loss gradient (2 * scale[n] * a on the border-b core) to the
    gradient arriving from above in ONE kernel (sumsq_core_bwd with an addend), instead of autograd
    summing two separately materialized gradients (an extra elementwise add per tap and step)."""

    @staticmethod
    def forward(ctx, a, scale, b: int, part=None):
        ctx.save_for_backward(a, scale)
        ctx.b = b
        ctx.part = part
        return a.view_as(a)

    @staticmethod
    def backward(ctx, g):
        a, scale = ctx.saved_tensors
        gx = torch.empty_like(a)
        native.lib().sumsq_core_bwd(a, scale, gx, ctx.b, g.contiguous(), ctx.part)
        return gx, None, None, None


def loss_tap(a: torch.Tensor, scale: torch.Tensor, b: int, part: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``a`` unchanged; its gradient gains the DeepDream loss term of ``a`` (GPU, contiguous a). The
    ReLU-output tag carries over: the consumer's backward relies on it to hand back a gradient
    already masked by a > 0 (the premasked contract). ``part`` ([N, P] fp32): the backward kernel
    also writes the layer's loss partials there (no separate forward loss launch)."""
    return _tag(_LossTapFn.apply(a, scale, b, part), _is_relu_out(a))


def sumsq_core(x: torch.Tensor, b: int) -> torch.Tensor:
    """sum(x[:, b:-b, b:-b, :]^2) per image, fp32 [N] (the DeepDream activation loss term)."""
    if x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.shape[3] % 8 == 0:
        return _SumSqCoreFn.apply(x, b)
    core = x[:, b:x.shape[1] - b, b:x.shape[2] - b, :].float()
    return (core * core).sum(dim=(1, 2, 3))


class _BottleneckFn(torch.autograd.Function):
    """ResNet bottleneck block y = ReLU(c3(ReLU(c2(ReLU(c1(x))))) + shortcut(x)) with a hand-written
    backward that needs no elementwise kernels. Under the premasked contract (premasked_grads):

      g2 = dgrad_c3(gy)            epilogue-masked by y2 > 0
      g1 = dgrad_c2(g2)            epilogue-masked by y1 > 0
      gs = gy (identity) | dgrad_short(gy)
      gx = dgrad_c1(g1) + gs       residual epilogue, masked by x > 0 when x is a ReLU output

    so no dgrad reads a ReLU mask in its A operand (the LDS-bound path) and the block hands the
    previous block an already-masked gradient. Without the contract the masks are applied the
    usual way (gy * (y > 0) materialized, A-operand masks for c2 / c1).
    """

    @staticmethod
    def forward(ctx, x, units, box):
        c1, c2, c3, sh = units
        # 1-bit ReLU masks (bit = value > 0, [pixels, C / 8]) written by the same epilogues as y1, y2, y:
        # the backward's masked input gradients read them instead of the 16-bit maps (16x fewer bytes);
        # None where the kernel that ran has no such epilogue. y's mask is the NEXT block's (box[0]).
        def relu_conv(inp, w, stride, pad, **kw):
            bits = None
            if RELU_BITS and inp.is_cuda and w.cout % 8 == 0:
                OH = (inp.shape[1] + 2 * pad[0] - w.KH) // stride + 1
                OW = (inp.shape[2] + 2 * pad[1] - w.KW) // stride + 1
                bits = torch.empty(inp.shape[0] * OH * OW, w.cout // 8, dtype=torch.uint8, device=inp.device)
            out = conv2d(inp, w, stride=stride, pad=pad, relu=True, obits=bits, **kw)
            return out, (bits if bits is not None and bits_flags() & 1 else None)

        y1, y1b = relu_conv(x, c1.fwd, c1.stride, c1.pad)
        y2, y2b = relu_conv(y1, c2.fwd, c2.stride, c2.pad)
        sc = x if sh is None else conv2d(x, sh.fwd, stride=sh.stride, pad=sh.pad, relu=False)
        y, box[0] = relu_conv(y2, c3.fwd, 1, c3.pad, res=sc)
        ctx.y1b, ctx.y2b = y1b, y2b
        ctx.units = units
        ctx.premasked = _PREMASKED[0]
        ctx.x_relu = _is_relu_out(x) and x.is_contiguous()
        ctx.xbits = getattr(x, "_dv_bits", None)  # x's mask, when the previous block wrote one
        ctx.save_for_backward(x, y1, y2, y)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y1, y2, y = ctx.saved_tensors
        c1, c2, c3, sh = ctx.units
        in_hw = (x.shape[1], x.shape[2])
        gy = gy.contiguous()
        pm = ctx.premasked
        gm = gy if pm else torch.ops.aten.threshold_backward(gy, y, 0)
        g2 = conv2d(gm, c3.bwd, stride=1, pad=c3.bwd_pad, relu=False, use_bias=False, emask=y2 if pm else None,
                    ebits=ctx.y2b if pm else None)
        g1 = _dgrad(c2, g2, None if pm else y2, (y1.shape[1], y1.shape[2]), emask=y1 if pm else None,
                    ebits=ctx.y1b if pm else None)
        emask = x if (pm and ctx.x_relu) else None
        a_mask = None if pm else y1
        if c1.stride > 1 and sh is not None and _pw_strided(c1) and _pw_strided(sh) and sh.stride == c1.stride \
                and x.is_contiguous():
            # both stride-s 1x1 convs read x: their input gradients live on the same every-s-th
            # pixels. E = g1 W1^T + gm Wsh^T (two accumulating GEMMs), then ONE kernel writes gx
            # (E at the strided pixels, masked by x > 0, zeros elsewhere)
            E = conv2d(g1, c1.bwd_sub[0][2], stride=1, pad=0, relu=False, mask=a_mask, use_bias=False)
            conv2d(gm, sh.bwd_sub[0][2], stride=1, pad=0, relu=False, use_bias=False, out=E, accumulate=True)
            gx = torch.empty_like(x)
            native.lib().subpixel_scatter(E[..., : x.shape[3]].contiguous() if E.shape[3] != x.shape[3] else E,
                                          emask, gx, c1.stride)
            return gx, None, None
        gs = gm if sh is None else _dgrad(sh, gm, None, in_hw)
        if c1.stride == 1:
            gx = conv2d(g1, c1.bwd, stride=1, pad=c1.bwd_pad, relu=False, mask=a_mask, use_bias=False, res=gs,
                        emask=emask, ebits=ctx.xbits if emask is not None else None)
        else:
            gx = _dgrad_strided(c1, g1, a_mask, in_hw) + gs
            if emask is not None:
                gx = torch.ops.aten.threshold_backward(gx, emask, 0)
        return gx, None, None


def _pw_strided(u: ConvUnit) -> bool:
    """A 1x1 / pad-0 conv whose sub-pixel decomposition has exactly one non-empty class (0, 0)."""
    return tuple(u.w.shape[2:]) == (1, 1) and tuple(u.pad) == (0, 0) and len(u.bwd_sub) == u.stride ** 2 and \
        u.bwd_sub[0][:2] == (0, 0) and u.bwd_sub[0][2] is not None and all(cw is None for _, _, cw, _ in u.bwd_sub[1:])


def bottleneck(x: torch.Tensor, c1: ConvUnit, c2: ConvUnit, c3: ConvUnit, short: Optional[ConvUnit]) -> torch.Tensor:
    """ReLU(c3(c2(c1(x))) + short(x)) (c1, c2 with ReLU; c3, short linear)."""
    if x.is_cuda:
        box = [None]
        y = _BottleneckFn.apply(x, (c1, c2, c3, short), box)
        if box[0] is not None:
            y._dv_bits = box[0]
        return _tag(y, True)
    sc = short(x) if short is not None else x
    return torch.relu(c3(c2(c1(x))) + sc)
