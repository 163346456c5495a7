"""Convolution op surface: packed weights + NHWC conv with fused prologues/epilogues.

Device tensors (bf16 or fp16) go through ``csrc/bindings.cpp:conv``, which routes each shape to one
gfx950 kernel family: the LDS-DMA implicit GEMM and its KW3P shared-tap / stream-K variants
(``conv_dma*.hip``, ``conv_dma_impl.h``), the halo-stream 3x3 kernels (``conv_halo_stream.hip``),
the 64-channel halo / row-streaming kernels (``conv_smalln.hip``), the persistent 1x1 kernel
(``conv_pw.hip``), with ``conv_igemm.hip`` as the register-staged fallback. CPU tensors run a
PyTorch reference of exactly the same math (fp32 compute, output rounded to the input dtype),
which is both the CPU execution path and the oracle the GPU tests compare against.

Reference semantics being implemented (rashanarshad/deconv_api):
  * conv up   = conv3x3 'same' + bias + ReLU           (app/deepdream.py:71-76, 99)
  * conv down = ReLU(conv(ReLU(y), flip(W)^T)), no bias (app/deepdream.py:78-89, 110, 260)
  * pool up   = 2x2 max with first-max switch          (app/deepdream.py:152-188)
  * pool down = switch-masked nearest upsampling       (app/deepdream.py:191-209)
"""
from __future__ import annotations

import contextlib
import os
import threading
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from . import native

AMODE = {"plain": 0, "unpool": 1, "transpose": 2}
EPI = {"bf16": 0, "pool": 1, "f32": 2}
IMPL = {"auto": 0, "reg": 1, "dma": 2, "halo": 3}

# Kernel selection policy (A/B testing), DV_CONV_IMPL = auto | reg | dma | halo. 'auto' lets the
# binding pick per shape (bindings.cpp: halo-tile for narrow 3x3 layers at large maps, LDS-DMA
# elsewhere, register-staged for the ReLU-mask prologue); 'reg' forces the register-staged kernel
# with its fused unpool gather.
_policy = {"impl": os.environ.get("DV_CONV_IMPL", "auto")}


def set_policy(impl: Optional[str] = None) -> None:
    if impl is not None:
        assert impl in IMPL
        _policy["impl"] = impl


def get_policy() -> dict:
    return dict(_policy)


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def oc_pad(oc: int) -> int:
    """Output-channel padding that selects the kernel's N tile (128 / 64 / 16)."""
    if oc > 64 and (oc % 128 == 0 or oc > 256):
        return _round_up(oc, 128)
    if oc > 16:
        return _round_up(oc, 64)
    return 16


@dataclass
class ConvWeights:
    """A conv in torch OIHW form plus its gfx950 GEMM packing.

    ``w_oihw``: fp32 [OC, C, KH, KW] cross-correlation weights (C already padded to 8).
    ``kind``: 'fwd' (x -> conv2d(x, w)) or 'transpose' (dy -> conv_transpose2d(dy, w), i.e. the
    input-gradient of a strided conv whose forward weights are ``w``).
    Packed device matrix: ``w_gemm[OCpad, Kpad]`` bf16 with K index ``(kh*KW + kw)*Cin + c``.
    """

    w_oihw: torch.Tensor
    bias: Optional[torch.Tensor]
    kind: str = "fwd"
    w_gemm: Optional[torch.Tensor] = None
    bias_pad: Optional[torch.Tensor] = None

    @property
    def KH(self) -> int:
        return self.w_oihw.shape[2]

    @property
    def KW(self) -> int:
        return self.w_oihw.shape[3]

    @property
    def cin(self) -> int:
        """channels of the kernel's input tensor"""
        return self.w_oihw.shape[1] if self.kind == "fwd" else self.w_oihw.shape[0]

    @property
    def cout(self) -> int:
        return self.w_oihw.shape[0] if self.kind == "fwd" else self.w_oihw.shape[1]

    @property
    def K(self) -> int:
        return self.KH * self.KW * self.cin

    @property
    def Kpad(self) -> int:
        return _round_up(self.K, 64)

    @property
    def OCpad(self) -> int:
        return oc_pad(self.cout)

    def gemm_matrix(self) -> torch.Tensor:
        """[OCpad, Kpad] fp32 GEMM B^T matrix (rows = output channels, K contiguous)."""
        if self.kind == "fwd":
            m = self.w_oihw.permute(0, 2, 3, 1)  # [OC, KH, KW, C]
        else:
            # transposed gather: out ci, K index (kh, kw, co) -> w[co, ci, kh, kw]
            m = self.w_oihw.permute(1, 2, 3, 0)  # [C_fwd, KH, KW, OC_fwd]
        m = m.reshape(self.cout, self.K).float()
        out = torch.zeros(self.OCpad, self.Kpad, dtype=torch.float32)
        out[: self.cout, : self.K] = m
        return out

    def to_device(self, device, dtype=torch.bfloat16) -> "ConvWeights":
        """Copy to ``device``; on the GPU also pack the [OCpad, Kpad] GEMM matrix in ``dtype``
        (bf16, or fp16 for the fp16 DeepDream path) and the fp32 padded bias."""
        device = torch.device(device)
        w_oihw = self.w_oihw.to(device)
        bias = None if self.bias is None else self.bias.to(device)
        cw = ConvWeights(w_oihw, bias, self.kind)
        if device.type == "cuda":
            cw.w_gemm = self.gemm_matrix().to(device=device, dtype=dtype).contiguous()
            if bias is not None:
                bp = torch.zeros(self.OCpad, dtype=torch.float32)
                bp[: self.cout] = self.bias.float().cpu()
                cw.bias_pad = bp.to(device)
        return cw


def pad_channels_oihw(w: torch.Tensor, mult: int = 8) -> torch.Tensor:
    """Zero-pad the input-channel dim (dim 1) of an OIHW weight to a multiple of ``mult``."""
    c = w.shape[1]
    cp = _round_up(c, mult)
    if cp == c:
        return w
    out = torch.zeros(w.shape[0], cp, *w.shape[2:], dtype=w.dtype, device=w.device)
    out[:, :c] = w
    return out


def deconv_weights(fwd: ConvWeights) -> ConvWeights:
    """Deconvnet 'down' conv of a stride-1 'same' conv (reference app/deepdream.py:78-89):
    kernel transposed in/out and flipped spatially, zero bias."""
    assert fwd.kind == "fwd"
    w = fwd.w_oihw.flip(2, 3).transpose(0, 1).contiguous()
    return ConvWeights(pad_channels_oihw(w), None, "fwd")


def transpose_subpixel(w_oihw: torch.Tensor, stride: int, pad):
    """Sub-pixel decomposition of the transposed conv (input gradient) of a stride-``s`` conv.

    Output pixels of parity class (rh, rw) (ih = s*i + rh) only ever meet the taps
    kh = kh0 + s*j with kh0 = (rh + pad_h) mod s, so the class is a *stride-1* conv of dy with the
    sub-kernel w[:, :, kh0::s, kw0::s] (flipped, in/out transposed) and padding Jh-1-dh, where
    dh = (rh + pad_h - kh0) / s. Versus the direct transposed gather, which runs every tap and
    masks s^2-1 of s^2 of them to zero, this does s^2 times less MFMA work.

    Returns [(rh, rw, w_sub [C, OC, Jh, Jw] or None (class receives no taps), (pad_h, pad_w))].
    """
    s = int(stride)
    ph, pw = pad
    KH, KW = w_oihw.shape[2:]
    out = []
    for rh in range(s):
        kh0 = (rh + ph) % s
        jh = len(range(kh0, KH, s))
        dh = (rh + ph - kh0) // s
        for rw in range(s):
            kw0 = (rw + pw) % s
            jw = len(range(kw0, KW, s))
            dw = (rw + pw - kw0) // s
            if jh == 0 or jw == 0:
                out.append((rh, rw, None, None))
                continue
            sub = w_oihw[:, :, kh0::s, kw0::s].flip(2, 3).transpose(0, 1).contiguous()
            out.append((rh, rw, sub, (jh - 1 - dh, jw - 1 - dw)))
    return out


# ----------------------------------------------------------------------------------------
# CPU / oracle helpers
# ----------------------------------------------------------------------------------------

def unpool_ref(p: torch.Tensor, code: torch.Tensor, code_div: int = 1) -> torch.Tensor:
    """NHWC max-unpool: out[n, 2ph+dy, 2pw+dx, c] = p[n, ph, pw, c] if code == 2dy+dx."""
    N, PH, PW, C = p.shape
    if code_div > 1:
        code = code.repeat_interleave(code_div, dim=0)
    pos = torch.arange(4, device=p.device).view(1, 1, 1, 4, 1)
    sel = code.long().unsqueeze(3) == pos  # [N, PH, PW, 4, C]
    vals = p.unsqueeze(3) * sel.to(p.dtype)
    vals = vals.view(N, PH, PW, 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, PH * 2, PW * 2, C)
    return vals


def maxpool_switch_ref(x: torch.Tensor):
    """NHWC 2x2/s2 max-pool with first-max (row-major) switch code 0..3."""
    N, H, W, C = x.shape
    win = x.view(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 4, C)
    val, idx = win.max(dim=3)  # torch returns the first maximal index
    # torch.max(dim) on CPU returns the first occurrence for ties; make it explicit anyway
    first = (win == val.unsqueeze(3)).to(torch.int8).argmax(dim=3)
    return val, first.to(torch.uint8)


def _act_out(y: torch.Tensor, relu: bool, dtype) -> torch.Tensor:
    if relu:
        y = y.clamp_min(0)
    return y


def conv2d(x: torch.Tensor, cw: ConvWeights, *, stride: int = 1, pad=None, relu: bool = True,
           relu_in: bool = False, in_mode: str = "plain", code: Optional[torch.Tensor] = None,
           code_div: int = 1, mask: Optional[torch.Tensor] = None, epilogue: str = "bf16",
           out: Optional[torch.Tensor] = None, accumulate: bool = False, out_hw=None,
           use_bias: bool = True, res: Optional[torch.Tensor] = None, emask: Optional[torch.Tensor] = None,
           stats: Optional[torch.Tensor] = None, stats_div: int = 1, unpool_out: Optional[torch.Tensor] = None,
           unpool_div: int = 1, relu_cols: int = 0, out2: Optional[torch.Tensor] = None, split_col: int = 0,
           obits: Optional[torch.Tensor] = None, ebits: Optional[torch.Tensor] = None):
    """NHWC convolution.

    x: [N, H, W, C] (channel-slice views allowed: stride(3) == 1). For ``in_mode='unpool'`` x is
    the pooled map [N, H/2, W/2, C] and ``code`` its switch codes ([N/code_div, H/2, W/2, C]).
    epilogue 'pool' returns ``(pooled, code)``; otherwise the output tensor.
    ``res``: fused residual (ResNet block tail), out = [ReLU](conv + bias + res), ReLU after the add;
    ``emask`` (with ``res``): the result is zeroed where emask <= 0.
    ``stats`` (GPU, fp32 epilogue): fp64 [N / stats_div, 2] receives {sum, sum of squares} of each
    group of ``stats_div`` output images (the single-pass mosaic deprocess consumes it).
    ``unpool_out``: switch codes [N / unpool_div, OH, OW, OC]; the result is max-unpooled in the
    epilogue and returned at [N, 2 OH, 2 OW, OC] (the deconvnet's conv-down feeding an unpool).
    ``relu_cols`` > 0: ``relu`` applies to output channels < relu_cols only (a merged GEMM whose
    trailing channels are pre-activation values; LDS-DMA kernel).
    ``out2`` / ``split_col`` (GPU, plain 16-bit forward): output channels >= split_col go to ``out2``
    (channel c -> out2[..., c - split_col]) and only the leading ones to ``out`` - one merged GEMM
    feeding two consumers (InceptionV3: the b1 branch's concat slice and the heads buffer).
    ``obits`` (GPU, uint8 [M, OC / 8]): also write the output's 1-bit ReLU mask (bit = value > 0);
    ``ebits`` (GPU, with ``emask``): the 1-bit mask of ``emask`` to read instead of it. Both ride only on
    the persistent 1x1 kernel and the halo-stream kernels' LDS-staged epilogues: ``bits_flags()`` tells
    whether the last call on this thread wrote obits (1) / used ebits (2); otherwise obits is unwritten
    and emask applied as usual.
    """
    if pad is None:
        pad = (cw.KH // 2, cw.KW // 2)
    elif isinstance(pad, int):
        pad = (pad, pad)
    N = x.shape[0]
    if in_mode == "unpool":
        H, W = x.shape[1] * 2, x.shape[2] * 2
    else:
        H, W = x.shape[1], x.shape[2]
    C = x.shape[3]
    assert C == cw.cin, f"conv2d: input has {C} channels, weights expect {cw.cin}"
    if in_mode == "transpose":
        if out_hw is None:
            out_hw = ((H - 1) * stride - 2 * pad[0] + cw.KH, (W - 1) * stride - 2 * pad[1] + cw.KW)
        OH, OW = out_hw
    elif out_hw is not None:  # explicit output window (sub-pixel classes); reads past the map are 0
        OH, OW = out_hw
    else:
        OH = (H + 2 * pad[0] - cw.KH) // stride + 1
        OW = (W + 2 * pad[1] - cw.KW) // stride + 1
    OC = cw.cout
    if x.is_cuda:
        return _conv2d_hip(x, cw, N, H, W, C, OH, OW, OC, stride, pad, relu, relu_in, in_mode, code, code_div,
                           mask, epilogue, out, accumulate, use_bias, res, emask, stats, stats_div, unpool_out,
                           unpool_div, relu_cols, out2, split_col, obits, ebits)
    _tls.bits = 0  # CPU: no bit masks
    assert stats is None, "conv2d: stats are produced by the GPU kernels only"
    if out2 is not None:  # CPU: the full result, split between the two destinations
        y = _conv2d_ref(x, cw, N, H, W, C, OH, OW, OC, stride, pad, relu, relu_in, in_mode, code, code_div,
                        mask, epilogue, None, False, use_bias, res, emask, relu_cols)
        out2.copy_(y[..., split_col:])
        if out is not None:
            out.copy_(y[..., :split_col])
            return out
        return y[..., :split_col]
    if unpool_out is not None:
        assert epilogue == "bf16" and out is None and not accumulate, "conv2d: unpool_out needs a fresh 16-bit output"
        y = _conv2d_ref(x, cw, N, H, W, C, OH, OW, OC, stride, pad, relu, relu_in, in_mode, code, code_div,
                        mask, epilogue, None, False, use_bias, res, emask)
        return unpool_ref(y, unpool_out, unpool_div).contiguous()
    return _conv2d_ref(x, cw, N, H, W, C, OH, OW, OC, stride, pad, relu, relu_in, in_mode, code, code_div,
                       mask, epilogue, out, accumulate, use_bias, res, emask, relu_cols)


def _conv2d_ref(x, cw, N, H, W, C, OH, OW, OC, stride, pad, relu, relu_in, in_mode, code, code_div, mask,
                epilogue, out, accumulate, use_bias, res=None, emask=None, relu_cols=0):
    dtype = x.dtype
    xf = x.float()
    if in_mode == "unpool":
        xf = unpool_ref(xf, code, code_div)
    if mask is not None:
        xf = xf * (mask.float() > 0)
    if relu_in:
        xf = xf.clamp_min(0)
    X = xf.permute(0, 3, 1, 2)
    bias = cw.bias.float() if (use_bias and cw.bias is not None) else None
    if in_mode == "transpose":
        base_h = (H - 1) * stride - 2 * pad[0] + cw.KH
        base_w = (W - 1) * stride - 2 * pad[1] + cw.KW
        Y = F.conv_transpose2d(X, cw.w_oihw.float(), bias, stride=stride, padding=pad,
                               output_padding=(OH - base_h, OW - base_w))
    else:
        # explicit (possibly negative = cropping) padding reproducing the kernel's window exactly
        rb = (OH - 1) * stride + cw.KH - H - pad[0]
        rr = (OW - 1) * stride + cw.KW - W - pad[1]
        X = F.pad(X, (pad[1], rr, pad[0], rb))
        Y = F.conv2d(X, cw.w_oihw.float(), bias, stride=stride)
    y = Y.permute(0, 2, 3, 1)
    if res is not None:
        y = y + res.float()
    if relu and relu_cols > 0:
        y = torch.cat([y[..., :relu_cols].clamp_min(0), y[..., relu_cols:]], dim=-1)
    elif relu:
        y = y.clamp_min(0)
    if emask is not None:
        y = y * (emask.float() > 0)
    if epilogue == "pool":
        y = y.to(dtype).float()  # pool on stored-precision values, like the fused GPU epilogue
        pv, pc = maxpool_switch_ref(y)
        pv = pv.to(dtype).contiguous()
        if out is not None:
            out.copy_(pv)
            pv = out
        return pv, pc.contiguous()
    odt = torch.float32 if epilogue == "f32" else dtype
    if out is not None:
        if accumulate:
            y = y + out.float()
        out.copy_(y.to(out.dtype))
        return out
    return y.to(odt).contiguous()


# DV_CONV_GROUP=0: every conv its own launch (A/B of the grouped launches)
GROUPED = os.environ.get("DV_CONV_GROUP", "1") != "0"
_group_refs: list = []  # tensors of the open group's recorded convs (kept alive until it launches)
_group_open = [False]


@contextlib.contextmanager
def conv_group(device=None):
    """Launch the INDEPENDENT convs issued inside the block together: every one the LDS-DMA kernel
    would run with a small-problem tile config is recorded and, at exit, launched as grouped kernels
    (csrc/conv_dma_group.hip: one grid, each workgroup runs a tile of one problem); the rest launch
    immediately as usual. No conv inside may read another's output. Numerics are unchanged: the same
    tile program runs on the same data. CPU tensors and DV_CONV_GROUP=0: a no-op."""
    if not GROUPED or _group_open[0] or (device is not None and torch.device(device).type != "cuda"):
        yield
        return
    lib = native.lib()
    lib.conv_group_begin()
    _group_open[0] = True
    try:
        yield
    finally:
        _group_open[0] = False
        try:
            lib.conv_group_end()
        finally:
            _group_refs.clear()


@contextlib.contextmanager
def conv_group_paused():
    """Inside a conv_group: the convs issued here launch at once, in order (a pair where the second
    accumulates into the first's output); the group's recorded convs stay recorded."""
    if not _group_open[0]:
        yield
        return
    lib = native.lib()
    lib.conv_group_pause(True)
    try:
        yield
    finally:
        lib.conv_group_pause(False)


def check_stream_k() -> None:
    """Raise if a KW3P stream-K hand-off timed out since the last check: its tile was finished
    without the other half of its K range (conv_dma_impl.h; the counter lives in host-coherent
    memory, so this costs one host load, no sync). Called after every serving batch and bench."""
    n = native.lib().sk_errors(True)
    if n:
        raise RuntimeError(f"{n} KW3P stream-K hand-off(s) timed out: those conv output tiles are wrong "
                           "(set DV_NO_KW3_SK=1 when other kernels hold the CUs for seconds)")


_tls = threading.local()


def bits_flags() -> int:
    """1-bit mask flags of this thread's last conv2d: 1 = obits written, 2 = ebits used."""
    return getattr(_tls, "bits", 0)


def _conv2d_hip(x, cw, N, H, W, C, OH, OW, OC, stride, pad, relu, relu_in, in_mode, code, code_div, mask,
                epilogue, out, accumulate, use_bias, res=None, emask=None, stats=None, stats_div=1,
                unpool_out=None, unpool_div=1, relu_cols=0, out2=None, split_col=0, obits=None, ebits=None):
    lib = native.lib()
    dt = x.dtype
    assert dt in (torch.bfloat16, torch.float16) and x.stride(3) == 1, \
        "conv2d(hip): x must be bf16/fp16 NHWC (channel stride 1)"
    assert cw.w_gemm is not None, "conv2d(hip): weights not packed for the device (ConvWeights.to_device)"
    assert cw.w_gemm.dtype == dt, f"conv2d(hip): weights packed as {cw.w_gemm.dtype}, input is {dt}"
    x_ld = x.stride(2)
    if in_mode != "unpool":
        assert x.stride(1) == W * x_ld and x.stride(0) == H * W * x_ld, "conv2d(hip): x pixels must be dense"
    M = N * OH * OW
    if epilogue == "pool":
        assert OH % 2 == 0 and OW % 2 == 0
        if out is None:
            out = torch.empty(N, OH // 2, OW // 2, OC, dtype=dt, device=x.device)
        out_code = torch.empty(N, OH // 2, OW // 2, OC, dtype=torch.uint8, device=x.device)
    elif unpool_out is not None:
        assert epilogue == "bf16" and out is None and not accumulate, "conv2d: unpool_out needs a fresh 16-bit output"
        out_code = None
        out = torch.empty(N, 2 * OH, 2 * OW, OC, dtype=dt, device=x.device)
        unpool_out = unpool_out.contiguous()
    else:
        out_code = None
        if out is None:
            odt = torch.float32 if epilogue == "f32" else dt
            # with out2, a fresh out holds the leading split_col channels in a row of OC (the kernel's
            # storage check covers OC columns); the caller gets the [..., :split_col] view
            out = torch.empty(N, OH, OW, OC, dtype=odt, device=x.device)
            if out2 is not None:
                out = out[..., :split_col]
    assert out.stride(-1) == 1
    out_ld = out.stride(-2) if out.dim() == 4 else OC
    mask_ld = 0
    if mask is not None:
        assert mask.dtype == dt and mask.stride(3) == 1
        mask_ld = mask.stride(2)
    if code is not None:
        code = code.contiguous()
    geom = [N, H, W, C, OH, OW, OC, cw.OCpad, cw.KH, cw.KW, stride, pad[0], pad[1], cw.K, cw.Kpad, M,
            int(relu), int(relu_in), int(accumulate), int(code_div), x_ld, mask_ld, out_ld]
    bias = cw.bias_pad if use_bias else None
    # res / unpool_out / relu_cols exist on the LDS-DMA kernel only; emask also on the halo-stream
    # kernels (the binding routes by shape under 'auto')
    dma_only = res is not None or unpool_out is not None or relu_cols > 0 or out2 is not None or \
        (emask is not None and _policy["impl"] not in ("auto",))
    if _group_open[0]:
        _group_refs.append((x, cw, out, code, mask, res, emask, out2))
    _tls.bits = lib.conv(x, cw.w_gemm, bias, out, out_code, code, mask, geom, AMODE[in_mode], EPI[epilogue],
                         IMPL["dma"] if dma_only else IMPL[_policy["impl"]],  # DMA-only epilogue features
                         res, emask, stats, stats_div, unpool_out, unpool_div, relu_cols, out2, split_col,
                         obits, ebits)
    if epilogue == "pool":
        return out, out_code
    return out


# DV_FUSED_TAIL=0 turns off the fused deconvnet tail (unpool -> conv 64->64 -> per-tap products -> shift-add)
FUSED_TAIL = os.environ.get("DV_FUSED_TAIL", "1") != "0"


# DV_STEM_FUSE=0 turns off the fused VGG16 stem (conv 8->64 -> conv 64->64 -> pool as one launch)
STEM_FUSE = os.environ.get("DV_STEM_FUSE", "1") != "0"


def stem_ok(x: torch.Tensor, c1: ConvWeights, c2: ConvWeights) -> bool:
    """Shapes the fused stem takes: an 8-channel bf16 NHWC image with sides % 16 == 0, 3x3 8 -> 64 -> 64."""
    return (STEM_FUSE and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[3] == 8 and
            x.shape[1] % 16 == 0 and x.shape[2] % 16 == 0 and x.is_contiguous() and
            c1.kind == "fwd" and c1.KH == 3 and c1.KW == 3 and c1.cin == 8 and c1.cout == 64 and
            c2.kind == "fwd" and c2.KH == 3 and c2.KW == 3 and c2.cin == 64 and c2.cout == 64 and
            c1.w_gemm is not None and c2.w_gemm is not None and c1.w_gemm.dtype == torch.bfloat16)


def stem_pool(x: torch.Tensor, c1: ConvWeights, c2: ConvWeights):
    """VGG16 block1_conv1 -> block1_conv2 -> block1_pool as ONE launch (``conv3x3_hs16_kernel`` STEM):
    each 16 x 16 output tile computes its 18 x 18 x 64 conv1 halo from the RGB image straight into LDS,
    so the 64-channel 224^2 map between the two convs (2 x 1.6 GB of HBM traffic per 256 images) is never
    written. Bit-identical to ``conv2d(conv2d(x, c1), c2, epilogue='pool')``. Returns ``(pooled, codes)``,
    or None when the device kernel does not take the shape (the caller runs the separate launches).
    Reference: app/deepdream.py:99 (the per-layer conv up of the deconvnet's forward)."""
    if not stem_ok(x, c1, c2):
        return None
    N, H, W, _ = x.shape
    out = torch.empty(N, H // 2, W // 2, 64, dtype=x.dtype, device=x.device)
    code = torch.empty(N, H // 2, W // 2, 64, dtype=torch.uint8, device=x.device)
    if not native.lib().conv_stem_pool(x, c1.w_gemm, c1.bias_pad, c2.w_gemm, c2.bias_pad, out, code):
        return None
    return out, code


def tail_w2(last: ConvWeights) -> torch.Tensor:
    """[32, 64] matrix of a 64 -> 3 (3x3) conv's taps: row (kh*3 + kw)*3 + c = W[c, :, kh, kw]
    (rows 27..31 zero), in the dtype of the packed GEMM matrix. Cached on ``last``."""
    w2 = getattr(last, "_tail_w2", None)
    if w2 is None:
        w = last.w_oihw.float()  # [3, 64, 3, 3]
        m = torch.zeros(32, w.shape[1], dtype=torch.float32, device=w.device)
        m[:27] = w.permute(2, 3, 0, 1).reshape(27, w.shape[1])
        dt = last.w_gemm.dtype if last.w_gemm is not None else torch.float32
        w2 = m.to(dt).contiguous()
        last._tail_w2 = w2
    return w2


def tail_ok(x: torch.Tensor, mid: ConvWeights, last: ConvWeights) -> bool:
    """Shapes the fused deconvnet tail takes: pooled 64-channel bf16 input, 3x3 64 -> 64 -> 3 downs."""
    return (FUSED_TAIL and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[3] == 64 and
            mid.kind == "fwd" and mid.KH == 3 and mid.KW == 3 and mid.cin == 64 and mid.cout == 64 and
            last.kind == "fwd" and last.KH == 3 and last.KW == 3 and last.cin == 64 and last.cout == 3 and
            mid.bias is None and last.bias is None)


def deconv_tail(x: torch.Tensor, code: torch.Tensor, code_div: int, mid: ConvWeights, last: ConvWeights,
                stats: Optional[torch.Tensor] = None, stats_div: int = 1) -> Optional[torch.Tensor]:
    """The deconvnet's last two conv-downs in two kernels (VGG16 block1_conv2.down -> block1_conv1.down):
    d = ReLU(conv_mid(ReLU(unpool(x, code)))), recon = ReLU(conv_last(d)) as fp32 [N, H, W, 3].

    The 64-channel map d never reaches HBM: the first kernel's epilogue multiplies each bf16 tile of d
    by the last conv's taps (``tail_w2``: Z = d W2^T, 27 of 32 channels, bf16) on MFMA, and a 9-tap
    shift-add kernel sums Z over each pixel's neighbourhood (+ ReLU, per-image stats). 64 B/px are
    written and read instead of 128 (reference: app/deepdream.py:110,260 conv down; :191-209 unpool).
    Returns None when the device kernel does not take the shape (the caller runs the two convs).
    """
    if not tail_ok(x, mid, last):
        return None
    N, PH, PW, _ = x.shape
    z = torch.empty(N, 2 * PH, 2 * PW, 32, dtype=x.dtype, device=x.device)
    lib = native.lib()
    if not lib.conv_unpool_z(x.contiguous(), code.contiguous(), int(code_div), mid.w_gemm, tail_w2(last), z):
        return None
    out = torch.empty(N, 2 * PH, 2 * PW, 3, dtype=torch.float32, device=x.device)
    lib.zsum3x3(z, out, stats, int(stats_div))
    return out


def deconv_tail_ref(x: torch.Tensor, code: torch.Tensor, code_div: int, mid: ConvWeights,
                    last: ConvWeights) -> torch.Tensor:
    """fp32 oracle of ``deconv_tail`` with the same rounding points (bf16 d, bf16 Z)."""
    u = torch.relu(unpool_ref(x.float().cpu(), code.cpu(), code_div))
    wm = mid.w_oihw.to(torch.bfloat16).float().cpu()  # the packed GEMM matrix's rounding
    d = F.conv2d(u.permute(0, 3, 1, 2), wm, padding=1)
    d = torch.relu(d).to(torch.bfloat16).float()  # [N, 64, H, W]
    w2 = tail_w2(last).float().cpu()  # [32, 64]
    z = torch.einsum("nchw,zc->nzhw", d, w2).to(torch.bfloat16).float()[:, :27]
    N, _, H, W = z.shape
    zp = F.pad(z, (1, 1, 1, 1))
    out = torch.zeros(N, 3, H, W)
    for kh in range(3):
        for kw in range(3):
            t = kh * 3 + kw
            out += zp[:, t * 3:t * 3 + 3, kh:kh + H, kw:kw + W]
    return torch.relu(out).permute(0, 2, 3, 1).contiguous()
