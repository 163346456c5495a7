"""Non-conv ops: filter selection, seeded first deconv, deprocess mosaic, resize+preprocess,
standalone pool/unpool. HIP kernels for device tensors (csrc/misc.hip), PyTorch reference on CPU."""
from __future__ import annotations

import numpy as np
from typing import Optional

import torch

from . import native
from .conv import maxpool_switch_ref, unpool_ref

CAFFE_MEAN = (103.939, 116.779, 123.68)


def softmax_rows(x: torch.Tensor) -> torch.Tensor:
    """Row softmax of fp32 [M, N] (HIP kernel on the GPU)."""
    if x.is_cuda:
        x = x.float().contiguous()
        y = torch.empty_like(x)
        native.lib().softmax_rows(x, y)
        return y
    return torch.softmax(x.float(), dim=-1)


def channel_sum(x: torch.Tensor) -> torch.Tensor:
    """x: [N, H, W, C] -> fp32 [N, C] per-image channel sums (reference app/deepdream.py:369-376
    sums each filter's map; the reference additionally sums over the batch axis, see
    ``batch_topk='global'`` in the engine)."""
    N, H, W, C = x.shape
    if x.is_cuda:
        x = x.contiguous()
        out = torch.empty(N, C, dtype=torch.float32, device=x.device)
        native.lib().channel_sum(x, out, N, H * W, C)
        return out
    return x.float().sum(dim=(1, 2))


def topk_positive(v: torch.Tensor, k: int):
    """Stable top-k of strictly positive entries per row (value desc, index asc).

    Returns (idx int32 [N, k] with -1 padding, val fp32 [N, k]). Mirrors
    app/deepdream.py:369-380 (``sum_value > 0`` filter, Python's stable sort, ``[:top]``)."""
    v = v.float().contiguous()
    N, C = v.shape
    if v.is_cuda:
        idx = torch.empty(N, k, dtype=torch.int32, device=v.device)
        val = torch.empty(N, k, dtype=torch.float32, device=v.device)
        native.lib().topk_pos(v, idx, val, k)
        return idx, val
    idx = torch.full((N, k), -1, dtype=torch.int32)
    val = torch.zeros(N, k, dtype=torch.float32)
    for n in range(N):
        row = v[n]
        pos = torch.nonzero(row > 0).flatten()
        if pos.numel() == 0:
            continue
        vals = row[pos]
        order = torch.argsort(-vals, stable=True)[:k]
        sel = pos[order]
        idx[n, : sel.numel()] = sel.to(torch.int32)
        val[n, : sel.numel()] = row[sel]
    return idx, val


def seed_map(out4: torch.Tensor, idx: torch.Tensor, mode: str = "all", batch_topk: str = "per_image",
             code: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Seed maps of the deconvnet's B*K backward chains (reference app/deepdream.py:450-465).

    out4 [B, H, W, C] target activation, idx [B, K] filter indices (-1: none). Returns fp32
    [B*K, H, W]: channel idx[b, k] of image b, in 'max' mode only where it equals the map's max (the
    max over the whole batch with batch_topk='global', where every image shares the filter). With
    ``code`` (u8 [B, H, W, C] max-pool switches of a pool target) the map is max-unpooled to
    [B*K, 2H, 2W] and clamped at 0. GPU: one HIP kernel (``seed_map_kernel``, one workgroup per
    chain) instead of permute/gather/amax/mask/unpool passes."""
    B, H, W, C = out4.shape
    K = idx.shape[1]
    m = {"all": 0, "max": 2 if batch_topk == "global" else 1}[mode]
    if out4.is_cuda and out4.dtype in (torch.bfloat16, torch.float16):
        up = 1 if code is None else 2
        S = torch.empty(B * K, H * up, W * up, device=out4.device, dtype=torch.float32)
        native.lib().seed_map(out4.contiguous(), idx.to(torch.int32).contiguous(),
                              None if code is None else code.contiguous(), S, m)
        return S
    fi = idx.long().clamp_min(0)
    o = out4.float().permute(0, 3, 1, 2)  # [B, C, H, W]
    S = torch.gather(o, 1, fi.view(B, K, 1, 1).expand(B, K, H, W))  # [B, K, H, W]
    if m:
        S = S * (S == S.amax(dim=(0, 2, 3) if m == 2 else (2, 3), keepdim=True))
    S = (S * (idx >= 0).view(B, K, 1, 1)).reshape(B * K, H, W)
    if code is None:
        return S.contiguous()
    cf = torch.gather(code.permute(0, 3, 1, 2), 1, fi.view(B, K, 1, 1).expand(B, K, H, W)).reshape(B * K, H, W)
    return unpool_ref(S.unsqueeze(-1), cf.unsqueeze(-1)).squeeze(-1).clamp_min(0).contiguous()


def seed_deconv3x3(S: torch.Tensor, f: torch.Tensor, wt: torch.Tensor) -> torch.Tensor:
    """First deconv step from a one-channel map.

    S: fp32 [B, H, W] (the selected filter's activation map), f: int32 [B] filter index (-1: none),
    wt: [F, 3, 3, Cin] with wt[f, kh, kw, ci] = W_keras[2-kh, 2-kw, ci, f].
    Returns relu(sum_taps S * wt[f]) as [B, H, W, Cin] (dtype of wt)."""
    B, H, W = S.shape
    F_, _, _, Cin = wt.shape
    if S.is_cuda:
        f = f.to(torch.int32).contiguous()  # values >= F are clamped in the kernel
        out = torch.empty(B, H, W, Cin, dtype=wt.dtype, device=S.device)
        native.lib().seed_deconv3x3(S.float().contiguous(), f, wt.contiguous(), out)
        return out
    fl = f.long()
    valid = fl >= 0
    wsel = wt.float()[fl.clamp_min(0)]  # [B, 3, 3, Cin]
    Sp = torch.nn.functional.pad(S.float(), (1, 1, 1, 1))
    out = torch.zeros(B, H, W, Cin)
    for kh in range(3):
        for kw in range(3):
            out += Sp[:, kh:kh + H, kw:kw + W, None] * wsel[:, None, None, kh, kw, :]
    out = out.clamp_min(0) * valid.view(B, 1, 1, 1)
    return out.to(wt.dtype)


def deprocess_mosaic(recon: torch.Tensor, tiles: int = 4, reverse_channels: bool = True,
                     stats: Optional[torch.Tensor] = None) -> torch.Tensor:
    """recon fp32 [B*tiles, H, W, 3] -> u8 mosaic [B, 2H, 2W, 3].

    ``stats`` (GPU): fp64 [B, 2] per-mosaic {sum, sum of squares} already produced by the final
    conv (``conv2d(..., stats=...)``); without it the GPU path computes them in a separate pass.
    Mosaic [[t0, t1], [t2, t3]] (app/main.py:67-69), then Keras ``deprocess_image`` on the whole
    mosaic (app/deepdream.py:483-498), then channel reversal for an RGB encoder (OpenCV writes
    channel 0 as blue, app/main.py:73)."""
    BT, H, W, _ = recon.shape
    B = BT // tiles
    rows = (tiles + 1) // 2
    if recon.is_cuda:
        out = torch.empty(B, rows * H, 2 * W, 3, dtype=torch.uint8, device=recon.device)
        native.lib().deprocess_mosaic(recon.float().contiguous(), out, tiles, reverse_channels, stats)
        return out
    r = recon.float().view(B, tiles, H, W, 3)
    out = torch.zeros(B, rows * H, 2 * W, 3, dtype=torch.uint8)
    for b in range(B):
        x = r[b].double()
        mean = x.mean()
        std = ((x - mean) ** 2).mean().sqrt()
        xs = r[b] - mean.float()
        xs = xs / (std.float() + 1e-7)
        xs = xs * 0.1 + 0.5
        xs = xs.clamp(0, 1) * 255
        xs = xs.clamp(0, 255).to(torch.uint8)
        if reverse_channels:
            xs = xs.flip(-1)
        for t in range(tiles):
            oy, ox = (t // 2) * H, (t % 2) * W
            out[b, oy:oy + H, ox:ox + W] = xs[t]
    return out


# ---------------------------------------------------------------------------------------
# cv2-compatible resize (INTER_LINEAR on uint8) + caffe preprocess
# ---------------------------------------------------------------------------------------

def _lin_tab(dst: int, src: int):
    scale = src / dst
    d = np.arange(dst, dtype=np.float64)
    fx = ((d + 0.5) * scale - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx).astype(np.float32)
    lo = sx < 0
    fx[lo] = 0
    sx[lo] = 0
    hi = sx >= src - 1
    fx[hi] = 0
    sx[hi] = src - 1
    s1 = np.minimum(sx + 1, src - 1)
    a0 = np.rint((np.float32(1.0) - fx) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(fx * np.float32(2048)).astype(np.int64)
    return sx, s1, a0, a1


def resize_mode(hs: int, ws: int, oh: int, ow: int) -> int:
    if hs == oh and ws == ow:
        return 2
    if hs == 2 * oh and ws == 2 * ow:
        return 1
    return 0


def resize_u8_ref(img: np.ndarray, oh: int = 224, ow: int = 224) -> np.ndarray:
    """NumPy model of ``cv2.resize(img, (ow, oh))`` (INTER_LINEAR, uint8, 3 channels): 11-bit
    fixed-point coefficients, half-pixel centres, clamped edges, vertical pass rounded as the
    OpenCV SIMD path; exact 2x downscale takes OpenCV's INTER_AREA fast path.
    Parity with OpenCV itself is unpinned (cv2 is not installed here): documented +-1 LSB."""
    hs, ws = img.shape[:2]
    mode = resize_mode(hs, ws, oh, ow)
    src = img.astype(np.int64)
    if mode == 2:
        return img.copy()
    if mode == 1:
        s = src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)
    x0, x1, a0, a1 = _lin_tab(ow, ws)
    y0, y1, b0, b1 = _lin_tab(oh, hs)
    rows = src[:, x0] * a0[None, :, None] + src[:, x1] * a1[None, :, None]  # [hs, ow, 3]
    r0 = rows[y0]
    r1 = rows[y1]
    t0 = ((r0 >> 4) * b0[:, None, None]) >> 16
    t1 = ((r1 >> 4) * b1[:, None, None]) >> 16
    return np.clip((t0 + t1 + 2) >> 2, 0, 255).astype(np.uint8)


def preprocess_ref(img224: np.ndarray, cpad: int = 8, dtype=torch.bfloat16) -> torch.Tensor:
    """uint8 RGB [H, W, 3] -> [H, W, cpad] with slot c = rgb[c] - CAFFE_MEAN[c] (app/main.py:60-61;
    the reference's BGR decode + channel reversal feeds RGB into the BGR-mean slots, quirk Q1)."""
    x = torch.from_numpy(np.ascontiguousarray(img224)).float()
    out = torch.zeros(*x.shape[:2], cpad)
    out[..., :3] = x - torch.tensor(CAFFE_MEAN)
    return out.to(dtype)


def resize_preprocess(img: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """uint8 [(B,) Hs, Ws, 3] RGB -> out [(B,) OH, OW, cpad]: cv2-compatible resize + caffe
    preprocess, one fused kernel on device (all images of a batch share the source size)."""
    batched = img.dim() == 4
    imgb = img if batched else img.unsqueeze(0)
    outb = out if batched else out.unsqueeze(0)
    Hs, Ws = imgb.shape[1:3]
    OH, OW = outb.shape[1:3]
    if img.is_cuda:
        native.lib().resize_preprocess(imgb.contiguous(), outb, resize_mode(Hs, Ws, OH, OW))
        return out
    for b in range(imgb.shape[0]):
        r = resize_u8_ref(imgb[b].numpy(), OH, OW)
        outb[b].copy_(preprocess_ref(r, outb.shape[3], outb.dtype))
    return out


def maxpool2x2(x: torch.Tensor):
    if x.is_cuda:
        N, H, W, C = x.shape
        out = torch.empty(N, H // 2, W // 2, C, dtype=x.dtype, device=x.device)
        code = torch.empty(N, H // 2, W // 2, C, dtype=torch.uint8, device=x.device)
        native.lib().maxpool2x2(x.contiguous(), out, code)
        return out, code
    v, c = maxpool_switch_ref(x.float())
    return v.to(x.dtype), c


def unpool2x2(p: torch.Tensor, code: torch.Tensor, code_div: int = 1, relu: bool = False) -> torch.Tensor:
    N, PH, PW, C = p.shape
    if p.is_cuda:
        out = torch.empty(N, PH * 2, PW * 2, C, dtype=p.dtype, device=p.device)
        native.lib().unpool2x2(p.contiguous(), code.contiguous(), out, code_div, relu)
        return out
    y = unpool_ref(p.float(), code, code_div)
    if relu:
        y = y.clamp_min(0)
    return y.to(p.dtype)
