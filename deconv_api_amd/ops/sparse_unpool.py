"""2:4 structured-sparse formulation of a conv-down that consumes a max-unpooled map.

Every deconvnet backward conv whose input is ``unpool(v, code)`` (app/deepdream.py:191-209 feeding
app/deepdream.py:78-89,110 -- block1_conv2, block2_conv2, block3_conv3, block4_conv3 .down in the
flagship) sees, per channel, at most one nonzero in every 2x2 pooling window. The dense implicit
GEMM (K = 9*C) spends 3/4 of its MACs on those zeros. This module is the exact, MFMA-shaped
re-grouping that turns the layer into a 2:4 sparse GEMM for gfx950's
``v_smfmac_f32_32x32x32_bf16`` (measured 1.94x the dense instruction's K rate,
``profiles/smfmac_probe.txt``):

* Split the output by sub-pixel phase (a, b) = (y % 2, x % 2). Output (2p+a, 2q+b) reads unpooled
  rows 2p+a-1..2p+a+1, i.e. the full 2-row window of pooled row p plus one row of pooled row
  p + da (da = -1 if a == 0 else +1, sub-row r = 1 - a); the same along columns.
* Per input channel the 9 taps therefore fall into: the full window of (p, q) -- 4 taps, <= 1
  nonzero (S1); one row of (p+da, q) and one column of (p, q+db) -- 2 + 2 taps, <= 1 nonzero each
  (S2); the corner of (p+da, q+db) -- 1 tap, paired with the next channel's corner plus two zero
  rows (S3). Every group of 4 K-rows holds <= 2 nonzeros: the 2:4 contract.
* The compressed A operand is built straight from the POOLED signal and its switch code: the S1
  value is ``relu(v)`` at index ``code``; no unpooled map is ever materialised.

Per 16 input channels: 5 sparse K-steps of 32 (S1 x2, S2 x2, S3 x1) = 160 logical K rows versus
144 dense, executed at half the instruction count per logical row -> 5 smfmac vs 9 dense MFMA
K-steps (1.8x fewer MFMA cycles on those four layers, ~14 of the flagship's 38 conv-ms,
profiles/layers_r1_kw3b_on.txt).

This file holds the packing (weights -> per-phase sparse B) and a PyTorch emulation of the
compressed-operand contract that the HIP kernel must reproduce; ``tests/test_sparse_unpool.py``
checks it against ``F.conv_transpose2d`` on the explicitly unpooled map.
The smfmac operand layout it targets was pinned on the MI355X by ``tools/smfmac_layout.hip``:
B lane l holds K rows (l//32)*16 + j (j < 16, contiguous); A lane l holds the 4 groups at K rows
{8h..8h+7} u {16+8h..16+8h+7}, h = l//32; sparsity index of compressed slot s in bits 2s..2s+1.
"""
from __future__ import annotations

import torch

CHUNK = 16          # input channels (of the conv-down, = forward output channels) per 5 K-steps
STEPS = 5           # S1, S1, S2, S2, S3
KSTEP = 32          # logical K rows per smfmac


def _delta(a: int) -> int:
    return -1 if a == 0 else 1


def corr_weights(w_oihw: torch.Tensor) -> torch.Tensor:
    """Forward conv weight [Co, Ci, 3, 3] -> the conv-down as a 'same' correlation kernel
    wd[ky, kx, co, ci] (out[y,x,ci] = sum U[y+ky-1, x+kx-1, co] * wd[ky,kx,co,ci]); this is the
    reference's flip(W)^T (app/deepdream.py:78-89)."""
    return w_oihw.flip(2, 3).permute(2, 3, 0, 1).contiguous()


def pack_phase_weights(w_oihw: torch.Tensor) -> torch.Tensor:
    """Sparse B operands: [4 phases (a*2+b), C_chunks, 5*32 logical K rows, Ci] (fp32).

    Row order inside a chunk follows the step layout described in the module docstring, so a
    K-step's 32 rows are contiguous and a group's 4 rows are the 4 positions its 2-bit sparsity
    index can select."""
    Co, Ci = w_oihw.shape[:2]
    assert Co % CHUNK == 0 and w_oihw.shape[2:] == (3, 3)
    wd = corr_weights(w_oihw.float())
    nch = Co // CHUNK
    out = torch.zeros(4, nch, STEPS * KSTEP, Ci, dtype=torch.float32, device=w_oihw.device)
    for a in range(2):
        for b in range(2):
            ph = a * 2 + b
            r, cc = 1 - a, 1 - b
            for ch in range(nch):
                base = ch * CHUNK
                for s in range(2):                       # S1: full window of (p, q)
                    for g in range(8):
                        c = base + 8 * s + g
                        for t in range(4):
                            sr, sc = t // 2, t % 2
                            out[ph, ch, s * 32 + 4 * g + t] = wd[sr - a + 1, sc - b + 1, c]
                for s in range(2):                       # S2: row of (p+da, q), column of (p, q+db)
                    for g in range(8):
                        c = base + 8 * s + g
                        k0 = (2 + s) * 32 + 4 * g
                        dy_row = 2 * _delta(a) + r - a
                        for t in range(2):
                            out[ph, ch, k0 + t] = wd[dy_row + 1, t - b + 1, c]
                        dx_col = 2 * _delta(b) + cc - b
                        for t in range(2):
                            out[ph, ch, k0 + 2 + t] = wd[t - a + 1, dx_col + 1, c]
                dy_c, dx_c = 2 * _delta(a) + r - a, 2 * _delta(b) + cc - b
                for g in range(8):                       # S3: corners of (p+da, q+db), 2 channels
                    k0 = 4 * 32 + 4 * g
                    out[ph, ch, k0] = wd[dy_c + 1, dx_c + 1, base + 2 * g]
                    out[ph, ch, k0 + 1] = wd[dy_c + 1, dx_c + 1, base + 2 * g + 1]
    return out


def _shift(x: torch.Tensor, dy: int, dx: int) -> torch.Tensor:
    """x[n, p+dy, q+dx, c] with zeros outside the map."""
    N, H, W, C = x.shape
    out = torch.zeros_like(x)
    ys, yd = (slice(dy, H), slice(0, H - dy)) if dy >= 0 else (slice(0, H + dy), slice(-dy, H))
    xs, xd = (slice(dx, W), slice(0, W - dx)) if dx >= 0 else (slice(0, W + dx), slice(-dx, W))
    out[:, yd, xd] = x[:, ys, xs]
    return out


def compress_operand(v: torch.Tensor, code: torch.Tensor, a: int, b: int):
    """Compressed A for phase (a, b): values [N, PH, PW, nch, 5 steps, 8 groups, 2] and the 2-bit
    sparsity indices (same shape, int64). v is the pooled signal (ReLU applied here, as the
    reference's DActivation does before the conv-down), code the 2*dy+dx switch code."""
    N, PH, PW, C = v.shape
    v = v.float().clamp_min(0)
    code = code.long()
    nch = C // CHUNK
    da, db = _delta(a), _delta(b)
    r, cc = 1 - a, 1 - b
    vr, kr = _shift(v, da, 0), _shift(code, da, 0)          # row neighbour (p+da, q)
    vc, kc = _shift(v, 0, db), _shift(code, 0, db)          # column neighbour (p, q+db)
    vd, kd = _shift(v, da, db), _shift(code, da, db)        # corner (p+da, q+db)
    shp = (N, PH, PW, nch, 2, 8)
    val = torch.zeros(N, PH, PW, nch, STEPS, 8, 2)
    idx = torch.zeros(N, PH, PW, nch, STEPS, 8, 2, dtype=torch.long)
    # S1: the one nonzero of the window is v itself at its switch position; the two slots keep
    # distinct, ascending indices (slot 0 covers rows 0..2, slot 1 row 3)
    c1 = code.view(shp)
    val[..., 0:2, :, 0] = v.view(shp) * (c1 < 3)
    idx[..., 0:2, :, 0] = c1.clamp_max(2)
    val[..., 0:2, :, 1] = v.view(shp) * (c1 == 3)
    idx[..., 0:2, :, 1] = 3
    # S2 slot 0: row r of window (p+da, q) -> nonzero iff the switch sits in that row
    hit_r = (kr // 2) == r
    val[..., 2:4, :, 0] = (vr * hit_r).view(shp)
    idx[..., 2:4, :, 0] = (kr % 2).view(shp)
    # S2 slot 1: column cc of window (p, q+db)
    hit_c = (kc % 2) == cc
    val[..., 2:4, :, 1] = (vc * hit_c).view(shp)
    idx[..., 2:4, :, 1] = (2 + kc // 2).view(shp)
    # S3: corner (r, cc) of window (p+da, q+db), two channels per group
    hit_d = kd == 2 * r + cc
    vdd = (vd * hit_d).view(N, PH, PW, nch, 8, 2)
    val[..., 4, :, :] = vdd
    idx[..., 4, :, 0] = 0
    idx[..., 4, :, 1] = 1
    return val, idx


def sparse_unpool_conv_ref(v: torch.Tensor, code: torch.Tensor, packed: torch.Tensor,
                           relu_out: bool = True) -> torch.Tensor:
    """Emulates the smfmac kernel: for each phase, decompress (value, index) pairs into their
    4-row groups and multiply by the packed sparse B. Returns the NHWC conv-down output
    [N, 2PH, 2PW, Ci] in fp32 (ReLU'd like the reference's conv-down output)."""
    N, PH, PW, C = v.shape
    Ci = packed.shape[-1]
    out = torch.zeros(N, 2 * PH, 2 * PW, Ci)
    for a in range(2):
        for b in range(2):
            val, idx = compress_operand(v, code, a, b)
            M = N * PH * PW
            G = val[0, 0, 0].numel() // 2                    # groups per pixel
            val = val.reshape(M, G, 2)
            idx = idx.reshape(M, G, 2)
            rows = torch.arange(G).view(1, G, 1) * 4 + idx   # logical K row selected per slot
            dense = torch.zeros(M, G * 4)
            dense.scatter_add_(1, rows.reshape(M, -1), val.reshape(M, -1))
            y = dense @ packed[a * 2 + b].reshape(-1, Ci).float()
            out[:, a::2, b::2] = y.view(N, PH, PW, Ci)
    return out.clamp_min(0) if relu_out else out


def smfmac_counts(M: int, Co: int, Ci: int):
    """(dense MFMA 32x32x16 count, sparse SMFMAC 32x32x32 count) for a conv-down on an unpooled
    map with M output pixels, Co unpooled channels and Ci outputs."""
    dense = M * Ci * 9 * Co // (32 * 32 * 16)
    sparse = M * Ci * (Co // CHUNK) * STEPS * KSTEP // (32 * 32 * 32)
    return dense, sparse


def pack_for_kernel(w_oihw: torch.Tensor, device=None) -> torch.Tensor:
    """Packed weights in the HIP kernel's layout: [4 phases, C/16, Ci, 160] bf16 (K-contiguous rows,
    one 320-byte row per output channel, staged verbatim into the kernel's LDS B tile)."""
    p = pack_phase_weights(w_oihw.float().cpu())
    return p.permute(0, 1, 3, 2).contiguous().to(device=device, dtype=torch.bfloat16)


def sparse_unpool_conv(v: torch.Tensor, code: torch.Tensor, wt: torch.Tensor, code_div: int = 1,
                       out: torch.Tensor | None = None) -> torch.Tensor:
    """ReLU(convT(ReLU(unpool(v, code)), W)) on the GPU via csrc/conv_sparse.hip (bf16 NHWC).
    ``wt`` comes from :func:`pack_for_kernel`; ``code`` is shared by ``code_div`` consecutive
    images (the B*K filter batch). CPU tensors take :func:`sparse_unpool_conv_ref`."""
    if not v.is_cuda:
        raise ValueError("sparse_unpool_conv: device op (use sparse_unpool_conv_ref on CPU)")
    from . import native

    NB, PH, PW, C = v.shape
    Ci = wt.shape[2]
    if out is None:
        out = torch.empty(NB, 2 * PH, 2 * PW, Ci, dtype=torch.bfloat16, device=v.device)
    native.lib().sparse_unpool_conv(v.contiguous(), code.contiguous(), wt, out, code_div)
    return out
