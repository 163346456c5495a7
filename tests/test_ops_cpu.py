"""CPU: algebraic identities the GPU paths rely on, checked with the fp32 reference ops."""
import pytest
import torch
import torch.nn.functional as F

from deconv_api_amd import ops
from deconv_api_amd.ops.conv import ConvWeights, transpose_subpixel


@pytest.mark.parametrize("k,s,p,H", [(7, 2, 3, 20), (3, 2, 0, 17), (1, 2, 0, 16), (3, 2, 1, 15), (5, 3, 2, 19),
                                     (3, 1, 1, 9)])
def test_transpose_subpixel_equals_conv_transpose(k, s, p, H):
    """dx of a stride-s conv == its s^2 parity classes computed as stride-1 convs."""
    g = torch.Generator().manual_seed(k * 100 + s * 10 + p)
    C, OC = 8, 16
    w = torch.randn(OC, C, k, k, generator=g)
    OH = (H + 2 * p - k) // s + 1
    gy = torch.randn(2, OH, OH, OC, generator=g)
    ref = ops.conv2d(gy, ConvWeights(w, None, "transpose"), stride=s, pad=p, relu=False, in_mode="transpose",
                     out_hw=(H, H), use_bias=False)
    want = F.grad.conv2d_input((2, C, H, H), w, gy.permute(0, 3, 1, 2), stride=s, padding=p).permute(0, 2, 3, 1)
    assert torch.allclose(ref, want, atol=1e-4)
    got = torch.zeros(2, H, H, C)
    for rh, rw, ws, pd in transpose_subpixel(w, s, (p, p)):
        hc, wc = len(range(rh, H, s)), len(range(rw, H, s))
        if ws is None or hc == 0 or wc == 0:
            continue
        got[:, rh::s, rw::s] = ops.conv2d(gy, ConvWeights(ws, None, "fwd"), stride=1, pad=pd, relu=False,
                                          out_hw=(hc, wc), use_bias=False)
    assert torch.allclose(got, want, atol=1e-4)


def test_mask_bit_trick_matches_definition():
    """csrc/common.h mask_pos_pk: keep a where m > 0 (bf16 and fp16 bit patterns), via integer ops."""
    import numpy as np

    rng = np.random.default_rng(0)
    m = rng.integers(0, 1 << 16, 4096, dtype=np.uint32)
    m[:8] = [0, 0x8000, 0x0001, 0x8001, 0x7FFF, 0xFFFF, 0x3C00, 0xBC00]
    a = rng.integers(0, 1 << 16, 4096, dtype=np.uint32)
    mp = m[0::2] | (m[1::2] << 16)
    ap = a[0::2] | (a[1::2] << 16)
    pos = (((mp & 0x7FFF7FFF) + 0x7FFF7FFF) & ~mp) & 0x80008000
    got = ap & ((pos >> 15) * 0xFFFF)
    keep = (m != 0) & (m & 0x8000 == 0)
    want_e = np.where(keep, a, 0)
    want = want_e[0::2] | (want_e[1::2] << 16)
    assert np.array_equal(got & 0xFFFFFFFF, want)
