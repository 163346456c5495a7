"""CPU: the fused deconvnet tail's oracle (Z = per-tap products + 9-tap shift-add) equals the two
plain convs it replaces (ops.conv2d CPU path) up to its two extra bf16 roundings."""
import numpy as np
import torch

from deconv_api_amd import ops
from deconv_api_amd.ops.conv import ConvWeights, tail_ok, tail_w2


def _cw(oc, c, seed):
    g = torch.Generator().manual_seed(seed)
    return ConvWeights((torch.randn(oc, c, 3, 3, generator=g) / np.sqrt(9 * c)).to(torch.bfloat16).float(), None)


def test_tail_oracle_matches_two_convs():
    g = torch.Generator().manual_seed(0)
    p = torch.randn(2, 6, 10, 64, generator=g).to(torch.bfloat16).float()
    code = torch.randint(0, 4, (1, 6, 10, 64), generator=g, dtype=torch.uint8)
    mid, last = _cw(64, 64, 1), _cw(3, 64, 2)
    ref = ops.deconv_tail_ref(p, code, 2, mid, last)
    d = ops.conv2d(p, mid, in_mode="unpool", code=code, code_div=2, relu_in=True, relu=True, use_bias=False)
    two = ops.conv2d(d.float(), last, relu=True, epilogue="f32", use_bias=False)
    assert ref.shape == two.shape == (2, 12, 20, 3)
    err = float((ref - two).abs().max() / two.abs().max())
    assert err < 2e-2


def test_tail_w2_layout_and_gate():
    last = _cw(3, 64, 5)
    w2 = tail_w2(last)
    assert w2.shape == (32, 64) and bool((w2[27:] == 0).all())
    # row (kh*3 + kw)*3 + c = W[c, :, kh, kw]
    assert torch.equal(w2[(1 * 3 + 2) * 3 + 1], last.w_oihw[1, :, 1, 2].float())
    assert not tail_ok(torch.zeros(1, 4, 4, 64, dtype=torch.bfloat16), _cw(64, 64, 1), last)  # CPU tensor
