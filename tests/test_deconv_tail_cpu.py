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


def test_stem_fusion_gate_and_cpu_forward():
    """The fused VGG16 stem (ops.stem_pool) is GPU-only: on CPU it declines and the engine's forward
    runs block1_conv1 / block1_conv2 + pool as before (same switches as the explicit ops)."""
    from deconv_api_amd.engine.deconvnet import DeconvNet
    from deconv_api_amd.models.vgg16 import VGG16

    c1 = ConvWeights(torch.zeros(64, 8, 3, 3), torch.zeros(64))
    c2 = _cw(64, 64, 3)
    x = torch.zeros(1, 32, 32, 8, dtype=torch.bfloat16)
    assert ops.stem_pool(x, c1, c2) is None
    rt = VGG16.random(0, include_top=False).build("cpu", torch.float32)
    g = torch.Generator().manual_seed(1)
    xi = torch.zeros(1, 32, 32, 8)
    xi[..., :3] = torch.randn(1, 32, 32, 3, generator=g) * 50
    st = DeconvNet(rt).forward(xi, "block1_pool")
    y1 = ops.conv2d(xi, rt.convs["block1_conv1"].fwd, relu=True)
    p, code = ops.conv2d(y1, rt.convs["block1_conv2"].fwd, relu=True, epilogue="pool")
    assert torch.equal(st.codes["block1_pool"], code) and torch.equal(st.out, p)
