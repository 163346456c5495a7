"""GPU: the fused VGG16 stem (block1_conv1 -> block1_conv2 -> block1_pool in one hs16 launch whose
64-channel intermediate map lives only in LDS, csrc/conv_halo_stream.hip STEM) against the two-launch
path it replaces (bit-identical: same MFMA operands, K order and bf16 rounding points) and against the
fp32 PyTorch reference of the same three ops."""
import numpy as np
import pytest
import torch

from deconv_api_amd import ops
from deconv_api_amd.ops.conv import ConvWeights

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(t):
    return t.to(torch.bfloat16).float()


def _stem_weights(seed):
    g = torch.Generator().manual_seed(seed)
    w1 = torch.zeros(64, 8, 3, 3)
    w1[:, :3] = _bf(torch.randn(64, 3, 3, 3, generator=g) / np.sqrt(27))  # RGB padded to 8 channels
    b1 = _bf(torch.randn(64, generator=g) * 0.1)
    w2 = _bf(torch.randn(64, 64, 3, 3, generator=g) / np.sqrt(576))
    b2 = _bf(torch.randn(64, generator=g) * 0.1)
    return ConvWeights(w1, b1), ConvWeights(w2, b2)


@pytest.mark.parametrize("N,H,W", [(2, 224, 224), (3, 64, 80), (2, 96, 64), (2, 96, 48), (1, 16, 16), (2, 48, 16)])
def test_gpu_stem_pool_fused(native_lib, N, H, W):
    g = torch.Generator().manual_seed(N * 1000 + H + W)
    x = torch.zeros(N, H, W, 8)
    x[..., :3] = _bf(torch.randn(N, H, W, 3, generator=g) * 60)
    c1, c2 = _stem_weights(H + W)
    c1d, c2d = c1.to_device(DEV), c2.to_device(DEV)
    xd = x.to(torch.bfloat16).to(DEV).contiguous()
    r = ops.stem_pool(xd, c1d, c2d)
    assert r is not None, "the fused stem kernel refused a supported shape"
    out, code = r
    assert out.shape == (N, H // 2, W // 2, 64) and code.shape == out.shape
    # the two-launch path: bit-identical where it runs the row-streaming first layer (maps >= 56^2) and
    # the hs16 pool kernel (maps >= 64^2 with W >= 64, bindings.cpp), whose MFMA operands / K order the
    # fused kernel reproduces; smaller maps take the implicit GEMMs (other summation orders): close
    y1 = ops.conv2d(xd, c1d, relu=True)
    y2, code2 = ops.conv2d(y1, c2d, relu=True, epilogue="pool")
    if H * W >= 64 * 64 and W >= 64:
        assert torch.equal(out, y2)
        assert torch.equal(code, code2)
    else:
        d = float((out.float() - y2.float()).norm() / y2.float().norm())
        assert d < 1e-2, d
        assert float((code == code2).float().mean()) > 0.98
    # fp32 reference with the same bf16 rounding point between the convs
    r1 = _bf(ops.conv2d(x, c1, relu=True))
    rp, _ = ops.conv2d(r1, c2, relu=True, epilogue="pool")
    got = out.float().cpu()
    rel = float((got - rp).norm() / rp.norm().clamp_min(1e-12))
    assert rel < 1e-2, rel
    # border tiles: the second conv's zero padding (not conv1 of the zero-padded image) at the edges
    assert torch.isfinite(got).all()


def test_gpu_stem_pool_refuses_odd_shapes(native_lib):
    c1, c2 = _stem_weights(1)
    c1d, c2d = c1.to_device(DEV), c2.to_device(DEV)
    x = torch.zeros(1, 40, 40, 8, dtype=torch.bfloat16, device=DEV)  # 40 % 16 != 0
    assert ops.stem_pool(x, c1d, c2d) is None


def test_gpu_deconvnet_forward_uses_fused_stem(native_lib):
    """The engine's forward routes block1 through the fused launch and still produces the same
    block1_pool switches and target activations as the unfused forward."""
    from deconv_api_amd.engine.deconvnet import DeconvNet
    from deconv_api_amd.models.vgg16 import VGG16

    rt = VGG16.random(0, include_top=False).build(DEV)
    eng = DeconvNet(rt)
    g = torch.Generator().manual_seed(5)
    x = torch.zeros(2, 224, 224, 8)
    x[..., :3] = torch.randn(2, 224, 224, 3, generator=g) * 60
    xd = x.to(torch.bfloat16).to(DEV).contiguous()
    fused = eng.forward(xd, "block2_conv1")
    c1, c2 = rt.convs["block1_conv1"].fwd, rt.convs["block1_conv2"].fwd
    y1 = ops.conv2d(xd, c1, relu=True)
    p, code = ops.conv2d(y1, c2, relu=True, epilogue="pool")
    assert torch.equal(fused.codes["block1_pool"], code)
    ref = ops.conv2d(p, rt.convs["block2_conv1"].fwd, relu=True)
    assert torch.equal(fused.out, ref)
