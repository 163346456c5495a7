"""Native sub-pixel merge (csrc/pool.hip subpixel_merge): the input gradient of a stride-2 conv assembled
from its parity-class GEMMs in one pass, incl. accumulate-into and the ReLU output mask, vs the s^2
strided copies + add + threshold it replaces (InceptionV3's stride-2 convs, config 3; reference
semantics: app/deepdream.py:99, the conv whose input gradient DeepDream ascends)."""
import pytest
import torch

from deconv_api_amd.ops import autograd as AG

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k,s,p,H,C,OC,dt", [(3, 2, 0, 35, 64, 96, torch.bfloat16), (3, 2, 1, 36, 32, 64, torch.float16),
                                           (3, 2, 0, 17, 192, 320, torch.bfloat16), (1, 2, 0, 28, 64, 128, torch.float16)])
def test_subpixel_merge_matches_copies(native_lib, k, s, p, H, C, OC, dt):
    g = torch.Generator().manual_seed(11)
    u = AG.ConvUnit("u", torch.randn(OC, C, k, k, generator=g) / 10, None, s, (p, p)).build("cuda", dt)
    OH = (H + 2 * p - k) // s + 1
    gy = torch.randn(4, OH, OH, OC, generator=g).to("cuda", dt)
    if not AG._subpixel_ok(u):
        pytest.skip("class layout not taken by the native merge")
    got = AG._subpixel_dgrad(gy, None, u, (H, H))
    # the reference: per-class GEMMs, strided copies (the pre-merge path)
    want = torch.zeros(4, H, H, C, dtype=dt, device="cuda")
    for rh, rw, cw, pd in u.bwd_sub:
        hc, wc = len(range(rh, H, s)), len(range(rw, H, s))
        if hc == 0 or wc == 0 or cw is None:
            continue
        part = AG.conv2d(gy, cw, stride=1, pad=pd, relu=False, out_hw=(hc, wc), use_bias=False)
        want[:, rh::s, rw::s] = part[..., :C]
    assert torch.equal(got, want)
    # into an existing gradient, masked by a ReLU output
    base = torch.randn(4, H, H, C, generator=g).to("cuda", dt)
    mask = torch.randn(4, H, H, C, generator=g).to("cuda", dt)
    out = base.clone()
    AG.dgrad_strided_into(u, gy, (H, H), out, accumulate=True, emask=mask)
    ref = ((base.float() + want.float()).to(dt).float() * (mask.float() > 0)).to(dt)
    if AG.strided_direct(u, gy, (H, H)):
        assert (out.float() - ref.float()).abs().max() <= 2e-2 * ref.float().abs().max()
    else:
        assert torch.equal(out, ref)
