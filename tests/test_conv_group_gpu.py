"""GPU: grouped LDS-DMA conv launches (csrc/conv_dma_group.hip, ops/conv.py:conv_group).

Independent small-problem convs recorded inside ``conv_group`` launch as one grid; each workgroup
runs the same tile program on the same data as the one-problem launch, so results must be BIT-
identical to launching every conv on its own. Checked on raw problems (mixed shapes, emask /
accumulate / relu_cols epilogues, fp16) and on whole InceptionV3 blocks forward + backward, whose
level-ordered branches (ops/inception.py) use the groups."""
import pytest
import torch

from deconv_api_amd import ops
from deconv_api_amd.ops import conv as C

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def no_splitk(native_lib):
    """Grouped problems never split K; the one-problem reference must not either (a K split sums
    the fp32 partials in another order)."""
    lib = ops.native.lib()
    lib.dma_tune(0, 1)
    yield
    lib.dma_tune(0, 0)


def _cw(cout, cin, k, dt, seed, kind="fwd"):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(cout, cin, k[0], k[1], generator=g) * (2.0 / (cin * k[0] * k[1])) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    return C.ConvWeights(w, b, kind).to_device("cuda", dt)


def _problems(dt):
    """(x, weights, kwargs) of independent convs with small-problem tile configs"""
    g = torch.Generator().manual_seed(0)
    mk = lambda *s: (torch.randn(*s, generator=g).clamp_min(0)).to(dt).cuda()  # noqa: E731
    out = []
    x1 = mk(4, 11, 11, 48)
    out.append((x1, _cw(64, 48, (5, 5), dt, 1), dict(pad=(2, 2))))
    x2 = mk(4, 11, 11, 64)
    out.append((x2, _cw(96, 64, (3, 3), dt, 2), dict(pad=(1, 1))))
    x3 = mk(4, 9, 9, 128)
    out.append((x3, _cw(192, 128, (1, 7), dt, 3), dict(pad=(0, 3))))
    x4 = mk(4, 9, 9, 160)
    em = mk(4, 9, 9, 160) - 0.3
    out.append((x4, _cw(160, 160, (7, 1), dt, 4), dict(pad=(3, 0), emask=em.contiguous())))
    x5 = mk(4, 11, 11, 192)
    out.append((x5, _cw(128, 192, (1, 1), dt, 5), dict(pad=(0, 0), relu_cols=64)))
    return out


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_grouped_launch_bit_identical(native_lib, dt):
    probs = _problems(dt)
    ref = [ops.conv2d(x, cw, **kw) for x, cw, kw in probs]
    acc_base = torch.randn(*ref[1].shape, generator=torch.Generator().manual_seed(9)).to(dt).cuda()
    want_acc = acc_base.clone()
    ops.conv2d(probs[1][0], probs[1][1], out=want_acc, accumulate=True, **probs[1][2])
    torch.cuda.synchronize()
    lib = ops.native.lib()
    outs = [torch.full_like(r, float("nan")) for r in ref]
    got_acc = acc_base.clone()
    lib.conv_group_begin()
    try:
        for (x, cw, kw), o in zip(probs, outs):
            ops.conv2d(x, cw, out=o, **kw)
        ops.conv2d(probs[1][0], probs[1][1], out=got_acc, accumulate=True, **probs[1][2])
    finally:
        n = lib.conv_group_end()
    torch.cuda.synchronize()
    assert 1 <= n < len(probs) + 1, n  # fewer launches than problems
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)
    assert torch.equal(got_acc, want_acc)


def test_conv_group_context_and_pause(native_lib):
    """The context manager records only while open; paused convs launch at once and in order (the
    second accumulates into the first)."""
    dt = torch.bfloat16
    (x1, w1, k1), (x2, w2, k2) = _problems(dt)[:2]
    a = ops.conv2d(x2, w2, **k2)
    want = a.clone()
    ops.conv2d(x2, w2, out=want, accumulate=True, **k2)
    with C.conv_group("cuda"):
        y1 = ops.conv2d(x1, w1, **k1)
        with C.conv_group_paused():
            b = ops.conv2d(x2, w2, **k2)
            ops.conv2d(x2, w2, out=b, accumulate=True, **k2)
    torch.cuda.synchronize()
    assert torch.equal(b, want)
    assert torch.equal(y1, ops.conv2d(x1, w1, **k1))


@pytest.mark.parametrize("bi,hw", [(0, 11), (2, 9), (3, 11), (4, 9), (5, 7), (9, 5)])
def test_inception_block_grouped_equals_ungrouped(native_lib, bi, hw, monkeypatch):
    """Whole mixed blocks, forward + backward (premasked contract), grouped vs DV_CONV_GROUP=0:
    bit-identical outputs and input gradients."""
    from deconv_api_amd.models.inception_v3 import InceptionV3
    from deconv_api_amd.ops import autograd as AG

    net = InceptionV3(0).build("cuda")
    cin = [192, 256, 288, 288, 768, 768, 768, 768, 768, 1280, 2048][bi]
    g = torch.Generator().manual_seed(bi)
    x = torch.randn(8, hw, hw, cin, generator=g).clamp_min(0).to(torch.bfloat16).cuda()
    res = {}
    for grouped in (False, True):
        monkeypatch.setattr(C, "GROUPED", grouped)
        xd = x.clone().requires_grad_(True)
        with AG.premasked_grads():
            y = net.iblocks[bi](AG.tag_relu_output(xd))
        gy = (torch.randn(*y.shape, generator=torch.Generator().manual_seed(1)).cuda() * (y.float() > 0)).to(y.dtype)
        with AG.premasked_grads():
            (gx,) = torch.autograd.grad(y, xd, gy)
        torch.cuda.synchronize()
        res[grouped] = (y.detach().clone(), gx.clone())
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
