"""GPU: every HIP kernel vs the PyTorch fp32 reference of the same op (ops/*.py CPU path).

bf16 inputs/weights are rounded identically on both sides, so the only differences are fp32
accumulation order and the final bf16 rounding of the GPU output."""
import os

import numpy as np
import pytest
import torch

from deconv_api_amd import ops
from deconv_api_amd.ops.conv import ConvWeights, pad_channels_oihw

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True, params=["auto", "reg", "dma"])
def conv_impl(request):
    """Run every test against the automatic kernel choice and the forced register-staged and
    LDS-DMA kernels (the halo-tile kernel has dedicated tests below)."""
    from deconv_api_amd.ops import conv as C

    old = C.get_policy()
    C.set_policy(impl=request.param)
    yield request.param
    C.set_policy(**old)


def _bf(t):
    return t.to(torch.bfloat16).float()


def _cw(oc, c, kh=3, kw=3, kind="fwd", bias=True, seed=0):
    g = torch.Generator().manual_seed(seed)
    shape = (oc, c, kh, kw)
    w = _bf(torch.randn(*shape, generator=g) / np.sqrt(c * kh * kw))
    b = _bf(torch.randn(oc if kind == "fwd" else c, generator=g) * 0.1) if bias else None
    return ConvWeights(w, b, kind)


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-6))


def _cmp_conv(x, cw, **kw):
    x = x.to(torch.bfloat16)
    ref = ops.conv2d(x.float(), cw, **kw)
    got = ops.conv2d(x.to(DEV), cw.to_device(DEV), **kw)
    return ref, got


@pytest.mark.parametrize("N,H,W,C,OC", [(2, 16, 16, 8, 64), (1, 14, 14, 64, 64), (2, 9, 7, 128, 256),
                                        (1, 12, 10, 16, 48), (3, 8, 8, 64, 3), (1, 5, 6, 512, 512),
                                        (2, 17, 13, 24, 200)])
def test_conv_fwd_bf16(native_lib, N, H, W, C, OC):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, H, W, C, generator=g)
    cw = _cw(OC, C)
    for relu in (True, False):
        ref, got = _cmp_conv(x, cw, relu=relu)
        assert got.shape == ref.shape and got.dtype == torch.bfloat16
        assert _rel(got, ref) < 1e-2


def test_conv_strided_and_rect_kernels(native_lib):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, 17, 15, 32, generator=g)
    for (kh, kw, s, pad) in [(1, 1, 1, (0, 0)), (1, 7, 1, (0, 3)), (7, 1, 1, (3, 0)), (3, 3, 2, (0, 0)),
                             (1, 1, 2, (0, 0)), (5, 5, 1, (2, 2)), (7, 7, 2, (3, 3))]:
        cw = _cw(64, 32, kh, kw)
        ref, got = _cmp_conv(x, cw, stride=s, pad=pad)
        assert got.shape == ref.shape, (kh, kw, s)
        assert _rel(got, ref) < 1e-2, (kh, kw, s)


def test_conv_f32_out_and_accumulate(native_lib):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 10, 12, 64, generator=g)
    cw = _cw(3, 64, bias=False)
    ref, got = _cmp_conv(x, cw, relu=True, epilogue="f32", use_bias=False)
    assert got.dtype == torch.float32 and _rel(got, ref) < 1e-3
    base = torch.randn(2, 10, 12, 64, generator=g)
    cw2 = _cw(64, 64)
    out_d = base.to(torch.bfloat16).to(DEV)
    ops.conv2d(x.to(torch.bfloat16).to(DEV), cw2.to_device(DEV), relu=False, out=out_d, accumulate=True)
    out_r = base.to(torch.bfloat16).float().clone()
    ops.conv2d(_bf(x), cw2, relu=False, out=out_r, accumulate=True)
    assert _rel(out_d, out_r) < 1e-2


def test_conv_pool_epilogue(native_lib):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 16, 14, 64, generator=g)
    cw = _cw(128, 64)
    (rp, rc), (gp, gc) = _cmp_conv(x, cw, epilogue="pool")
    assert gp.shape == (2, 8, 7, 128) and gc.dtype == torch.uint8
    assert _rel(gp, rp) < 1e-2
    # switch codes must agree wherever the window max is not a near-tie
    full = ops.conv2d(_bf(x), cw).float()
    win = full.view(2, 8, 2, 7, 2, 128).permute(0, 1, 3, 2, 4, 5).reshape(2, 8, 7, 4, 128)
    top2 = win.topk(2, dim=3).values
    clear = (top2[:, :, :, 0] - top2[:, :, :, 1]) > 0.02 * top2[:, :, :, 0].abs().clamp_min(1e-3)
    agree = (gc.cpu() == rc)[clear]
    assert agree.float().mean() > 0.999


@pytest.mark.parametrize("N,H,W,C,OC", [(2, 56, 56, 256, 256), (3, 28, 28, 512, 512), (2, 16, 14, 64, 128),
                                        (3, 10, 14, 64, 192), (1, 12, 12, 32, 48)])
def test_conv_pool_epilogue_transposed(native_lib, monkeypatch, N, H, W, C, OC):
    """Pooled-max epilogue with DPP-transposed 8-B stores (epilogue_pool_t) == staged through LDS
    (epilogue_pool_lds, 16-B stores, DV_POOL_EPI=lds) == the per-element stores (DV_NO_POOL_T=1) bit for bit,
    values and switch codes; partial channel blocks (OC 48: the 8-B path) and M tails."""
    monkeypatch.setenv("DV_NO_POOL_V3", "1")
    monkeypatch.setenv("DV_NO_HS16", "1")
    monkeypatch.setenv("DV_KW3", "0")
    g = torch.Generator().manual_seed(N * H + OC)
    x = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16).to(DEV)
    cwd = _cw(OC, C).to_device(DEV)
    got_p, got_c = ops.conv2d(x, cwd, relu=True, epilogue="pool")  # the register-transposed 8-B stores
    monkeypatch.setenv("DV_POOL_EPI", "lds")  # LDS-staged 16-B stores where OC % 16 == 0 (opt-in)
    lds_p, lds_c = ops.conv2d(x, cwd, relu=True, epilogue="pool")
    monkeypatch.delenv("DV_POOL_EPI")
    assert torch.equal(got_p, lds_p) and torch.equal(got_c, lds_c)
    monkeypatch.setenv("DV_NO_POOL_T", "1")
    ref_p, ref_c = ops.conv2d(x, cwd, relu=True, epilogue="pool")
    assert torch.equal(got_p, ref_p) and torch.equal(got_c, ref_c)


@pytest.mark.parametrize("N,H,W", [(2, 112, 120), (1, 118, 112), (1, 224, 224)])
def test_conv_pool_v3(native_lib, N, H, W):
    """64 -> 64 conv + fused pool at >= 112^2 maps (weight-resident halo kernel) vs the fp32 reference
    and vs the implicit-GEMM pool epilogue (DV_NO_POOL_V3)."""
    import os

    g = torch.Generator().manual_seed(41)
    x = torch.relu(torch.randn(N, H, W, 64, generator=g))
    cw = _cw(64, 64)
    (rp, rc), (gp, gc) = _cmp_conv(x, cw, epilogue="pool")
    assert gp.shape == (N, H // 2, W // 2, 64) and gc.shape == gp.shape
    assert _rel(gp, rp) < 1e-2
    full = ops.conv2d(_bf(x), cw).float()
    win = full.view(N, H // 2, 2, W // 2, 2, 64).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 4, 64)
    top2 = win.topk(2, dim=3).values
    clear = (top2[:, :, :, 0] - top2[:, :, :, 1]) > 0.02 * top2[:, :, :, 0].abs().clamp_min(1e-3)
    assert (gc.cpu() == rc)[clear].float().mean() > 0.999
    os.environ["DV_NO_POOL_V3"] = "1"
    try:
        ip, ic = ops.conv2d(x.to(torch.bfloat16).to(DEV), cw.to_device(DEV), epilogue="pool")
    finally:
        del os.environ["DV_NO_POOL_V3"]
    assert _rel(gp, ip) < 1e-2
    assert (gc == ic).float().mean() > 0.995


@pytest.mark.parametrize("N,H,W,OC", [(2, 224, 224, 64), (3, 60, 70, 64), (1, 57, 33, 48)])
def test_conv_first_layer_stream(native_lib, N, H, W, OC):
    """8-channel (padded RGB) -> OC first-layer conv on the row-streaming kernel vs the fp32 reference
    and vs the implicit-GEMM kernel (DV_NO_C8_STREAM)."""
    import os

    g = torch.Generator().manual_seed(43)
    x = torch.randn(N, H, W, 8, generator=g) * 50
    x[..., 3:] = 0
    cw = _cw(OC, 8)
    ref, got = _cmp_conv(x, cw, relu=True)
    assert got.shape == ref.shape and _rel(got, ref) < 1e-2
    os.environ["DV_NO_C8_STREAM"] = "1"
    try:
        alt = ops.conv2d(x.to(torch.bfloat16).to(DEV), cw.to_device(DEV), relu=True)
    finally:
        del os.environ["DV_NO_C8_STREAM"]
    assert _rel(got, alt) < 1e-2


@pytest.mark.parametrize("N,H,W,C,OC", [(6, 112, 112, 128, 128), (11, 112, 112, 128, 64), (5, 115, 121, 64, 128),
                                        (21, 56, 56, 256, 256)])
def test_conv_large_m_tiles(native_lib, conv_impl, N, H, W, C, OC):
    """Large-M launches (>= one 256x128 / 512x64 tile per CU): bf16 vector
    epilogue, f32 epilogue, fused pool+switch and the transposed dgrad."""
    g = torch.Generator().manual_seed(21)
    x = torch.randn(N, H, W, C, generator=g)
    cw = _cw(OC, C)
    ref, got = _cmp_conv(x, cw, relu=True)
    assert got.shape == ref.shape and _rel(got, ref) < 1e-2
    ref, got = _cmp_conv(x, cw, relu=False, epilogue="f32")
    assert _rel(got, ref) < 1e-3
    if H % 2 == 0 and W % 2 == 0:
        (rp, _), (gp, _) = _cmp_conv(x, cw, epilogue="pool")
        assert _rel(gp, rp) < 1e-2
    ct = _cw(C, OC, kind="transpose", bias=False)  # input gradient of a forward conv OC -> C
    kw = dict(relu=True, in_mode="transpose", stride=1, pad=(1, 1), out_hw=(H, W), use_bias=False)
    ref = ops.conv2d(_bf(x), ct, **kw)
    got = ops.conv2d(x.to(torch.bfloat16).to(DEV), ct.to_device(DEV), **kw)
    assert got.shape == ref.shape and _rel(got, ref) < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,C,OC,bias,relu", [(2, 112, 112, 128, 128, False, True), (2, 112, 112, 128, 64, False, True),
                                                   (1, 112, 112, 64, 128, True, True), (1, 70, 100, 96, 128, True, False),
                                                   (3, 64, 77, 32, 64, True, True), (1, 65, 64, 256, 120, True, True)])
def test_conv_halo_stream(native_lib, dt, N, H, W, C, OC, bias, relu):
    """Halo-stream kernel (3x3 s1 p1, C % 32 == 0, OCpad 64/128, >= 64x64 maps; auto policy) vs the
    fp32 reference and vs the implicit-GEMM path (DV_NO_HS): ragged tiles, OC < OCpad, no-bias, fp16."""
    import os

    g = torch.Generator().manual_seed(29)
    x = torch.randn(N, H, W, C, generator=g)
    cw = _cw(OC, C, bias=bias)
    xd = x.to(dt).to(DEV)
    ref = ops.conv2d(x.to(dt).float(), cw, relu=relu, use_bias=bias)
    got = ops.conv2d(xd, cw.to_device(DEV, dt), relu=relu, use_bias=bias)
    assert got.shape == ref.shape and got.dtype == dt and _rel(got, ref) < 1e-2
    os.environ["DV_HS16_EPI"] = "reg"  # hs16 register-layout 8-B store epilogue: bit-identical to the LDS one
    try:
        reg = ops.conv2d(xd, cw.to_device(DEV, dt), relu=relu, use_bias=bias)
    finally:
        del os.environ["DV_HS16_EPI"]
    assert torch.equal(got, reg)
    for env in ("DV_NO_HS", "DV_NO_HS16"):  # implicit GEMM; 16x32-tile kernel instead of 16x16
        os.environ[env] = "1"
        try:
            alt = ops.conv2d(xd, cw.to_device(DEV, dt), relu=relu, use_bias=bias)
        finally:
            del os.environ[env]
        assert _rel(got, alt) < 1e-2, env


@pytest.mark.parametrize("H,W", [(72, 80), (64, 80)])
def test_conv_halo_stream_slices(native_lib, H, W):
    """Halo-stream kernels (16x32 tiles; 16x16 tiles when H, W % 16 == 0) on a channel-slice input
    view (x_ld > C) writing into a channel-slice output view (out_ld > OC, concat layout) of a larger
    buffer: no byte outside the slices changes."""
    g = torch.Generator().manual_seed(37)
    big = torch.randn(2, H, W, 160, generator=g).to(torch.bfloat16).to(DEV)
    cw = _cw(128, 96)
    x = big[..., 32:128]
    ref = ops.conv2d(big[..., 32:128].float().cpu(), cw, relu=True)
    buf = torch.full((2, H, W, 192), 7.0, dtype=torch.bfloat16, device=DEV)
    got = ops.conv2d(x, cw.to_device(DEV), relu=True, out=buf[..., 40:168])
    assert _rel(got, ref) < 1e-2
    assert (buf[..., :40] == 7).all() and (buf[..., 168:] == 7).all()


@pytest.mark.parametrize("N,H,W,C,OC", [(2, 112, 112, 128, 128), (1, 64, 96, 64, 128), (1, 80, 70, 96, 64),
                                        (2, 48, 32, 32, 64)])
def test_conv_halo_stream_pool(native_lib, N, H, W, C, OC):
    """Fused 2x2 max-pool + switch epilogue of the halo-stream kernel (DPP pair exchange) vs the fp32
    reference: pooled values, and switch codes wherever the window max is not a near-tie."""
    g = torch.Generator().manual_seed(31)
    x = torch.randn(N, H, W, C, generator=g)
    cw = _cw(OC, C)
    (rp, rc), (gp, gc) = _cmp_conv(x, cw, epilogue="pool")
    assert gp.shape == (N, H // 2, W // 2, OC) and _rel(gp, rp) < 1e-2
    full = ops.conv2d(_bf(x), cw).float()
    win = full.view(N, H // 2, 2, W // 2, 2, OC).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 4, OC)
    top2 = win.topk(2, dim=3).values
    clear = (top2[:, :, :, 0] - top2[:, :, :, 1]) > 0.02 * top2[:, :, :, 0].abs().clamp_min(1e-3)
    assert (gc.cpu() == rc)[clear].float().mean() > 0.999


def test_conv_relu_in_every_kernel(native_lib, conv_impl):
    """relu_in (ReLU on the input) on signed inputs: the LDS-DMA kernel stages A verbatim, so the
    binding ReLUs a dense copy; plain, channel-slice view, transposed and masked inputs."""
    g = torch.Generator().manual_seed(23)
    full = torch.randn(2, 12, 14, 192, generator=g)
    cw = _cw(128, 128)
    fd = full.to(torch.bfloat16).to(DEV)
    for lo in (0, 32):
        xd = fd[..., lo:lo + 128]  # channel-slice view (x_ld = 192)
        ref = ops.conv2d(_bf(full[..., lo:lo + 128]), cw, relu=True, relu_in=True)
        got = ops.conv2d(xd, cw.to_device(DEV), relu=True, relu_in=True)
        assert _rel(got, ref) < 1e-2
    x = full[..., :128].contiguous()
    mask = torch.randn(2, 12, 14, 128, generator=g)
    ct = _cw(128, 64, kind="transpose", bias=False)
    kw = dict(relu=False, relu_in=True, in_mode="transpose", stride=1, pad=(1, 1), out_hw=(12, 14), use_bias=False)
    ref = ops.conv2d(_bf(x), ct, mask=_bf(mask), **kw)
    got = ops.conv2d(x.to(torch.bfloat16).to(DEV), ct.to_device(DEV), mask=mask.to(torch.bfloat16).to(DEV), **kw)
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("N,H,C,OC,div", [(8, 14, 512, 512, 4), (4, 28, 256, 256, 2), (2, 56, 256, 128, 1),
                                          (3, 9, 64, 24, 3)])
def test_conv_unpool_out_epilogue(native_lib, N, H, C, OC, div):
    """Max-unpool fused into the conv epilogue (unpool_out) == unpool of the plain conv output (the
    plain launch may split K at small M: summation order differs) and == the fp32 reference path."""
    g = torch.Generator().manual_seed(47)
    x = torch.relu(torch.randn(N, H, H, C, generator=g)).to(torch.bfloat16)
    code = torch.randint(0, 4, (N // div, H, H, OC), generator=g, dtype=torch.uint8)
    cw = _cw(OC, C, bias=False)
    cwd = cw.to_device(DEV)
    got = ops.conv2d(x.to(DEV), cwd, relu=True, use_bias=False, unpool_out=code.to(DEV), unpool_div=div)
    plain = ops.conv2d(x.to(DEV), cwd, relu=True, use_bias=False)
    assert got.shape == (N, 2 * H, 2 * H, OC)
    want = ops.unpool_ref(plain, code.to(DEV), div)
    assert _rel(got, want) < 1e-2
    assert ((got != 0) & (want == 0)).sum() == 0  # nothing lands off the switch position
    ref = ops.conv2d(x.float(), cw, relu=True, use_bias=False, unpool_out=code, unpool_div=div)
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C,OC,div", [(4, 224, 224, 64, 64, 4), (2, 64, 96, 128, 128, 2), (3, 48, 32, 64, 120, 1)])
def test_conv_unpool_input(native_lib, N, H, W, C, OC, div):
    """unpool (pooled map + switch codes, input ReLU) -> conv, on whichever kernel the router picks for
    the shape (weight-resident halo kernel, or the materialized unpool + DMA conv), vs the fp32
    reference. (Round 6 removed the opt-in hs16 unpool kernel, DV_HSU: 5.23 vs 4.57 ms on its one
    candidate layer, profiles/layers_r1_hsu_{off,on}.txt.)"""
    g = torch.Generator().manual_seed(53)
    p = torch.randn(N, H // 2, W // 2, C, generator=g)  # signed: the input ReLU matters
    code = torch.randint(0, 4, (N // div, H // 2, W // 2, C), generator=g, dtype=torch.uint8)
    cw = _cw(OC, C, bias=False)
    kw = dict(relu=True, relu_in=True, in_mode="unpool", code_div=div, use_bias=False)
    ref = ops.conv2d(_bf(p), cw, code=code, **kw)
    pd, cd, cwd = p.to(torch.bfloat16).to(DEV), code.to(DEV), cw.to_device(DEV)
    got = ops.conv2d(pd, cwd, code=cd, **kw)
    assert got.shape == (N, H, W, OC) and _rel(got, ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C,OC,dt", [(200, 28, 28, 32, 256, torch.bfloat16), (90, 14, 13, 96, 512, torch.bfloat16),
                                           (300, 20, 20, 64, 256, torch.float16), (120, 36, 36, 64, 128, torch.bfloat16)])
def test_conv_kw3_persistent(native_lib, monkeypatch, N, H, W, C, OC, dt):
    """Persistent KW3 (conv_dma_kw3p_kernel, DV_KW3_VAR=2, the default): several tiles per workgroup
    with a partial last round, odd K-step counts (C = 32 / 96: the LDS stage parity runs across tiles),
    image-row and image boundaries inside tiles, the 512 x 128 tile, a channel-slice output view;
    bias + ReLU and plain. Equal BIT FOR BIT to the LDS-staged KW3 epilogue (DV_KW3_VAR=0: same
    accumulation order, same rounding) and to the fp32 reference up to bf16 rounding."""
    monkeypatch.setenv("DV_KW3", "2")
    monkeypatch.setenv("DV_NO_SPLITK", "1")
    monkeypatch.setenv("DV_NO_KW3_SK", "1")  # whole tiles (stream-K rounds split tiles differently)
    g = torch.Generator().manual_seed(N + C)
    x = torch.randn(N, H, W, C, generator=g).to(dt)
    cw = _cw(OC, C)
    xd, cwd = x.to(DEV), cw.to_device(DEV, dt)
    for relu in (True, False):
        outs = {}
        for var in ("0", "2", "2reg"):  # 2reg: KW3P with the register-transposed 8-B stores (DV_KW3P_EPI=reg)
            monkeypatch.setenv("DV_KW3_VAR", var[0])
            if var == "2reg":
                monkeypatch.setenv("DV_KW3P_EPI", "reg")
            big = torch.full((N, H, W, OC + 8), 7.0, dtype=dt, device=DEV)
            outs[var] = ops.conv2d(xd, cwd, relu=relu, out=big[..., :OC])
            monkeypatch.delenv("DV_KW3P_EPI", raising=False)
            assert bool((big[..., OC:] == 7.0).all()), "wrote past the channel slice"
        assert torch.equal(outs["0"], outs["2"]), relu
        assert torch.equal(outs["0"], outs["2reg"]), relu
        ref = ops.conv2d(x[: min(N, 8)].float(), cw, relu=relu)
        assert _rel(outs["2"][: min(N, 8)], ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C,OC,div,dt", [(600, 14, 14, 64, 256, 4, torch.bfloat16),
                                                (90, 28, 28, 96, 256, 2, torch.bfloat16),
                                                (80, 56, 56, 32, 128, 4, torch.bfloat16),
                                                (131, 10, 12, 32, 512, 1, torch.bfloat16),
                                                (300, 20, 20, 64, 256, 3, torch.float16)])
def test_conv_kw3p_unpool_out(native_lib, monkeypatch, N, H, W, C, OC, div, dt):
    """Persistent KW3 with the LDS-sliced max-unpool-out epilogue (conv_dma_kw3p_kernel<.., UNP>, the
    default for the deconvnet's block{3,4,5}_conv1.down): several tiles per workgroup, tiles crossing
    image rows and images, an M tail (N*H*W not a multiple of the tile), the 512 x 128 tile, code_div
    1..4, odd K-step counts (C = 96). Equal BIT FOR BIT to the non-persistent KW3 workgroup-staged
    unpool epilogue (DV_NO_KW3P_UNPOOL=1: same accumulation order, same rounding), nothing off the
    switch positions, and the fp32 reference up to bf16 rounding."""
    monkeypatch.setenv("DV_KW3", "2")
    monkeypatch.setenv("DV_NO_SPLITK", "1")
    monkeypatch.setenv("DV_NO_KW3_SK", "1")  # whole tiles (stream-K: test_conv_kw3p_stream_k)
    g = torch.Generator().manual_seed(N + W)
    x = torch.relu(torch.randn(N, H, W, C, generator=g)).to(dt)
    code = torch.randint(0, 4, (N // div, H, W, OC), generator=g, dtype=torch.uint8)
    cw = _cw(OC, C, bias=False)
    xd, cwd, cd = x.to(DEV), cw.to_device(DEV, dt), code.to(DEV)
    kw = dict(relu=True, use_bias=False, unpool_out=cd, unpool_div=div)
    got = ops.conv2d(xd, cwd, **kw)
    monkeypatch.setenv("DV_NO_KW3P_UNPOOL", "1")
    base = ops.conv2d(xd, cwd, **kw)
    monkeypatch.delenv("DV_NO_KW3P_UNPOOL")
    assert got.shape == (N, 2 * H, 2 * W, OC)
    assert torch.equal(got, base)
    plain = ops.conv2d(xd, cwd, relu=True, use_bias=False)
    want = ops.unpool_ref(plain, cd, div)
    assert ((got != 0) & (want == 0)).sum() == 0  # nothing lands off the switch position
    n = 2 * div
    ref = ops.conv2d(x[:n].float(), cw, relu=True, use_bias=False, unpool_out=code[: n // div], unpool_div=div)
    assert _rel(got[:n], ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C,OC,div,dt", [(600, 14, 14, 64, 256, 0, torch.bfloat16),
                                                (300, 14, 14, 96, 512, 4, torch.bfloat16),
                                                (80, 56, 56, 32, 128, 2, torch.bfloat16),
                                                (80, 56, 56, 64, 128, 0, torch.bfloat16),
                                                (150, 28, 28, 32, 512, 0, torch.float16),
                                                (700, 14, 14, 32, 256, 1, torch.float16)])
def test_conv_kw3p_stream_k(native_lib, monkeypatch, N, H, W, C, OC, div, dt):
    """Stream-K KW3P (conv_dma_kw3p_kernel<.., SK>: each workgroup a contiguous range of K steps, split
    tiles handed over as fp32 partials with the sc1 / flag protocol): plain (div 0) and unpool-out
    epilogues, 256 x 256 (one and two column groups) and 512 x 128 tiles, odd step counts (C = 96).
    Against the whole-tile kernel (DV_NO_KW3_SK=1): equal up to the one extra fp32 rounding of a split
    tile's sum (a few bf16 ulps at most), and against the fp32 reference."""
    monkeypatch.setenv("DV_NO_SPLITK", "1")
    g = torch.Generator().manual_seed(N + C + OC)
    x = torch.relu(torch.randn(N, H, W, C, generator=g)).to(dt)
    cw = _cw(OC, C, bias=div == 0)
    xd, cwd = x.to(DEV), cw.to_device(DEV, dt)
    kw = dict(relu=True, use_bias=div == 0)
    code = None
    if div:
        code = torch.randint(0, 4, (N // div, H, W, OC), generator=g, dtype=torch.uint8)
        kw.update(unpool_out=code.to(DEV), unpool_div=div)
    got = ops.conv2d(xd, cwd, **kw)
    monkeypatch.setenv("DV_NO_KW3_SK", "1")
    whole = ops.conv2d(xd, cwd, **kw)
    monkeypatch.delenv("DV_NO_KW3_SK")
    assert got.shape == whole.shape
    d = (got.float() - whole.float()).abs()
    assert float(d.max()) <= 2 ** -6 * float(whole.float().abs().max()), float(d.max())
    assert float((d > 0).float().mean()) < 0.05  # only the split tiles' rounding differs
    n = 2 * max(div, 1)
    if div:
        kw_ref = dict(relu=True, use_bias=False, unpool_out=code[: n // div], unpool_div=div)
        ref = ops.conv2d(x[:n].float(), cw, **kw_ref)
    else:
        ref = ops.conv2d(x[:n].float(), cw, relu=True)
    assert _rel(got[:n], ref) < 1e-2
    ntail = 2 * max(div, 1)  # the last images: the last workgroups' ranges and split tiles
    if div:
        ref = ops.conv2d(x[-ntail:].float(), cw, relu=True, use_bias=False, unpool_out=code[-(ntail // div):],
                         unpool_div=div)
    else:
        ref = ops.conv2d(x[-ntail:].float(), cw, relu=True)
    assert _rel(got[-ntail:], ref) < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,W,C,OC", [(5, 7, 7, 64, 256), (3, 14, 13, 96, 512), (2, 28, 28, 256, 256), (1, 9, 1, 32, 256),
                                        (4, 10, 9, 64, 128), (2, 56, 56, 256, 128)])
def test_conv_kw3_shared_taps(native_lib, monkeypatch, dt, N, H, W, C, OC):
    """3x3 convs whose three kw taps share one staged A tile (conv_dma_kw3_kernel), forced on small
    shapes so most tiles cross image rows and images: bf16/fp16 out, f32 out, accumulate, residual
    + emask epilogues and the fused unpool-out epilogue, vs the fp32 reference."""
    monkeypatch.setenv("DV_KW3", "2")
    monkeypatch.setenv("DV_NO_SPLITK", "1")
    g = torch.Generator().manual_seed(59)
    x = torch.randn(N, H, W, C, generator=g).to(dt)
    cw = _cw(OC, C)
    xd, cwd = x.to(DEV), cw.to_device(DEV, dt)
    ref = ops.conv2d(x.float(), cw, relu=True)
    got = ops.conv2d(xd, cwd, relu=True)
    assert got.dtype == dt and _rel(got, ref) < 1e-2
    if dt == torch.bfloat16:
        ref = ops.conv2d(x.float(), cw, relu=False, epilogue="f32")
        assert _rel(ops.conv2d(xd, cwd, relu=False, epilogue="f32"), ref) < 1e-3
        base = torch.randn(N, H, W, OC, generator=g).to(dt)
        out_d = base.to(DEV)
        ops.conv2d(xd, cwd, relu=False, out=out_d, accumulate=True)
        out_r = base.float().clone()
        ops.conv2d(x.float(), cw, relu=False, out=out_r, accumulate=True)
        assert _rel(out_d, out_r) < 1e-2
        if H % 2 == 0 and W % 2 == 0:
            code = torch.randint(0, 4, (N, H, W, OC), generator=g, dtype=torch.uint8)
            got = ops.conv2d(xd, cwd, relu=True, use_bias=False, unpool_out=code.to(DEV))
            ref = ops.conv2d(x.float(), cw, relu=True, use_bias=False, unpool_out=code)
            assert _rel(got, ref) < 1e-2
    res = torch.randn(N, H, W, OC, generator=g).to(dt)
    em = torch.randn(N, H, W, OC, generator=g).to(dt)
    ref = ops.conv2d(x.float(), cw, relu=True, res=res.float(), emask=em.float())
    got = ops.conv2d(xd, cwd, relu=True, res=res.to(DEV), emask=em.to(DEV))
    assert _rel(got, ref) < 1e-2


def test_conv_unpool_gather(native_lib):
    g = torch.Generator().manual_seed(5)
    K = 2
    p = torch.randn(4, 6, 7, 64, generator=g)  # B*K signals at pooled res
    code = torch.randint(0, 4, (2, 6, 7, 64), generator=g, dtype=torch.uint8)
    cw = _cw(32, 64, bias=False)
    kw = dict(relu=True, relu_in=True, in_mode="unpool", code=code, code_div=K, use_bias=False)
    ref = ops.conv2d(_bf(p), cw, **kw)
    got = ops.conv2d(p.to(torch.bfloat16).to(DEV), cw.to_device(DEV),
                     **{**kw, "code": code.to(DEV)})
    assert got.shape == (4, 12, 14, 32) and _rel(got, ref) < 1e-2


def test_conv_mask_and_transpose(native_lib, conv_impl):
    g = torch.Generator().manual_seed(6)
    dy = torch.randn(2, 8, 9, 64, generator=g)
    mask = torch.randn(2, 8, 9, 64, generator=g)
    cw = _cw(64, 32, 3, 3, kind="transpose", bias=False)  # forward conv 32 -> 64, its dgrad
    for s, pad in [(2, (0, 0)), (2, (1, 1)), (1, (1, 1))]:
        out_hw = ((8 - 1) * s - 2 * pad[0] + 3, (9 - 1) * s - 2 * pad[1] + 3)
        kw = dict(relu=False, in_mode="transpose", stride=s, pad=pad, out_hw=out_hw, use_bias=False)
        ref = ops.conv2d(_bf(dy), cw, mask=_bf(mask), **kw)
        got = ops.conv2d(dy.to(torch.bfloat16).to(DEV), cw.to_device(DEV),
                         mask=mask.to(torch.bfloat16).to(DEV), **kw)
        assert got.shape == ref.shape and _rel(got, ref) < 1e-2, (s, pad)
    # transpose == autograd input-gradient of the strided forward conv
    x = torch.randn(1, 11, 11, 32, generator=g, requires_grad=True)
    wf = cw.w_oihw
    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), wf, stride=2)
    gy = torch.randn_like(y)
    (gx,) = torch.autograd.grad(y, x, gy)
    got = ops.conv2d(gy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).to(DEV), cw.to_device(DEV),
                     relu=False, in_mode="transpose", stride=2, pad=(0, 0), out_hw=(11, 11), use_bias=False)
    assert _rel(got, gx) < 2e-2


@pytest.mark.parametrize("N,H,W,C,OC,unpool,epi", [(2, 20, 40, 64, 64, False, "bf16"), (1, 18, 34, 64, 64, True, "bf16"),
                                                    (3, 16, 64, 64, 3, False, "f32"), (1, 40, 30, 64, 48, True, "bf16"),
                                                    (2, 12, 12, 64, 16, True, "f32"), (5, 33, 17, 64, 3, False, "f32"),
                                                    (3, 48, 72, 64, 64, True, "bf16"), (2, 16, 32, 64, 64, True, "bf16"),
                                                    (4, 10, 6, 64, 64, True, "bf16"), (2, 224, 224, 64, 3, False, "f32"),
                                                    (2, 9, 64, 64, 3, False, "bf16"), (1, 7, 100, 64, 16, False, "f32"),
                                                    (1, 3, 36, 64, 5, False, "f32")])
def test_conv_halo_kernel(native_lib, N, H, W, C, OC, unpool, epi):
    from deconv_api_amd.ops import conv as Cm

    g = torch.Generator().manual_seed(13)
    cw = _cw(OC, C, bias=not unpool)
    kw = dict(relu=True, relu_in=True, epilogue=epi, use_bias=not unpool)
    if unpool:
        x = torch.randn(N, H // 2, W // 2, C, generator=g)
        code = torch.randint(0, 4, (N, H // 2, W // 2, C), generator=g, dtype=torch.uint8)
        kw.update(in_mode="unpool", code=code)
    else:
        x = torch.randn(N, H, W, C, generator=g)
    ref = ops.conv2d(_bf(x), cw, **kw)
    if unpool:
        kw["code"] = code.to(DEV)
    old = Cm.get_policy()
    Cm.set_policy(impl="halo")
    try:
        got = ops.conv2d(x.to(torch.bfloat16).to(DEV), cw.to_device(DEV), **kw)
    finally:
        Cm.set_policy(**old)
    assert got.shape == ref.shape and _rel(got, ref) < 1e-2
    if unpool and OC == 64 and epi == "bf16":  # v2 (register-resident weights) vs v1: same math
        import os

        os.environ["DV_HALO_V1"] = "1"
        try:
            Cm.set_policy(impl="halo")
            v1 = ops.conv2d(x.to(torch.bfloat16).to(DEV), cw.to_device(DEV), **kw)
        finally:
            del os.environ["DV_HALO_V1"]
            Cm.set_policy(**old)
        assert _rel(got, v1) < 1e-2


def test_conv_channel_slices(native_lib):
    """input/output as channel-slice views of wider tensors (concat without copies)."""
    g = torch.Generator().manual_seed(7)
    big = torch.randn(2, 9, 9, 96, generator=g).to(torch.bfloat16)
    x = big[..., 32:96]
    cw = _cw(40, 64)
    ref = ops.conv2d(x.float(), cw)
    out = torch.zeros(2, 9, 9, 128, dtype=torch.bfloat16, device=DEV)
    ops.conv2d(big.to(DEV)[..., 32:96], cw.to_device(DEV), out=out[..., 16:56])
    assert _rel(out[..., 16:56], ref) < 1e-2
    assert out[..., :16].abs().sum() == 0 and out[..., 56:].abs().sum() == 0


def test_channel_sum_topk(native_lib):
    g = torch.Generator().manual_seed(8)
    x = torch.relu(torch.randn(5, 14, 14, 512, generator=g)).to(torch.bfloat16)
    s_ref = x.float().sum(dim=(1, 2))
    s = ops.channel_sum(x.to(DEV))
    torch.testing.assert_close(s.cpu(), s_ref, rtol=1e-4, atol=1e-2)
    v = torch.randint(-3, 4, (7, 1000), generator=g).float()
    v[3] = -1.0
    i_ref, v_ref = ops.topk_positive(v, 8)
    i_got, v_got = ops.topk_positive(v.to(DEV), 8)
    assert torch.equal(i_got.cpu(), i_ref) and torch.equal(v_got.cpu(), v_ref)
    big = torch.randn(3, 25088, generator=g)
    assert torch.equal(ops.topk_positive(big.to(DEV), 8)[0].cpu(), ops.topk_positive(big, 8)[0])


def test_seed_deconv(native_lib):
    g = torch.Generator().manual_seed(9)
    S = torch.relu(torch.randn(6, 14, 14, generator=g))
    f = torch.tensor([0, 5, 511, -1, 7, 3], dtype=torch.int32)
    wt = torch.randn(512, 3, 3, 512, generator=g).to(torch.bfloat16) * 0.05
    ref = ops.seed_deconv3x3(S, f, wt)
    got = ops.seed_deconv3x3(S.to(DEV), f.to(DEV), wt.to(DEV))
    assert _rel(got, ref) < 1e-2
    assert got[3].abs().sum() == 0
    # an out-of-range filter index is clamped to F - 1 inside the kernel (no host clamp launch)
    f_hi = f.clone()
    f_hi[2] = 4096
    got_hi = ops.seed_deconv3x3(S.to(DEV), f_hi.to(DEV), wt.to(DEV))
    assert torch.equal(got_hi, got)
    # a block5-sized map (B*K = 1024 signals x 14^2 x 512): 32-bit index math over 12.8 M chunks
    Sb = torch.relu(torch.randn(1024, 14, 14, generator=g))
    fb = torch.randint(-1, 512, (1024,), generator=g, dtype=torch.int32)
    gb = ops.seed_deconv3x3(Sb.to(DEV), fb.to(DEV), wt.to(DEV))
    for i in (0, 511, 1023):
        assert _rel(gb[i:i + 1], ops.seed_deconv3x3(Sb[i:i + 1], fb[i:i + 1], wt)) < 1e-2
    # the one-workgroup-per-signal small-map kernel (default at <= 4096 px) == the grid-stride kernel
    os.environ["DV_SEED_V1"] = "1"
    try:
        g1 = ops.seed_deconv3x3(Sb.to(DEV), fb.to(DEV), wt.to(DEV))
        w64 = wt[..., :64].contiguous()
        h1 = ops.seed_deconv3x3(S.to(DEV), f.to(DEV), w64.to(DEV))
    finally:
        del os.environ["DV_SEED_V1"]
    # (same taps in the same order; the compilers' FMA contraction differs between the two bodies, so
    # a value may differ in its last bf16 bit)
    assert _rel(g1, gb) < 4e-3
    assert _rel(h1, ops.seed_deconv3x3(S.to(DEV), f.to(DEV), w64.to(DEV))) < 4e-3  # Cin 64: 32 pixel groups


@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("mode,batch_topk", [("all", "per_image"), ("max", "per_image"), ("max", "global"),
                                             ("all", "global")])
def test_seed_map(native_lib, pool, mode, batch_topk):
    """HIP seed-map kernel vs the fp32 torch gather/amax/mask(/unpool) reference (exact)."""
    g = torch.Generator().manual_seed(11)
    B, H, W, C, K = 3, 7, 9, 64, 4
    out4 = torch.relu(torch.randint(-2, 5, (B, H, W, C), generator=g).float()).to(torch.bfloat16)  # ties
    if batch_topk == "global":
        idx = torch.tensor([[5, 63, 0, -1]], dtype=torch.int32).expand(B, K).contiguous()
    else:
        idx = torch.randint(0, C, (B, K), generator=g, dtype=torch.int32)
        idx[1, 2] = -1
    code = torch.randint(0, 4, (B, H, W, C), generator=g, dtype=torch.uint8) if pool else None
    ref = ops.seed_map(out4, idx, mode, batch_topk, code)
    got = ops.seed_map(out4.to(DEV), idx.to(DEV), mode, batch_topk, None if code is None else code.to(DEV))
    assert got.shape == ref.shape == (B * K, H * (2 if pool else 1), W * (2 if pool else 1))
    assert torch.equal(got.cpu(), ref)


def test_deprocess_mosaic(native_lib):
    g = torch.Generator().manual_seed(10)
    r = torch.relu(torch.randn(8, 224, 224, 3, generator=g)) * 3
    ref = ops.deprocess_mosaic(r)
    got = ops.deprocess_mosaic(r.to(DEV)).cpu()
    d = (got.int() - ref.int()).abs()
    assert got.shape == (2, 448, 448, 3) and d.max() <= 1 and (d > 0).float().mean() < 1e-3
    # precomputed per-image statistics (as the final conv's epilogue supplies them) give the same mosaic
    rd = r.to(DEV).reshape(2, -1).double()
    st = torch.stack([rd.sum(1), (rd * rd).sum(1)], 1).contiguous()
    got2 = ops.deprocess_mosaic(r.to(DEV), stats=st).cpu()
    assert (got2.int() - got.int()).abs().max() <= 1


@pytest.mark.parametrize("N,H,W,stats_div", [(8, 32, 64, 4), (4, 9, 40, 2), (8, 224, 224, 4)])
def test_conv_stream_stats(native_lib, N, H, W, stats_div):
    """The final 64 -> 3 conv-down's epilogue statistics (per group of stats_div images) equal the
    fp64 sums of its own fp32 output, on the row-streaming kernel and on the generic fallback pass."""
    from deconv_api_amd.ops import conv as Cm

    g = torch.Generator().manual_seed(12)
    x = torch.relu(torch.randn(N, H, W, 64, generator=g)).to(torch.bfloat16).to(DEV)
    cw = _cw(3, 64, bias=False).to_device(DEV)
    old = Cm.get_policy()
    for impl in ("auto", "dma"):
        Cm.set_policy(impl=impl)
        try:
            st = torch.full((N // stats_div, 2), 7.0, dtype=torch.float64, device=DEV)
            y = ops.conv2d(x, cw, relu=True, relu_in=True, epilogue="f32", use_bias=False, stats=st,
                           stats_div=stats_div)
        finally:
            Cm.set_policy(**old)
        yd = y.reshape(N // stats_div, -1).double()
        ref = torch.stack([yd.sum(1), (yd * yd).sum(1)], 1)
        assert torch.allclose(st, ref, rtol=1e-9, atol=1e-6), impl


def test_resize_preprocess_exact(native_lib):
    rng = np.random.default_rng(0)
    for hs, ws in [(300, 400), (448, 448), (224, 224), (100, 57), (1000, 224)]:
        img = rng.integers(0, 256, size=(hs, ws, 3), dtype=np.uint8)
        out = torch.empty(224, 224, 8, dtype=torch.bfloat16, device=DEV)
        ops.resize_preprocess(torch.from_numpy(img).to(DEV), out)
        ref = ops.preprocess_ref(ops.resize_u8_ref(img))
        assert torch.equal(out.cpu(), ref), (hs, ws)


def test_pool_unpool_standalone(native_lib):
    g = torch.Generator().manual_seed(11)
    x = torch.relu(torch.randint(-2, 3, (2, 12, 10, 64), generator=g).float()).to(torch.bfloat16)  # ties
    v, c = ops.maxpool2x2(x.to(DEV))
    rv, rc = ops.maxpool2x2(x)
    assert torch.equal(v.cpu(), rv) and torch.equal(c.cpu(), rc)
    # signed values, -inf windows and a 256-channel map (vectorized kernel), and C = 12 (scalar kernel)
    for shape in ((3, 28, 28, 256), (2, 6, 8, 12)):
        y = torch.randn(*shape, generator=g).to(torch.bfloat16)
        y[0, :2, :2] = float("-inf")
        yv, yc = ops.maxpool2x2(y.to(DEV))
        ry, rcy = ops.maxpool2x2(y)
        assert torch.equal(yv.cpu(), ry) and torch.equal(yc.cpu(), rcy), shape
    p = torch.randn(4, 6, 5, 64, generator=g).to(torch.bfloat16)
    u = ops.unpool2x2(p.to(DEV), c, code_div=2, relu=True)
    assert torch.equal(u.cpu(), ops.unpool2x2(p, c.cpu(), code_div=2, relu=True))


def test_conv_deterministic(native_lib):
    g = torch.Generator().manual_seed(12)
    x = torch.randn(4, 28, 28, 256, generator=g).to(torch.bfloat16).to(DEV)
    cw = _cw(512, 256).to_device(DEV)
    a = ops.conv2d(x, cw)
    b = ops.conv2d(x, cw)
    assert torch.equal(a, b)


@pytest.mark.parametrize("N,H,W,C,OC,stride", [(2, 16, 16, 64, 64, 1), (1, 9, 7, 128, 256, 1),
                                               (2, 17, 13, 24, 200, 1), (2, 15, 15, 64, 128, 2)])
def test_conv_fp16_fwd_mask_transpose(native_lib, conv_impl, N, H, W, C, OC, stride):
    """fp16 storage + f16 MFMA (DeepDream config 5): forward, ReLU-masked dgrad and strided
    transposed dgrad vs the fp32 reference on fp16-rounded operands."""
    g = torch.Generator().manual_seed(5)
    h = lambda t: t.to(torch.float16).float()  # noqa: E731
    x = h(torch.randn(N, H, W, C, generator=g))
    w = h(torch.randn(OC, C, 3, 3, generator=g) / np.sqrt(9 * C))
    b = h(torch.randn(OC, generator=g) * 0.1)
    cw = ConvWeights(w, b, "fwd")
    cwd = cw.to_device(DEV, torch.float16)
    ref = ops.conv2d(x, cw, stride=stride)
    got = ops.conv2d(x.to(torch.float16).to(DEV), cwd, stride=stride)
    assert got.dtype == torch.float16 and _rel(got, ref) < 4e-3
    # dgrad through the ReLU: masked, transposed gather (stride > 1) or flipped kernel (stride 1)
    gy = h(torch.randn(*ref.shape, generator=g))
    ct = ConvWeights(w, None, "transpose")
    if stride == 1:
        wd = pad_channels_oihw(w.flip(2, 3).transpose(0, 1).contiguous())
        cb = ConvWeights(wd, None, "fwd")
        kw = dict(stride=1, relu=False, mask=None, use_bias=False)
    else:
        cb = ct
        kw = dict(stride=stride, pad=1, relu=False, in_mode="transpose", out_hw=(H, W), use_bias=False)
    for use_mask in (False, True):
        m = ref if use_mask else None
        kw["mask"] = m
        r = ops.conv2d(gy, cb, **kw)
        kw["mask"] = None if m is None else m.to(torch.float16).to(DEV)
        o = ops.conv2d(gy.to(torch.float16).to(DEV), cb.to_device(DEV, torch.float16), **kw)
        assert _rel(o, r) < 4e-3, (stride, use_mask)


def test_pool_fp16(native_lib):
    from deconv_api_amd.ops.autograd import avg_pool, max_pool

    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 13, 11, 24, generator=g).to(torch.float16).float()
    for fn in (max_pool, avg_pool):
        xc = x.clone().requires_grad_(True)
        yc = fn(xc, 3, 2, 1)
        gy = torch.randn_like(yc).to(torch.float16).float()
        (gc,) = torch.autograd.grad(yc, xc, gy)
        xd = x.to(torch.float16).cuda().requires_grad_(True)
        yd = fn(xd, 3, 2, 1)
        (gd,) = torch.autograd.grad(yd, xd, gy.to(torch.float16).cuda())
        assert yd.dtype == torch.float16 and _rel(yd, yc) < 2e-3 and _rel(gd, gc) < 2e-3


@pytest.mark.parametrize("H,W,pad", [(13, 11, 1), (13, 11, 0), (14, 16, 0), (9, 10, 1), (3, 3, 0), (35, 35, 0)])
def test_maxpool_3x3_s2_bwd(native_lib, H, W, pad):
    """3x3 / stride-2 max-pool gradient (the unrolled 2 x 2 window path of maxpool_bwd_kernel) vs the
    CPU path, with ties (first max wins) from a coarse value grid, odd / even sizes, pad 0 and 1."""
    from deconv_api_amd.ops.autograd import max_pool

    g = torch.Generator().manual_seed(H * 31 + W + pad)
    x = (torch.randint(-4, 5, (3, H, W, 16), generator=g).float() / 4).to(torch.bfloat16).float()
    xc = x.clone().requires_grad_(True)
    yc = max_pool(xc, 3, 2, pad)
    gy = torch.randn_like(yc).to(torch.bfloat16).float()
    (gc,) = torch.autograd.grad(yc, xc, gy)
    xd = x.to(torch.bfloat16).cuda().requires_grad_(True)
    yd = max_pool(xd, 3, 2, pad)
    (gd,) = torch.autograd.grad(yd, xd, gy.to(torch.bfloat16).cuda())
    assert torch.equal(yd.float().cpu(), yc.detach())
    assert _rel(gd, gc) < 1e-2


@pytest.mark.parametrize("s,pad", [(1, 1), (1, 0), (2, 0), (2, 1)])
@pytest.mark.parametrize("kind", ["max", "avg"])
def test_pool_bwd_unrolled_bit_identical(native_lib, monkeypatch, kind, s, pad):
    """The unrolled 3x3 backward paths (max: stride 2, avg: stride 1) against the generic window loop
    (DV_NO_POOL_UNROLL=1, read per call): bit-identical gradients; and both against the CPU path."""
    from deconv_api_amd.ops.autograd import avg_pool, max_pool

    fn = max_pool if kind == "max" else avg_pool
    g = torch.Generator().manual_seed(7 * s + pad)
    x = (torch.randint(-4, 5, (2, 17, 12, 24), generator=g).float() / 4).to(torch.bfloat16).float()
    xc = x.clone().requires_grad_(True)
    yc = fn(xc, 3, s, pad)
    gy = torch.randn_like(yc).to(torch.bfloat16).float()
    (gc,) = torch.autograd.grad(yc, xc, gy)

    def dev_grad():
        xd = x.to(torch.bfloat16).cuda().requires_grad_(True)
        (gd,) = torch.autograd.grad(fn(xd, 3, s, pad), xd, gy.to(torch.bfloat16).cuda())
        return gd

    fast = dev_grad()
    monkeypatch.setenv("DV_NO_POOL_UNROLL", "1")
    slow = dev_grad()
    assert torch.equal(fast, slow)
    assert _rel(fast, gc) < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C,OC,N,H", [(64, 16, 3, 20), (64, 64, 2, 33), (128, 128, 2, 17), (256, 512, 1, 14),
                                      (512, 256, 4, 7), (16, 8, 2, 40)])
def test_conv_masked_dgrad_shapes(native_lib, conv_impl, dt, C, OC, N, H):
    """ReLU-masked A operand over every tile config of both kernels, with +0/-0/negative mask values
    and rows spanning images."""
    g = torch.Generator().manual_seed(C + OC + H)
    r = lambda t: t.to(dt).float()  # noqa: E731
    x = r(torch.randn(N, H, H + 3, C, generator=g))
    m = torch.randn(N, H, H + 3, C, generator=g).clamp_min(0)
    m[m == 0] = torch.where(torch.rand(int((m == 0).sum()), generator=g) < 0.5, 0.0, -0.0)
    m = r(m) - r(torch.rand(N, H, H + 3, C, generator=g) < 0.05).float() * 3.0  # a few negatives
    cw = ConvWeights(r(torch.randn(OC, C, 3, 3, generator=g) / np.sqrt(9 * C)), None, "fwd")
    ref = ops.conv2d(x, cw, relu=False, mask=r(m), use_bias=False)
    got = ops.conv2d(x.to(dt).to(DEV), cw.to_device(DEV, dt), relu=False, mask=m.to(dt).to(DEV), use_bias=False)
    assert got.dtype == dt and _rel(got, ref) < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C,OC,N,H", [(64, 256, 2, 19), (256, 64, 3, 8), (128, 512, 1, 12), (512, 2048, 2, 7)])
def test_conv_residual_relu_epilogue(native_lib, dt, C, OC, N, H):
    """Fused ResNet block tail: ReLU(conv1x1(x) + bias + res) in the LDS-DMA epilogue."""
    g = torch.Generator().manual_seed(C * 7 + OC)
    r = lambda t: t.to(dt).float()  # noqa: E731
    x = r(torch.randn(N, H, H, C, generator=g))
    res = r(torch.randn(N, H, H, OC, generator=g))
    cw = ConvWeights(r(torch.randn(OC, C, 1, 1, generator=g) / np.sqrt(C)), r(torch.randn(OC, generator=g)), "fwd")
    ref = ops.conv2d(x, cw, relu=True, res=res)
    assert torch.allclose(ref, (ops.conv2d(x, cw, relu=False) + res).clamp_min(0), atol=1e-5)
    got = ops.conv2d(x.to(dt).to(DEV), cw.to_device(DEV, dt), relu=True, res=res.to(dt).to(DEV))
    assert got.dtype == dt and _rel(got, ref) < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_sumsq_core_fwd_bwd(native_lib, dt):
    from deconv_api_amd.ops.autograd import sumsq_core

    g = torch.Generator().manual_seed(9)
    for shape, b in [((3, 17, 23, 64), 2), ((2, 70, 70, 512), 2), ((1, 6, 6, 8), 1)]:
        x = torch.randn(*shape, generator=g).to(dt).float()
        xc = x.clone().requires_grad_(True)
        lc = sumsq_core(xc, b)
        gl = torch.rand(shape[0], generator=g)
        (gc,) = torch.autograd.grad(lc, xc, gl)
        xd = x.to(dt).to(DEV).requires_grad_(True)
        ld = sumsq_core(xd, b)
        (gd,) = torch.autograd.grad(ld, xd, gl.to(DEV))
        assert ld.dtype == torch.float32 and torch.allclose(ld.cpu(), lc, rtol=1e-5)
        assert gd.dtype == dt and _rel(gd, gc) < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C,OC,k,ld", [(64, 147, 1, 152), (64, 64, 3, 64), (128, 200, 3, 208), (32, 3, 3, 8)])
def test_conv_vector_epilogue_emask_partial_chunks(native_lib, dt, C, OC, k, ld):
    """LDS-staged epilogue: output-mask (emask) without residual, row stride != OC, OC % 8 != 0
    (element-wise tail chunk), accumulate into an existing output."""
    g = torch.Generator().manual_seed(OC + k)
    r = lambda t: t.to(dt).float()  # noqa: E731
    N, H = 2, 13
    x = r(torch.randn(N, H, H, C, generator=g))
    cw = ConvWeights(r(torch.randn(OC, C, k, k, generator=g) / np.sqrt(C * k * k)), r(torch.randn(OC, generator=g)),
                     "fwd")
    em = r(torch.randn(N, H, H, OC, generator=g))
    base = r(torch.randn(N, H, H, ld, generator=g))
    ref = ops.conv2d(x, cw, relu=False) * (em > 0)
    buf = base.to(dt).to(DEV)
    got = ops.conv2d(x.to(dt).to(DEV), cw.to_device(DEV, dt), relu=False, out=buf[..., :OC],
                     emask=em.to(dt).to(DEV))
    assert _rel(got, ref) < 1e-2
    assert torch.equal(buf[..., OC:].cpu(), base[..., OC:].to(dt))  # padding columns untouched
    acc = ops.conv2d(x, cw, relu=True) + base[..., :OC]
    buf = base.to(dt).to(DEV)
    got = ops.conv2d(x.to(dt).to(DEV), cw.to_device(DEV, dt), relu=True, out=buf[..., :OC], accumulate=True)
    assert _rel(got, acc) < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,C,OC,epi,relu", [(1, 7, 512, 512, "bf16", True), (2, 4, 256, 1000, "f32", False),
                                               (4, 2, 1024, 64, "bf16", False), (1, 14, 512, 16, "f32", True)])
def test_conv_splitk_small_m(native_lib, monkeypatch, dt, N, H, C, OC, epi, relu):
    """Small-M convs take the split-K path (fp32 partials + reduce epilogue); compare with the fp32
    reference and with the unsplit kernel."""
    if dt == torch.float16 and epi == "f32":
        pytest.skip("fp16 path has 16-bit epilogues only")
    g = torch.Generator().manual_seed(C + OC)
    r = lambda t: t.to(dt).float()  # noqa: E731
    x = r(torch.randn(N, H, H, C, generator=g))
    cw = ConvWeights(r(torch.randn(OC, C, 3, 3, generator=g) / np.sqrt(9 * C)), r(torch.randn(OC, generator=g)), "fwd")
    ref = ops.conv2d(x, cw, relu=relu, epilogue=epi)
    dw = cw.to_device(DEV, dt)
    got = ops.conv2d(x.to(dt).to(DEV), dw, relu=relu, epilogue=epi)
    assert _rel(got, ref) < 1e-2
    monkeypatch.setenv("DV_NO_SPLITK", "1")
    whole = ops.conv2d(x.to(dt).to(DEV), dw, relu=relu, epilogue=epi)
    assert _rel(got, whole) < 1e-2


def test_softmax_rows(native_lib):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(5, 1000, generator=g) * 4
    got = ops.softmax_rows(x.to(DEV))
    assert torch.allclose(got.cpu(), torch.softmax(x, -1), rtol=1e-5, atol=1e-7)


def test_dense_layers_as_mfma_gemm(native_lib):
    """Dense up (fused bias + ReLU / softmax) and down (y . W^T, ReLU of the layer below) on the
    MFMA kernel match the fp32 CPU engine for dense targets."""
    from deconv_api_amd.engine.deconvnet import DeconvNet
    from deconv_api_amd.models.vgg16 import VGG16, vgg16_specs

    m = VGG16.random(0, specs=vgg16_specs(width_div=8, image_size=32, fc=64, classes=24))
    rt = m.build(DEV, torch.bfloat16)
    assert all(d.up is not None and d.down is not None for d in rt.dense.values())
    cpu = DeconvNet(m.build("cpu", torch.float32))
    gpu = DeconvNet(m.build(DEV, torch.bfloat16))
    x = torch.randn(3, 32, 32, 8, generator=torch.Generator().manual_seed(1)) * 50
    x[..., 3:] = 0
    x = x.to(torch.bfloat16).float()
    for layer in ("fc1", "fc2", "predictions"):
        sg, sc = gpu.forward(x.to(torch.bfloat16).to(DEV), layer), cpu.forward(x, layer)
        assert _rel(sg.out, sc.out) < 3e-2, layer
        idx, _ = gpu.select_filters(sg.out, 4)
        rg, rc = gpu.backward(sg, idx).cpu(), cpu.backward(sc, idx.cpu())
        a, b = rg.double().flatten(), rc.double().flatten()
        assert float(a @ b / (a.norm() * b.norm() + 1e-30)) > 0.98, layer


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C,OC,H,W,pad,use_emask", [
    (32, 32, 75, 75, 0, False),   # InceptionV3 conv2d_2 forward ('valid'), one channel chunk (NB1)
    (32, 32, 73, 73, 2, True),    # its input gradient: full pad, ReLU-masked output
    (64, 32, 73, 71, 1, True),    # conv2d_3 input gradient (64 -> 32), ragged tiles
    (32, 64, 73, 73, 1, False),   # conv2d_3 forward
    (64, 64, 64, 64, 1, True),    # hs16 (16-multiple output) with an output mask
    (64, 128, 66, 66, 0, False),  # hs16, 'valid' (64 x 64 output)
    (96, 96, 70, 67, 1, True),    # OC 96 -> 128-channel tile, 3 chunks, ragged
    (96, 192, 73, 73, 0, False),  # InceptionV3 conv2d_5 (channels padded 80 -> 96): OCpad 192, two launches
    (192, 96, 71, 71, 2, True),   # its input gradient (full pad, ReLU-masked)
])
def test_conv_halo_stream_pad_emask(native_lib, monkeypatch, dt, C, OC, H, W, pad, use_emask):
    """Halo-stream 3x3 kernels with pad 0/1/2 (output H + 2 pad - 2), ragged tiles and the emask
    epilogue (ReLU-masked input gradients) against the fp32 reference and the LDS-DMA kernel."""
    g = torch.Generator().manual_seed(C * 3 + OC + H + pad)
    r = lambda t: t.to(dt).float()  # noqa: E731
    N = 2
    x = r(torch.randn(N, H, W, C, generator=g))
    cw = ConvWeights(r(torch.randn(OC, C, 3, 3, generator=g) / np.sqrt(9 * C)), r(torch.randn(OC, generator=g)), "fwd")
    OH, OW = H + 2 * pad - 2, W + 2 * pad - 2
    em = r(torch.randn(N, OH, OW, OC, generator=g)) if use_emask else None
    relu = not use_emask
    ref = ops.conv2d(x, cw, pad=pad, relu=relu, emask=em)
    assert ref.shape == (N, OH, OW, OC)
    dw = cw.to_device(DEV, dt)
    emd = em.to(dt).to(DEV) if use_emask else None
    got = ops.conv2d(x.to(dt).to(DEV), dw, pad=pad, relu=relu, emask=emd)
    assert got.dtype == dt and _rel(got, ref) < 1e-2
    if use_emask:
        assert bool(((got.float().cpu() != 0) & (em <= 0)).sum() == 0)
    monkeypatch.setenv("DV_HS16_EPI", "reg")  # hs16: register-layout 8-B stores, bit-identical
    assert torch.equal(got, ops.conv2d(x.to(dt).to(DEV), dw, pad=pad, relu=relu, emask=emd))
    monkeypatch.delenv("DV_HS16_EPI")
    monkeypatch.setenv("DV_NO_HS", "1")
    dma = ops.conv2d(x.to(dt).to(DEV), dw, pad=pad, relu=relu, emask=emd)
    assert _rel(dma, ref) < 1e-2


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("mode", ["emask", "accumulate", "res", "relu"])
def test_conv_splitk_full_epilogue(native_lib, dt, mode):
    """Split-K partials + the reduce kernel with the full epilogue (emask / accumulate / residual /
    ReLU), forced on the small-problem 64x64 tile (as DeepDream's small octaves run it)."""
    g = torch.Generator().manual_seed(len(mode))
    r = lambda t: t.to(dt).float()  # noqa: E731
    N, H, C, OC = 4, 9, 160, 96
    x = r(torch.randn(N, H, H, C, generator=g))
    cw = ConvWeights(r(torch.randn(OC, C, 3, 3, generator=g) / np.sqrt(9 * C)), r(torch.randn(OC, generator=g)), "fwd")
    em = r(torch.randn(N, H, H, OC, generator=g))
    base = r(torch.randn(N, H, H, OC, generator=g))
    kw = {"emask": dict(relu=False, emask=em), "accumulate": dict(relu=True), "res": dict(relu=True, res=base),
          "relu": dict(relu=True)}[mode]
    if mode == "accumulate":
        ref = ops.conv2d(x, cw, relu=True) + base
    else:
        ref = ops.conv2d(x, cw, **kw)
    dev_kw = {k: (v.to(dt).to(DEV) if torch.is_tensor(v) else v) for k, v in kw.items()}
    lib = native_lib
    for ks in (1, 2, 4):
        lib.dma_tune(8, ks)
        try:
            if mode == "accumulate":
                out = base.to(dt).to(DEV)
                got = ops.conv2d(x.to(dt).to(DEV), cw.to_device(DEV, dt), out=out, accumulate=True, **dev_kw)
            else:
                got = ops.conv2d(x.to(dt).to(DEV), cw.to_device(DEV, dt), **dev_kw)
        finally:
            lib.dma_tune(0, 0)
        assert _rel(got, ref) < 1e-2, (mode, ks)
        if mode == "emask":
            assert bool(((got.float().cpu() != 0) & (em <= 0)).sum() == 0)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("C,OC,mode", [(64, 256, "res"), (256, 64, "relu"), (64, 256, "emask"), (128, 512, "res_emask"),
                                       (64, 96, "accumulate"), (192, 64, "relu_slice")])
def test_conv_pointwise_persistent(native_lib, monkeypatch, dt, C, OC, mode):
    """Persistent pointwise kernel (large-M 1x1 convs; tile sequence through one 2-stage LDS ring):
    every epilogue mode against the fp32 reference and the one-tile-per-workgroup DMA kernel, with
    an M tail (M % tile != 0) and a channel-slice input (x_ld > C)."""
    g = torch.Generator().manual_seed(C + OC + len(mode))
    r = lambda t: t.to(dt).float()  # noqa: E731
    N, H, W = 2, 181, 183  # M = 66246: > 4 x 256 tiles of 128 x 128, ragged tail
    ld = C + 64 if mode == "relu_slice" else C
    xb = r(torch.randn(N, H, W, ld, generator=g))
    x = xb[..., :C]
    cw = ConvWeights(r(torch.randn(OC, C, 1, 1, generator=g) / np.sqrt(C)), r(torch.randn(OC, generator=g)), "fwd")
    res = r(torch.randn(N, H, W, OC, generator=g))
    em = r(torch.randn(N, H, W, OC, generator=g))
    kw = {"res": dict(relu=True, res=res), "relu": dict(relu=True), "emask": dict(relu=False, emask=em),
          "res_emask": dict(relu=True, res=res, emask=em), "accumulate": dict(relu=True),
          "relu_slice": dict(relu=True)}[mode]
    ref = ops.conv2d(x, cw, pad=0, **kw)
    if mode == "accumulate":
        ref = ref + res
    dw = cw.to_device(DEV, dt)
    xd = xb.to(dt).to(DEV)[..., :C]
    dkw = {k: (v.to(dt).to(DEV) if torch.is_tensor(v) else v) for k, v in kw.items()}

    def run():
        if mode == "accumulate":
            out = res.to(dt).to(DEV)
            return ops.conv2d(xd, dw, pad=0, out=out, accumulate=True, **dkw)
        return ops.conv2d(xd, dw, pad=0, **dkw)

    got = run()
    assert got.dtype == dt and _rel(got, ref) < 1e-2, mode
    monkeypatch.setenv("DV_NO_PW", "1")  # read once per process: compare with a forced-tile DMA launch
    native_lib.dma_tune(3 if OC > 64 else 5, 1)
    try:
        dma = run()
    finally:
        native_lib.dma_tune(0, 0)
    assert _rel(got, dma) < 1e-2, mode


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("N,H,C,OC,split,relu_cols", [(2, 9, 192, 208, 64, 176), (1, 35, 288, 272, 64, 240),
                                                       (64, 17, 768, 640, 192, 448), (2, 181, 64, 192, 64, 128)])
def test_conv_two_destination_epilogue(native_lib, dt, N, H, C, OC, split, relu_cols):
    """Merged 1x1 GEMM with the two-destination epilogue (out2 / split_col; InceptionV3's b1 +
    heads): leading channels into a channel slice of one buffer, the rest into another, relu_cols
    honoured; small-M DMA tiles and the large-M persistent kernel (last case)."""
    g = torch.Generator().manual_seed(OC + split)
    r = lambda t: t.to(dt).float()  # noqa: E731
    x = r(torch.randn(N, H, H, C, generator=g))
    cw = ConvWeights(r(torch.randn(OC, C, 1, 1, generator=g) / np.sqrt(C)), r(torch.randn(OC, generator=g)), "fwd")
    ref = ops.conv2d(x, cw, pad=0, relu=True, relu_cols=relu_cols)
    Y = torch.full((N, H, H, split + 104), 7.0).to(dt).to(DEV)  # destination 1: a slice at channel 40
    T = torch.empty(N, H, H, OC - split, dtype=dt, device=DEV)
    ops.conv2d(x.to(dt).to(DEV), cw.to_device(DEV, dt), pad=0, relu=True, relu_cols=relu_cols,
               out=Y[..., 40:40 + split], out2=T, split_col=split)
    assert _rel(Y[..., 40:40 + split], ref[..., :split]) < 1e-2
    assert _rel(T, ref[..., split:]) < 1e-2
    Yc = Y.float().cpu()
    assert bool((Yc[..., :40] == 7.0).all()) and bool((Yc[..., 40 + split:] == 7.0).all())  # untouched


@pytest.mark.parametrize("N,H,W,div", [(4, 40, 48, 2), (2, 224, 224, 1), (8, 16, 96, 4), (2, 42, 70, 2)])
def test_deconv_tail_fused(native_lib, N, H, W, div):
    """Fused deconvnet tail (unpool -> 3x3 conv 64->64 -> ReLU -> per-tap products Z -> 9-tap
    shift-add -> ReLU, fp32 + per-image stats) vs its fp32 oracle with the same bf16 rounding points,
    and vs the unfused two-conv path; edge tiles on both kernels (H % 8/16, W % 32 != 0)."""
    g = torch.Generator().manual_seed(N * H + W)
    p = _bf(torch.randn(N, H // 2, W // 2, 64, generator=g))
    code = torch.randint(0, 4, (N // div, H // 2, W // 2, 64), generator=g, dtype=torch.uint8)
    mid = _cw(64, 64, bias=False, seed=3)
    last = _cw(3, 64, bias=False, seed=4)
    ref = ops.deconv_tail_ref(p, code, div, mid, last)
    midd, lastd = mid.to_device(DEV), last.to_device(DEV)
    pd, cd = p.to(torch.bfloat16).to(DEV), code.to(DEV)
    st = torch.full((N // div, 2), 7.0, dtype=torch.float64, device=DEV)
    got = ops.deconv_tail(pd, cd, div, midd, lastd, stats=st, stats_div=div)
    assert got is not None and got.shape == (N, H, W, 3)
    assert _rel(got, ref) < 2e-3
    yd = got.reshape(N // div, -1).double()
    assert torch.allclose(st, torch.stack([yd.sum(1), (yd * yd).sum(1)], 1), rtol=1e-9, atol=1e-6)
    d = ops.conv2d(pd, midd, in_mode="unpool", code=cd, code_div=div, relu_in=True, relu=True, use_bias=False)
    two = ops.conv2d(d, lastd, relu=True, epilogue="f32", use_bias=False)
    a, b = got.flatten().double().cpu(), two.flatten().double().cpu()
    assert float(a @ b / (a.norm() * b.norm())) > 0.9999
    assert _rel(got, two) < 2e-2
    # the tail kernel's schedules (DV_TAIL_V bits: transposed MFMA / expansion inside the MFMA loop)
    # compute the same dot products in the same K order: bit-identical to the round-4 schedule
    for v in ("0", "1", "2"):
        os.environ["DV_TAIL_V"] = v
        try:
            alt = ops.deconv_tail(pd, cd, div, midd, lastd)
        finally:
            del os.environ["DV_TAIL_V"]
        assert torch.equal(alt, got), v


@pytest.mark.parametrize("N,H,W", [(3, 64, 64), (2, 60, 70)])
def test_conv_c8_stream_first_layer(native_lib, N, H, W):
    """VGG16 block1_conv1 shape (8-channel padded RGB -> 64, 3x3 s1 p1, ReLU) on the row-streaming
    kernel (conv3x3_c8_stream_kernel: full 4-row / 32-px strips and the ragged-edge path), whose
    epilogue gathers 8 consecutive channels per lane with v_permlane16_swap for 16-B stores; vs
    the fp32 reference, and vs the generic path (DV_NO_C8_STREAM)."""
    g = torch.Generator().manual_seed(61)
    x = torch.rand(N, H, W, 8, generator=g) * 2 - 1
    x[..., 3:] = 0
    cw = _cw(64, 8)
    ref = ops.conv2d(_bf(x), cw, relu=True)
    xd, cwd = _bf(x).to(torch.bfloat16).to(DEV), cw.to_device(DEV)
    got = ops.conv2d(xd, cwd, relu=True)
    assert got.shape == (N, H, W, 64) and _rel(got, ref) < 1e-2
    os.environ["DV_NO_C8_STREAM"] = "1"
    try:
        alt = ops.conv2d(xd, cwd, relu=True)
    finally:
        del os.environ["DV_NO_C8_STREAM"]
    assert _rel(got, alt) < 1e-2


def test_conv_kw3_tail_split(native_lib):
    """KW3 grid of 1.05 rounds (135 row tiles x 2 on 256 CUs): the full round runs as KW3 and the
    last partial round's rows as a 128x128 DMA tail launch from row m_base (kw3_split); vs the
    plain DMA kernel (DV_KW3=0) and, on a slice, the fp32 reference."""
    g = torch.Generator().manual_seed(67)
    N, H, W, C, OC = 44, 28, 28, 256, 512
    x = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16)
    cw = _cw(OC, C)
    xd, cwd = x.to(DEV), cw.to_device(DEV)
    got = ops.conv2d(xd, cwd, relu=True)
    os.environ["DV_KW3"] = "0"
    try:
        alt = ops.conv2d(xd, cwd, relu=True)
    finally:
        del os.environ["DV_KW3"]
    assert _rel(got, alt) < 1e-2
    tail = slice(N - 3, N)  # the tail launch's images (rows >= 128 x 256)
    ref = ops.conv2d(x[tail].float(), cw, relu=True)
    assert _rel(got[tail], ref) < 1e-2
    ref0 = ops.conv2d(x[:2].float(), cw, relu=True)
    assert _rel(got[:2], ref0) < 1e-2
