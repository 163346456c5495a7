"""DeepDream (BASELINE configs 3 and 5, an extension beyond the reference): CPU semantics tests
plus GPU tests that compare the HIP autograd units against PyTorch fp32 autograd."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import deconv_api_amd.engine.deepdream as deepdream_mod

from deconv_api_amd.engine.deepdream import (DeepDream, DreamSettings, RESNET_LAYERS, TiledDeepDream,
                                             inception_deprocess, inception_preprocess, resize)
from deconv_api_amd.models.inception_v3 import InceptionV3, fold_bn
from deconv_api_amd.models.resnet50 import ResNet50


@pytest.fixture(scope="module")
def inc_cpu():
    return InceptionV3(0).build("cpu")


def test_inception_shapes_and_params(inc_cpu):
    o = inc_cpu.forward(torch.randn(1, 299, 299, 8), ["mixed2", "mixed7", "mixed10"])
    assert o["mixed2"].shape == (1, 35, 35, 288)
    assert o["mixed7"].shape == (1, 17, 17, 768)
    assert o["mixed10"].shape == (1, 8, 8, 2048)
    assert inc_cpu.num_params() == 21768352  # Keras InceptionV3(include_top=False) trainable params


def test_resnet_shapes():
    m = ResNet50(0).build("cpu")
    o = m.forward(torch.randn(1, 224, 224, 8), ["conv2_block3_out", "conv5_block3_out"])
    assert o["conv2_block3_out"].shape == (1, 56, 56, 256) and o["conv5_block3_out"].shape == (1, 7, 7, 2048)


def test_fold_bn():
    g = torch.Generator().manual_seed(0)
    w = torch.randn(8, 4, 3, 3, generator=g)
    gamma, beta, mean, var = (torch.rand(8, generator=g) + 0.5, torch.randn(8, generator=g), torch.randn(8, generator=g),
                              torch.rand(8, generator=g) + 0.1)
    x = torch.randn(2, 4, 9, 9, generator=g)
    ref = F.batch_norm(F.conv2d(x, w, padding=1), mean, var, gamma, beta, False, 0.0, 1e-3)
    wf, bf = fold_bn(w, gamma, beta, mean, var)
    torch.testing.assert_close(F.conv2d(x, wf, bf, padding=1), ref, rtol=1e-4, atol=1e-4)


def test_loss_matches_keras_formula(inc_cpu):
    dd = DeepDream(inc_cpu)
    x = torch.rand(2, 139, 139, 3) * 2 - 1
    acts = inc_cpu.forward(F.pad(x, (0, 5)), list(dd.s.layers))
    want = torch.zeros(2)
    for name, c in dd.s.layers.items():
        a = acts[name]
        want += c * (a[:, 2:-2, 2:-2, :] ** 2).sum((1, 2, 3)) / a[0].numel()
    torch.testing.assert_close(dd.loss(acts), want)


def test_grad_normalized_and_finite_difference(inc_cpu):
    torch.manual_seed(0)
    dd = DeepDream(inc_cpu)
    x = torch.rand(1, 120, 120, 3) * 2 - 1
    loss, g = dd.loss_and_grad(x)
    assert torch.allclose(g.abs().mean(), torch.tensor(1.0), atol=1e-5)
    # directional finite difference along the (unnormalized) gradient direction
    d = g / g.norm()
    eps = 1e-2
    lp = dd.loss(inc_cpu.forward(F.pad(x + eps * d, (0, 5)), list(dd.s.layers)))
    lm = dd.loss(inc_cpu.forward(F.pad(x - eps * d, (0, 5)), list(dd.s.layers)))
    assert float(lp - lm) > 0  # ascent direction increases the loss


def test_octaves_and_max_loss(inc_cpu):
    s = DreamSettings(octaves=3, iterations=2)
    dd = DeepDream(inc_cpu, s)
    assert dd.octave_shapes(300, 200) == [(153, 102), (214, 142), (300, 200)]
    x = torch.rand(1, 153, 153, 3) * 2 - 1
    frozen = DeepDream(inc_cpu, DreamSettings(iterations=3, max_loss=-1.0))  # every loss > max_loss
    assert torch.equal(frozen.gradient_ascent(x), x)
    moved = DeepDream(inc_cpu, DreamSettings(iterations=1, max_loss=None)).gradient_ascent(x)
    assert not torch.equal(moved, x)


def test_detail_reinjection_identity(inc_cpu):
    """With zero steps the octave loop must return the original image (lost detail re-injected)."""
    dd = DeepDream(inc_cpu, DreamSettings(octaves=3, iterations=1, step=0.0))
    x = torch.rand(1, 160, 160, 3) * 2 - 1
    torch.testing.assert_close(dd.run(x), x, rtol=1e-5, atol=1e-5)


def test_pre_deprocess_roundtrip():
    u8 = torch.randint(0, 256, (1, 5, 5, 3), dtype=torch.uint8)
    assert (inception_deprocess(inception_preprocess(u8)).int() - u8.int()).abs().max() <= 1


def test_tiled_single_rank_matches_untiled_when_one_tile():
    net = ResNet50(1).build("cpu")
    s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=1, iterations=1, max_loss=None)
    x = torch.rand(1, 96, 96, 3) * 2 - 1
    tiled = TiledDeepDream(net, s, tile=256)  # one tile covers the image: roll commutes with the net?
    a = tiled.gradient_ascent(x)
    assert a.shape == x.shape and torch.isfinite(a).all() and not torch.equal(a, x)


# --------------------------------------------------------------------------- GPU
def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float(a @ b / (a.norm() * b.norm()))


@pytest.mark.gpu
def test_gpu_pool_kernels(native_lib):
    from deconv_api_amd.ops.autograd import avg_pool, max_pool

    g = torch.Generator().manual_seed(1)
    for k, s, p in [(3, 2, 0), (3, 1, 1), (3, 2, 1), (2, 2, 0), (5, 1, 2)]:  # 3x3: unrolled kernels
        x = torch.randn(2, 13, 11, 24, generator=g).to(torch.bfloat16).float()
        for fn in (max_pool, avg_pool):
            xc = x.clone().requires_grad_(True)
            yc = fn(xc, k, s, p)
            gy = torch.randn_like(yc).to(torch.bfloat16).float()
            (gc,) = torch.autograd.grad(yc, xc, gy)
            xd = x.to(torch.bfloat16).cuda().requires_grad_(True)
            yd = fn(xd, k, s, p)
            (gd,) = torch.autograd.grad(yd, xd, gy.to(torch.bfloat16).cuda())
            assert (yd.float().cpu() - yc).abs().max() < 2e-2 * yc.abs().max()
            assert (gd.float().cpu() - gc).abs().max() < 2e-2 * gc.abs().max() + 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["inception", "resnet"])
def test_gpu_dream_gradient_matches_cpu(native_lib, which):
    if which == "inception":
        cpu, gpu = InceptionV3(0).build("cpu"), InceptionV3(0).build("cuda")
        s = DreamSettings()
        hw = 139
    else:
        cpu, gpu = ResNet50(0).build("cpu"), ResNet50(0).build("cuda")
        s = DreamSettings(layers=dict(RESNET_LAYERS))
        hw = 128
    x = (torch.rand(2, hw, hw, 3, generator=torch.Generator().manual_seed(2)) * 2 - 1)
    x = x.to(torch.bfloat16).float()
    lc, gc = DeepDream(cpu, s).loss_and_grad(x)
    lg, gg = DeepDream(gpu, s).loss_and_grad(x.cuda())
    assert torch.allclose(lg.cpu(), lc, rtol=5e-2)
    for b in range(2):
        assert _cos(gg[b].cpu(), gc[b]) > 0.95


@pytest.mark.gpu
def test_gpu_resnet_dream_fp16(native_lib):
    """BASELINE config 5 precision: fp16 storage + f16 MFMA through ResNet-50's conv/pool kernels."""
    cpu, gpu = ResNet50(0).build("cpu"), ResNet50(0).build("cuda", torch.float16)
    s = DreamSettings(layers=dict(RESNET_LAYERS))
    x = (torch.rand(2, 128, 128, 3, generator=torch.Generator().manual_seed(4)) * 2 - 1)
    x = x.to(torch.float16).float()
    dd = DeepDream(gpu, s)
    assert dd.dtype == torch.float16
    lc, gc = DeepDream(cpu, s).loss_and_grad(x)
    lg, gg = dd.loss_and_grad(x.cuda())
    assert torch.isfinite(gg).all() and torch.allclose(lg.cpu(), lc, rtol=3e-2)
    for b in range(2):
        assert _cos(gg[b].cpu(), gc[b]) > 0.97


@pytest.mark.gpu
def test_gpu_graph_replay_equals_eager(native_lib):
    net = InceptionV3(0).build("cuda")
    s = DreamSettings(iterations=3, octaves=2)
    x = (torch.rand(2, 150, 150, 3, generator=torch.Generator().manual_seed(3)) * 2 - 1).cuda()
    eager = DeepDream(net, s, use_graphs=False).run(x)
    graph = DeepDream(net, s, use_graphs=True).run(x)
    assert (eager - graph).abs().max() < 1e-3
    assert (graph - x).abs().max() > 1e-3


class _SquareNet:
    """loss = sum(x^2): its input gradient is local (2x), so any tiling must stitch to 2x exactly."""
    device = torch.device("cpu")

    def forward(self, x, names):
        return {"l": x}


@pytest.mark.parametrize("H,W,tile,B", [(37, 53, 16, 2), (64, 64, 32, 1), (20, 90, 25, 3)])
def test_tiled_gather_scatter_is_exact(H, W, tile, B):
    """Rolled batched tile gather + owned-pixel scatter + un-roll reproduce the untiled gradient."""
    s = DreamSettings(layers={"l": 1.0}, octaves=1, iterations=3, max_loss=None, border=0)
    x = torch.rand(B, H, W, 3, generator=torch.Generator().manual_seed(H)) * 2 - 1
    got = TiledDeepDream(_SquareNet(), s, tile=tile).gradient_ascent(x)
    want = x.clone()
    for _ in range(3):
        want += s.step * want / want.abs().mean(dim=(1, 2, 3), keepdim=True)
    assert torch.allclose(got, want, atol=1e-5)


@pytest.mark.gpu
def test_gpu_tiled_graph_equals_eager(native_lib):
    """The hipGraph-captured tiled step (device-side roll shift) == the eager tiled step."""
    net = ResNet50(0).build("cuda", torch.float16)
    s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=2, iterations=3)
    x = (torch.rand(2, 200, 260, 3, generator=torch.Generator().manual_seed(5)) * 2 - 1).cuda()
    eager = TiledDeepDream(net, s, tile=128, seed=3, use_graphs=False).run(x)
    graph = TiledDeepDream(net, s, tile=128, seed=3, use_graphs=True).run(x)
    assert torch.isfinite(graph).all() and (graph - x).abs().max() > 1e-3
    assert (eager - graph).abs().max() < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("k,s,p,cin", [(7, 2, 3, 3), (3, 2, 0, 3), (3, 2, 1, 32)])
def test_gpu_strided_conv_unit_input_grad(native_lib, k, s, p, cin):
    """Strided conv units' input gradient (GEMM+col2im for few channels, sub-pixel classes
    otherwise, both with the ReLU mask) vs CPU autograd."""
    from deconv_api_amd.ops import autograd as AG

    g = torch.Generator().manual_seed(k + cin)
    w = torch.randn(64, cin, k, k, generator=g) / (k * k * cin) ** 0.5
    b = torch.randn(64, generator=g) * 0.1
    w = w.to(torch.float16).float()
    x = torch.randn(2, 37, 41, cin, generator=g).to(torch.float16).float()
    for relu in (False, True):
        cpu = AG.ConvUnit("u", w, b, s, (p, p), relu=relu).build("cpu")
        gpu = AG.ConvUnit("u", w, b, s, (p, p), relu=relu).build("cuda", torch.float16)
        assert (gpu.col_w is not None) == (cin <= 8)
        xc = x.clone().requires_grad_(True)
        yc = cpu(xc)
        gy = torch.randn(*yc.shape, generator=g).to(torch.float16).float()
        (gc,) = torch.autograd.grad(yc, xc, gy)
        x8 = torch.nn.functional.pad(x, (0, (-cin) % 8)).to(torch.float16).cuda().requires_grad_(True)
        yd = gpu(x8)
        (gd,) = torch.autograd.grad(yd, x8, gy.to(torch.float16).cuda())
        gd = gd[..., :cin].float().cpu()
        if not relu:  # exact up to fp16 rounding of the GEMM output
            assert (gd - gc).abs().max() < 5e-3 * gc.abs().max()
        else:  # fp16 forward rounding can flip a few ReLU-mask entries near 0
            a, b2 = gd.flatten().double(), gc.flatten().double()
            assert float(a @ b2 / (a.norm() * b2.norm())) > 0.999


@pytest.mark.gpu
@pytest.mark.parametrize("stride,proj,premasked", [(1, False, False), (1, True, True), (2, True, False),
                                                   (2, True, True), (1, False, True)])
def test_gpu_bottleneck_block_grad(native_lib, stride, proj, premasked):
    """Fused bottleneck autograd node vs CPU autograd of the unfused block (bf16)."""
    from deconv_api_amd.ops import autograd as AG

    g = torch.Generator().manual_seed(stride * 10 + proj)
    cin, w = (64, 16) if proj else (64, 16)
    mk = lambda n, ci, co, k, s, p, relu: AG.ConvUnit(  # noqa: E731
        n, torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5, torch.randn(co, generator=g) * 0.1, s, (p, p),
        relu=relu)
    units = [mk("c1", cin, w, 1, stride, 0, True), mk("c2", w, w, 3, 1, 1, True), mk("c3", w, 64, 1, 1, 0, False),
             mk("sh", cin, 64, 1, stride, 0, False) if (proj or stride > 1) else None]
    x = torch.randn(2, 14, 18, cin, generator=g).clamp_min(0).to(torch.bfloat16).float()
    cpu = [u.__class__(u.name, u.w, u.b, u.stride, u.pad, u.relu).build("cpu") if u else None for u in units]
    gpu = [u.build("cuda") if u else None for u in units]
    xc = x.clone().requires_grad_(True)
    yc = AG.bottleneck(xc, *cpu)
    gy = torch.randn(*yc.shape, generator=g)
    if premasked:
        gy = gy * (yc.detach() > 0)
    (gc,) = torch.autograd.grad(yc, xc, gy)
    if premasked:
        gc = gc * (x > 0)  # the contract: the block hands back a gradient masked by its ReLU input
    xd = x.to(torch.bfloat16).cuda().requires_grad_(True)
    if premasked:
        with AG.premasked_grads():
            yd = AG.bottleneck(AG.tag_relu_output(xd), *gpu)
    else:
        yd = AG.bottleneck(xd, *gpu)
    assert (yd.float().cpu() - yc.detach()).abs().max() < 3e-2 * yc.abs().max()
    (gd,) = torch.autograd.grad(yd, xd, gy.to(torch.bfloat16).cuda())
    a, b = gd.float().cpu().flatten().double(), gc.flatten().double()
    assert float(a @ b / (a.norm() * b.norm())) > 0.99


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gpu_relu_bits_conv_pw(native_lib, dt):
    """1-bit ReLU masks on the persistent 1x1 kernel: obits == packbits(out > 0) (bit c % 8 of byte c / 8);
    a masked input gradient with ebits == the same with the 16-bit emask, bit for bit."""
    import numpy as np

    from deconv_api_amd import ops
    from deconv_api_amd.ops import autograd as AG

    g = torch.Generator().manual_seed(5)
    u = AG.ConvUnit("c", torch.randn(256, 64, 1, 1, generator=g) / 8, torch.randn(256, generator=g) * 0.1, 1, (0, 0),
                    relu=True).build("cuda", dt)
    x = torch.randn(4, 128, 128, 64, generator=g).to(dt).cuda()
    ob = torch.zeros(4 * 128 * 128, 32, dtype=torch.uint8, device="cuda")
    y = ops.conv2d(x, u.fwd, relu=True, obits=ob)
    assert ops.conv.bits_flags() == 1
    want = np.packbits((y.float() > 0).cpu().numpy().reshape(-1, 256), axis=1, bitorder="little")
    assert np.array_equal(ob.cpu().numpy(), want)
    gs = torch.randn(4, 128, 128, 256, generator=g).to(dt).cuda()
    ref = ops.conv2d(x, u.fwd, relu=False, use_bias=False, res=gs, emask=y)
    assert ops.conv.bits_flags() == 0
    got = ops.conv2d(x, u.fwd, relu=False, use_bias=False, res=gs, emask=y, ebits=ob)
    assert ops.conv.bits_flags() == 2 and torch.equal(got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("hw,cout", [(128, 64), (66, 64), (64, 128)])
def test_gpu_relu_bits_halo_stream(native_lib, hw, cout):
    """1-bit masks on the halo-stream 3x3 kernels' LDS-staged epilogues (hs16 at sides % 16, the 16 x 32
    kernel otherwise): obits == packbits(out > 0); ebits == emask bit for bit."""
    import numpy as np

    from deconv_api_amd import ops
    from deconv_api_amd.ops import autograd as AG

    g = torch.Generator().manual_seed(hw + cout)
    u = AG.ConvUnit("c", torch.randn(cout, 64, 3, 3, generator=g) / 24, torch.randn(cout, generator=g) * 0.1, 1,
                    (1, 1), relu=True).build("cuda", torch.float16)
    x = torch.randn(3, hw, hw, 64, generator=g).to(torch.float16).cuda()
    ob = torch.zeros(3 * hw * hw, cout // 8, dtype=torch.uint8, device="cuda")
    y = ops.conv2d(x, u.fwd, relu=True, obits=ob)
    assert ops.conv.bits_flags() == 1
    want = np.packbits((y.float() > 0).cpu().numpy().reshape(-1, cout), axis=1, bitorder="little")
    assert np.array_equal(ob.cpu().numpy(), want)
    gy = torch.randn(3, hw, hw, cout, generator=g).to(torch.float16).cuda()
    w = AG.ConvUnit("d", torch.randn(cout, cout, 3, 3, generator=g) / 24, None, 1, (1, 1), relu=False).build(
        "cuda", torch.float16)
    ref = ops.conv2d(gy, w.fwd, relu=False, use_bias=False, emask=y)
    got = ops.conv2d(gy, w.fwd, relu=False, use_bias=False, emask=y, ebits=ob)
    assert ops.conv.bits_flags() == 2 and torch.equal(got, ref)


@pytest.mark.gpu
def test_gpu_relu_bits_bottleneck_chain_identical(native_lib, monkeypatch):
    """Two chained bottlenecks (premasked): the second block's input gradient masked by the first block's
    1-bit mask == masked by its 16-bit output (DV_RELU_BITS=0), bit for bit."""
    from deconv_api_amd.ops import autograd as AG

    g = torch.Generator().manual_seed(9)
    mk = lambda n, ci, co, k, p, relu: AG.ConvUnit(  # noqa: E731
        n, torch.randn(co, ci, k, k, generator=g) / (ci * k * k) ** 0.5, torch.randn(co, generator=g) * 0.1, 1, (p, p),
        relu=relu).build("cuda", torch.float16)
    blocks = [[mk("c1", 256, 64, 1, 0, True), mk("c2", 64, 64, 3, 1, True), mk("c3", 64, 256, 1, 0, False), None]
              for _ in range(2)]
    x = torch.randn(8, 64, 64, 256, generator=g).clamp_min(0).to(torch.float16).cuda()
    gy = torch.randn(8, 64, 64, 256, generator=g).to(torch.float16).cuda()
    out = {}
    for bits in (True, False):
        monkeypatch.setattr(AG, "RELU_BITS", bits)
        xd = x.clone().requires_grad_(True)
        with AG.premasked_grads():
            y = AG.bottleneck(AG.tag_relu_output(xd), *blocks[0])
            assert (getattr(y, "_dv_bits", None) is not None) == bits
            z = AG.bottleneck(y, *blocks[1])
        (gx,) = torch.autograd.grad(z, xd, gy * (z.detach() > 0))
        out[bits] = gx
    assert torch.equal(out[True], out[False])


@pytest.mark.gpu
@pytest.mark.parametrize("bi,hw", [(0, 11), (3, 11), (4, 9), (8, 9), (9, 5)])
@pytest.mark.parametrize("premasked", [False, True])
@pytest.mark.parametrize("strided_direct", [True, False])
def test_gpu_inception_block_grad(native_lib, bi, hw, premasked, strided_direct, monkeypatch):
    """One-node InceptionV3 mixed block (direct concat-slice writes, commuted avg-pool branch,
    accumulate/emask epilogues) vs CPU autograd of the unfused block: mixed0 (A), mixed3 (B),
    mixed4 (C), mixed8 (D, strided + max), mixed9 (E, split convs). Strided-conv gradients both as
    one transposed conv into gx (small maps) and as sub-pixel GEMMs (large maps)."""
    from deconv_api_amd.ops import autograd as AG

    monkeypatch.setattr(AG, "STRIDED_DIRECT_FLOPS", 1e30 if strided_direct else 0.0)
    cpu, gpu = InceptionV3(0).build("cpu"), InceptionV3(0).build("cuda")
    cin = [192, 256, 288, 288, 768, 768, 768, 768, 768, 1280, 2048][bi]
    g = torch.Generator().manual_seed(bi + 17 * premasked)
    x = torch.randn(2, hw, hw, cin, generator=g).clamp_min(0).to(torch.bfloat16).float()
    xc = x.clone().requires_grad_(True)
    yc = cpu.iblocks[bi](xc)
    gy = torch.randn(*yc.shape, generator=g)
    if premasked:
        gy = gy * (yc.detach() > 0)
    (gc,) = torch.autograd.grad(yc, xc, gy)
    if premasked:
        gc = gc * (x > 0)
    xd = x.to(torch.bfloat16).cuda().requires_grad_(True)
    if premasked:
        with AG.premasked_grads():
            yd = gpu.iblocks[bi](AG.tag_relu_output(xd))
    else:
        yd = gpu.iblocks[bi](xd)
    assert yd.shape == yc.shape
    assert _cos(yd.float().cpu(), yc.detach()) > 0.999
    (gd,) = torch.autograd.grad(yd, xd, gy.to(torch.bfloat16).cuda())
    assert _cos(gd.float().cpu(), gc) > 0.995


@pytest.mark.gpu
def test_gpu_fused_step_equals_unfused(native_lib):
    """Fused step tail (HIP sumsq partials + loss gradients, one normalize/update kernel writing the
    next network input, device-side max_loss) == the torch-op step, eager and graph-replayed."""
    net = InceptionV3(0).build("cuda")
    x = (torch.rand(2, 150, 150, 3, generator=torch.Generator().manual_seed(6)) * 2 - 1).cuda()
    for max_loss in (None, 1e-9):  # 1e-9: every image stops at its first step (device-side flag)
        for iters, octs in ((1, 1), (3, 2)):
            s = DreamSettings(iterations=iters, octaves=octs, max_loss=max_loss)
            ref = DeepDream(net, s, use_graphs=False)
            ref.fused = False
            want = ref.run(x)
            got = {}
            for graphs in (False, True):
                for taps in (False, True):
                    deepdream_mod.TAPS = taps
                    try:
                        dd = DeepDream(net, s, use_graphs=graphs)
                        assert dd.fused
                        got[graphs, taps] = r = dd.run(x)
                    finally:
                        deepdream_mod.TAPS = True
                    if max_loss is not None or (iters == 1 and not taps):
                        # one step, same arithmetic: equal up to the fp32 update rounding
                        assert (r - want).abs().max() < 1e-4, (max_loss, graphs, taps)
                    elif iters == 1:  # loss taps sum the loss gradient in fp32 (one rounding, not two)
                        assert _cos(r - x, want - x) > 0.9999 and (r - want).abs().max() < 1e-2, (graphs, taps)
                    else:  # later steps feed bf16-rounded inputs to a chaotic map: same dream direction
                        # (1-ulp differences of step 1 grow: ~0.96 without taps, ~0.92 with them)
                        assert _cos(r - x, want - x) > 0.9, (max_loss, graphs, taps)
            # the captured graph replays exactly the eager fused steps
            assert (got[True, True] - got[False, True]).abs().max() < 1e-3, (max_loss, iters)


@pytest.mark.gpu
@pytest.mark.parametrize("src,dst", [((108, 108), (152, 152)), ((213, 213), (299, 299)), ((37, 53), (20, 71)),
                                     ((64, 64), (64, 64)), ((1, 5), (3, 1))])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_gpu_octave_resize_matches_interpolate(native_lib, src, dst, dt):
    """octave_resize (csrc/dream.hip) == F.interpolate(bilinear, align_corners=True) of (a + b - c), in fp32
    on the GPU and against the fp64 CPU oracle; the 16-bit network-input copy is the rounded image with
    channels 3..7 zero; an identity resize is exact."""
    gen = torch.Generator().manual_seed(3)
    a, b, c = (torch.randn(3, *src, 3, generator=gen) for _ in range(3))
    want = deepdream_mod.resize((a + b - c).double(), dst).float()
    y = torch.empty(3, *dst, 3, device="cuda")
    yin = torch.full((3, *dst, 8), 7.0, dtype=dt, device="cuda")
    native_lib.octave_resize(a.cuda(), b.cuda(), c.cuda(), y, yin)
    # fp32 source positions (as torch's kernel): |error| <= slope x position ulp, ~1e-5 on these values
    assert float((y.cpu() - want).abs().max()) < 2e-4
    gpu_ref = deepdream_mod.resize((a + b - c).cuda(), dst)
    assert float((y - gpu_ref).abs().max()) < 5e-5
    assert torch.equal(yin[..., :3], y.to(dt)) and not yin[..., 3:].any()
    y2 = torch.empty_like(y)
    native_lib.octave_resize(a.cuda(), None, None, y2, None)
    assert float((y2.cpu() - deepdream_mod.resize(a.double(), dst).float()).abs().max()) < 2e-4
    if src == dst:
        assert torch.equal(y2.cpu(), a)


@pytest.mark.gpu
def test_gpu_fused_octaves_match_torch_octaves(native_lib):
    """The fused octave loop (one octave_resize per transition, detail precomputed) == the torch octave loop
    (F.interpolate + adds) around the same fused gradient ascent."""
    net = InceptionV3(0).build("cuda")
    x = (torch.rand(2, 220, 230, 3, generator=torch.Generator().manual_seed(8)) * 2 - 1).cuda()
    for iters, max_loss in ((1, 1e-9), (2, None)):
        dd = DeepDream(net, DreamSettings(iterations=iters, octaves=3, max_loss=max_loss), use_graphs=True)
        dd.split = 1
        got = dd.run(x)
        shapes = dd.octave_shapes(220, 230)
        img, shrunk = x, deepdream_mod.resize(x, shapes[0])
        for hw in shapes:  # the generic loop of DeepDream.octave_steps
            img = dd.gradient_ascent(deepdream_mod.resize(img, hw))
            img = img + (deepdream_mod.resize(x, hw) - deepdream_mod.resize(shrunk, hw))
            shrunk = deepdream_mod.resize(x, hw)
        if max_loss is not None:  # no update: pure resize/detail arithmetic
            assert float((got - img).abs().max()) < 1e-4
        else:
            # bf16-rounded network inputs: 1-ulp differences of the resize grow through the steps (0.98-0.997 seen)
            assert _cos(got - x, img - x) > 0.95 and float((got - img).abs().max()) < 0.25


@pytest.mark.gpu
def test_gpu_split_batch_streams(native_lib):
    """A batch run as 2 concurrent sub-batches (own streams, own graphs) == the whole batch."""
    net = InceptionV3(0).build("cuda")
    x = (torch.rand(4, 150, 150, 3, generator=torch.Generator().manual_seed(9)) * 2 - 1).cuda()
    for iters in (1, 3):
        s = DreamSettings(iterations=iters, octaves=2)
        one = DeepDream(net, s, use_graphs=True)
        two = DeepDream(net, s, use_graphs=True)
        two.split = 2
        want, got = one.run(x), two.run(x)
        assert {k[-1] for k in two._graphs} == {0, 1}  # one graph set per sub-batch
        if iters == 1:
            assert (got - want).abs().max() < 1e-3
        else:
            assert _cos(got - x, want - x) > 0.95
        again = two.run(x)  # replays of both sub-batches' cached graphs
        assert (again - got).abs().max() < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("max_loss", [None, 1e-9])
def test_gpu_tiled_fused_equals_torch(native_lib, max_loss):
    """Fused tiled step (HIP rolled gather, owned-pixel packs with loss/|g| tails, pack-driven
    update; one hipGraph per octave incl. all steps; octave transitions as ONE octave_resize launch
    each) == the torch tiled implementation (F.interpolate + adds between octaves), on a shape
    whose tiles overlap (200 x 260 with 128 tiles -> 2 x 3 tiles of 100 x 87)."""
    net = ResNet50(0).build("cuda", torch.float16)
    x = (torch.rand(2, 200, 260, 3, generator=torch.Generator().manual_seed(8)) * 2 - 1).cuda()
    for iters in (1, 3):
        s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=2, iterations=iters, max_loss=max_loss)
        ref = TiledDeepDream(net, s, tile=128, seed=3, use_graphs=False)
        ref.tile_fused = False
        want = ref.run(x)
        for graphs in (False, True):
            dd = TiledDeepDream(net, s, tile=128, seed=3, use_graphs=graphs)
            assert dd.tile_fused
            got = dd.run(x)
            assert torch.isfinite(got).all()
            if max_loss is not None:  # every image stops at its first step: only the octave arithmetic
                # (octave_resize vs F.interpolate: fp32 rounding of the same bilinear weights)
                assert (got - want).abs().max() < 1e-4, (iters, graphs)
            else:  # same gradients up to 16-bit rounding of the first step's inputs (tools/diag_tiled.py)
                assert _cos(got - x, want - x) > (0.998 if iters == 1 else 0.99), (iters, graphs)
            got2 = dd.run(x)  # replay of the cached state/graph (fresh shifts from the generator)
            assert torch.isfinite(got2).all()


@pytest.mark.gpu
@pytest.mark.parametrize("chunks,streams", [(2, 1), (3, 2)])
def test_gpu_tiled_local_chunks_streams(native_lib, monkeypatch, chunks, streams):
    """DV_TILE_LOCAL_CHUNKS / DV_TILE_CHUNK_STREAMS: one rank's units as several chunks, forked onto
    side streams and joined before each step's update (inside the octave graph when captured) ==
    the one-chunk step up to the conv rounding of smaller batches."""
    import deconv_api_amd.engine.deepdream as D

    net = ResNet50(0).build("cuda", torch.float16)
    s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=2, iterations=3, max_loss=None)
    x = (torch.rand(3, 200, 260, 3, generator=torch.Generator().manual_seed(8)) * 2 - 1).cuda()
    want = TiledDeepDream(net, s, tile=128, seed=3, use_graphs=False).run(x)
    monkeypatch.setattr(D, "TILE_LOCAL_CHUNKS", chunks)
    monkeypatch.setattr(D, "TILE_CHUNK_STREAMS", streams)
    for graphs in (False, True):
        dd = TiledDeepDream(net, s, tile=128, seed=3, use_graphs=graphs)
        got = dd.run(x)
        torch.cuda.synchronize()
        assert all(st.C == chunks for st in dd._tgraphs.values())
        assert torch.isfinite(got).all() and _cos(got - x, want - x) > 0.99, graphs
        assert torch.isfinite(dd.run(x)).all()


@pytest.mark.gpu
def test_gpu_tiled_whole_octave_graph_1024(native_lib):
    """Regression for the round-1 illegal-address fault: one hipGraph holding every step of a tiled
    octave at 1024^2 (tile 512, fp16) replays, twice, and matches the eager fused steps."""
    net = ResNet50(0).build("cuda", torch.float16)
    s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=2, iterations=2, max_loss=None)
    x = (torch.rand(1, 1024, 1024, 3, generator=torch.Generator().manual_seed(11)) * 2 - 1).cuda()
    eager = TiledDeepDream(net, s, tile=512, seed=5, use_graphs=False).run(x)
    dd = TiledDeepDream(net, s, tile=512, seed=5, use_graphs=True)
    graph = dd.run(x)
    torch.cuda.synchronize()
    assert all(st.graph is not None for st in dd._tgraphs.values())
    assert torch.isfinite(graph).all() and _cos(graph - x, eager - x) > 0.99
    assert torch.isfinite(dd.run(x)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("p,H,W", [(0, 37, 41), (0, 40, 38), (1, 33, 36)])
def test_gpu_stem_conv_direct(native_lib, p, H, W):
    """InceptionV3 conv2d_1 geometry (3 -> 32, 3x3 / stride 2) on the direct VALU kernels
    (csrc/conv_stem.hip): forward (bias + ReLU) and the input gradient (premasked, as DeepDream runs
    it) vs CPU autograd and vs the GEMM + col2im path of the same unit."""
    from deconv_api_amd.ops import autograd as AG

    k, cout = 3, 32
    g = torch.Generator().manual_seed(H * W + p)
    w = (torch.randn(cout, 3, k, k, generator=g) / (3 * k * k) ** 0.5).to(torch.bfloat16).float()
    b = torch.randn(cout, generator=g) * 0.1
    x = torch.randn(2, H, W, 3, generator=g).to(torch.bfloat16).float()
    cpu = AG.ConvUnit("u", w, b, 2, (p, p), relu=True).build("cpu")
    gpu = AG.ConvUnit("u", w, b, 2, (p, p), relu=True).build("cuda", torch.bfloat16)
    assert gpu.stem_w is not None and gpu.col_w is not None
    xc = x.clone().requires_grad_(True)
    yc = cpu(xc)
    gy = (torch.randn(*yc.shape, generator=g) * (yc > 0)).to(torch.bfloat16).float()  # premasked gradient
    (gc,) = torch.autograd.grad(yc, xc, gy)
    x8 = torch.nn.functional.pad(x, (0, 5)).to(torch.bfloat16).cuda()
    outs = {}
    for path in ("direct", "gemm"):
        if path == "gemm":
            gpu.stem_w = None
        xd = x8.clone().requires_grad_(True)
        with AG.premasked_grads():
            yd = gpu(xd)
        (gd,) = torch.autograd.grad(yd, xd, gy.to(torch.bfloat16).cuda())
        gd = gd.float().cpu()
        outs[path] = (yd.float().cpu(), gd)
        assert (yd.float().cpu() - yc).abs().max() < 2e-2 * yc.abs().max()
        assert (gd[..., :3] - gc).abs().max() < 2e-2 * gc.abs().max()
    assert float(outs["direct"][1][..., 3:].abs().max()) == 0.0  # padding channels get no gradient
    assert (outs["direct"][1][..., :3] - outs["gemm"][1][..., :3]).abs().max() < 2e-2 * gc.abs().max()


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("N,H,W,bias", [(2, 37, 41, True), (1, 64, 96, True), (3, 150, 133, False), (2, 224, 224, True)])
def test_gpu_stem7_fwd(native_lib, monkeypatch, dt, N, H, W, bias):
    """ResNet-50 conv1 forward (3 -> 64, 7x7 / 2, pad 3, bias + ReLU) on the tap-paired MFMA kernel
    (csrc/conv_stem7.hip) vs an fp32 PyTorch conv of the same rounded operands and vs the implicit
    GEMM path of the same unit (a different fp32 summation order: equal up to one 16-bit rounding);
    odd sizes and partial output tiles."""
    from deconv_api_amd.ops import autograd as AG

    g = torch.Generator().manual_seed(N * H + W)
    w = (torch.randn(64, 3, 7, 7, generator=g) / (3 * 49) ** 0.5).to(dt).float()
    b = torch.randn(64, generator=g) * 0.1 if bias else None
    x = torch.randn(N, H, W, 3, generator=g).to(dt).float()
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, b, stride=2, padding=3).relu().permute(0, 2, 3, 1)
    gpu = AG.ConvUnit("u", w, b, 2, (3, 3), relu=True).build("cuda", dt)
    assert gpu.stem7_w is not None
    x8 = torch.nn.functional.pad(x, (0, 5)).to(dt).cuda()
    y7 = AG._stem_fwd(x8, gpu)
    assert y7 is not None and y7.shape == ref.shape
    monkeypatch.setattr(AG, "STEM7", False)
    assert AG._stem_fwd(x8, gpu) is None
    yg = gpu(x8).float().cpu()
    y7 = y7.float().cpu()
    tol = (8e-3 if dt == torch.float16 else 2e-2) * ref.abs().max()
    assert (y7 - ref).abs().max() < tol
    assert (y7 - yg).abs().max() < tol


@pytest.mark.gpu
@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("H,W,premasked", [(37, 41, True), (64, 96, True), (150, 133, False), (224, 224, True)])
def test_gpu_stem_dgrad_fused(native_lib, monkeypatch, dt, H, W, premasked):
    """ResNet-50 conv1 (3 -> 64, 7x7 / 2, pad 3) input gradient: the fused MFMA GEMM + col2im kernel
    (csrc/conv_stem_dgrad.hip) equals the two-kernel GEMM (cols in HBM) + col2im path BIT FOR BIT
    (same fp32 accumulation order, same 16-bit rounding of the cols) and CPU autograd up to rounding;
    several dx tiles, odd sizes, with the ReLU mask (not premasked) and without."""
    from deconv_api_amd.ops import autograd as AG

    g = torch.Generator().manual_seed(H + W)
    w = (torch.randn(64, 3, 7, 7, generator=g) / (3 * 49) ** 0.5).to(dt).float()
    b = torch.randn(64, generator=g) * 0.1
    x = torch.randn(2, H, W, 3, generator=g).to(dt).float()
    cpu = AG.ConvUnit("u", w, b, 2, (3, 3), relu=True).build("cpu")
    gpu = AG.ConvUnit("u", w, b, 2, (3, 3), relu=True).build("cuda", dt)
    assert gpu.stem_w is None and gpu.col_w is not None
    xc = x.clone().requires_grad_(True)
    yc = cpu(xc)
    gy = torch.randn(*yc.shape, generator=g)
    if premasked:
        gy = gy * (yc > 0)
    gy = gy.to(dt).float()
    (gc,) = torch.autograd.grad(yc, xc, gy)
    x8 = torch.nn.functional.pad(x, (0, 5)).to(dt).cuda()
    outs = {}
    for fused in (True, False):
        monkeypatch.setattr(AG, "STEM_FUSED", fused)
        xd = x8.clone().requires_grad_(True)
        if premasked:
            with AG.premasked_grads():
                yd = gpu(xd)
        else:
            yd = gpu(xd)
        (gd,) = torch.autograd.grad(yd, xd, gy.to(dt).cuda())
        outs[fused] = gd.float().cpu()
    assert torch.equal(outs[True], outs[False])
    assert float(outs[True][..., 3:].abs().max()) == 0.0
    assert (outs[True][..., :3] - gc).abs().max() < 2e-2 * gc.abs().max()


@pytest.mark.gpu
def test_gpu_pool_backward_accumulate(native_lib):
    """pool backward with accumulate=True adds the pooled gradient to the existing gx (max and avg)."""
    from deconv_api_amd.ops import native as nat

    g = torch.Generator().manual_seed(3)
    N, H, W, C = 2, 13, 11, 24
    for kind in (0, 1):
        k, s, p = (3, 2, 0) if kind == 0 else (3, 1, 1)
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16).cuda()
        y = torch.empty(N, OH, OW, C, dtype=torch.bfloat16, device="cuda")
        idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device="cuda") if kind == 0 else None
        geom = [N, H, W, C, OH, OW, k, s, p]
        nat.lib().pool(x, y, idx, kind, 0, geom)
        gy = torch.randn(N, OH, OW, C, generator=g).to(torch.bfloat16).cuda()
        plain = torch.empty_like(x)
        nat.lib().pool(gy, plain, idx, kind, 1, geom)
        base = torch.randn(N, H, W, C, generator=g).to(torch.bfloat16).cuda()
        acc = base.clone()
        nat.lib().pool(gy, acc, idx, kind, 1, geom, None, False, True)
        assert (acc.float() - (base.float() + plain.float())).abs().max() < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 1), (2, 2), (3, 3)])
def test_gpu_tiled_virtual_ranks_match_one_rank(native_lib, world, chunks):
    """The multi-rank fused tiled step (each rank's tile_gather / network / tile_pack into ITS slot
    of the packs, then tile_update over ``world`` packs) run for virtual ranks on one GPU equals the
    1-rank octave: the rank/world indexing of tile_pack (unit offsets, ucap) and tile_update (world
    packs, chunked [chunk][rank] layouts) is exercised without a multi-GPU box. Units land in different
    rank / chunk batches, so conv tile choices (and fp32 summation order) differ slightly: compared up
    to rounding."""
    from deconv_api_amd.models.resnet50 import ResNet50

    net = ResNet50(0).build("cuda", torch.float16)
    x = (torch.rand(2, 256, 320, 3, generator=torch.Generator().manual_seed(3)) * 2 - 1).cuda()
    # one step: only the first gradient's rounding differs; three steps: fp16 rounding feeds back
    for iters, cos_min, mean_max in ((1, 0.9995, 1e-3), (3, 0.995, 3e-3)):
        s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=1, iterations=iters, max_loss=None)
        ref = TiledDeepDream(net, s, tile=128, seed=11, use_graphs=False).gradient_ascent(x)
        got = TiledDeepDream(net, s, tile=128, seed=11, use_graphs=False).virtual_octave(x, world, chunks)
        d = (got - ref).abs()
        c = _cos((got - x).flatten().cpu(), (ref - x).flatten().cpu())
        assert c > cos_min, (iters, c)
        assert float(d.mean()) < mean_max and float(d.max()) < 5e-2, (iters, float(d.mean()), float(d.max()))


@pytest.mark.gpu
def test_gpu_tiled_collective_octave_captured(native_lib):
    """torchrun, one rank, DV_TILE_COLLECTIVE=1: the collective code path of the tiled octave (the
    per-step all-gather of the packs over RCCL) is captured INSIDE the octave's hipGraph and equals
    the collective-free 1-rank octave bit for bit; the chunked overlapped step (DV_TILE_CHUNKS=2: each
    chunk's async all-gather beside the next chunk's network, both captured) equals it up to the conv
    rounding of the smaller per-chunk batches."""
    import json
    import os
    import socket
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "tools/tiled_collective.py"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    # on failure keep the child's error lines (the watchdog message precedes a long frame dump)
    why = [ln for ln in r.stderr.splitlines() if "rror" in ln or "what()" in ln or "abort" in ln.lower()]
    assert r.returncode == 0, "\n".join(why[:40]) + "\n...\n" + r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["collective"] is True, out
    assert out["octave_graph"] is True and out["step_graphs"] is False, out
    assert out["equal"] is True, out
    # chunked (2 chunks on 2 streams; each chunk's all-gather is issued from the capture-origin stream
    # behind that chunk's event, not from the chunk's stream, so the process group sees it as captured)
    assert out["chunks"] == 2 and out["chunk_streams"] == 2 and out["chunked_octave_graph"] is True, out
    assert out["chunked_cos"] > 0.995 and out["chunked_maxdiff"] < 5e-2, out


@pytest.mark.gpu
def test_gpu_capture_while_other_thread_polls_events(native_lib):
    """Every DeepDream capture is thread-local (runtime/capture.py): octave graphs (untiled and
    tiled) are captured while a second thread loops on Event.record/query/synchronize on its own
    stream - what the RCCL watchdog and the deconv service's completion thread do. In torch's
    default global mode those calls invalidate the capture (round-3 intermittent abort)."""
    import threading

    stop = threading.Event()
    polls = [0]
    errors = []

    def poller():
        try:
            s = torch.cuda.Stream()
            buf = torch.zeros(1 << 16, device="cuda")
            while not stop.is_set():
                with torch.cuda.stream(s):
                    buf.add_(1.0)
                    ev = torch.cuda.Event()
                    ev.record(s)
                ev.query()
                ev.synchronize()
                polls[0] += 1
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    inc = InceptionV3(0).build("cuda")
    res = ResNet50(0).build("cuda", torch.float16)
    xi = (torch.rand(2, 150, 150, 3, generator=torch.Generator().manual_seed(21)) * 2 - 1).cuda()
    xr = (torch.rand(2, 200, 260, 3, generator=torch.Generator().manual_seed(22)) * 2 - 1).cuda()
    si = DreamSettings(iterations=3, octaves=2, max_loss=None)
    sr = DreamSettings(layers=dict(RESNET_LAYERS), octaves=2, iterations=3, max_loss=None)
    want_i = DeepDream(inc, si, use_graphs=False).run(xi)
    want_r = TiledDeepDream(res, sr, tile=128, seed=4, use_graphs=False).run(xr)
    torch.cuda.synchronize()
    t = threading.Thread(target=poller, daemon=True)
    t.start()
    try:
        while polls[0] < 10 and not errors:  # the poller is running before the first capture opens
            pass
        before = polls[0]
        ddi = DeepDream(inc, si, use_graphs=True)
        got_i = ddi.run(xi)
        ddr = TiledDeepDream(res, sr, tile=128, seed=4, use_graphs=True)
        got_r = ddr.run(xr)
        torch.cuda.synchronize()
        during = polls[0] - before
    finally:
        stop.set()
        t.join(timeout=30)
    assert not errors, errors
    assert during > 0
    assert all(st.graph is not None for st in ddi._graphs.values())
    assert all(st.graph is not None for st in ddr._tgraphs.values())
    assert (got_i - want_i).abs().max() < 1e-3
    assert _cos(got_r - xr, want_r - xr) > 0.99
