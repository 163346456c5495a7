"""Strict GPU parity: the bf16 HIP backward vs the fp32 CPU backward fed the
GPU's OWN forward state -- its switch codes, its target activation and its selected filters.

The loose engine tests (test_engine_gpu.py) compare two independent forwards, where a bf16
rounding can flip a near-tied max-pool switch or top-k choice and move whole reconstruction
regions; that is a property of the reference's algorithm (first-max ties, app/deepdream.py:170-187),
not arithmetic error. Feeding the CPU backward the GPU's discrete decisions isolates the
arithmetic: every reconstruction must then reach cos >= 0.999 against the fp32 reference, and the
deprocessed uint8 mosaic a PSNR floor. Full-size VGG16 with the classifier head, every one of the
22 named layers (reference: app/deepdream.py:441-476 visits every layer), both modes."""
import math

import pytest
import torch

from deconv_api_amd import ops
from deconv_api_amd.engine.deconvnet import DeconvNet, ForwardState
from deconv_api_amd.models.vgg16 import VGG16

pytestmark = pytest.mark.gpu

LAYERS = ["block1_conv1", "block1_conv2", "block1_pool", "block2_conv1", "block2_conv2", "block2_pool",
          "block3_conv1", "block3_conv2", "block3_conv3", "block3_pool", "block4_conv1", "block4_conv2",
          "block4_conv3", "block4_pool", "block5_conv1", "block5_conv2", "block5_conv3", "block5_pool",
          "flatten", "fc1", "fc2", "predictions"]


@pytest.fixture(scope="module")
def engines(native_lib):
    m = VGG16.random(0)  # include_top: flatten / fc1 / fc2 / predictions targets
    gpu = DeconvNet(m.build("cuda", torch.bfloat16))
    cpu = DeconvNet(m.build("cpu", torch.float32))
    g = torch.Generator().manual_seed(21)
    img = torch.randint(0, 256, (1, 224, 224, 3), generator=g, dtype=torch.uint8)
    x = torch.empty(1, 224, 224, 8, dtype=torch.bfloat16, device="cuda")
    ops.resize_preprocess(img.cuda(), x)
    return gpu, cpu, x


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a @ b) / (a.norm() * b.norm() + 1e-30))


def _psnr(a, b):
    mse = float(((a.double() - b.double()) ** 2).mean())
    return math.inf if mse == 0 else 10 * math.log10(255.0 ** 2 / mse)


def test_layer_list_is_the_models(engines):
    gpu, _, _ = engines
    assert gpu.names[1:] == LAYERS


@pytest.mark.parametrize("mode", ["all", "max"])
@pytest.mark.parametrize("layer", LAYERS)
def test_strict_backward_parity(engines, layer, mode):
    gpu, cpu, x = engines
    st = gpu.forward(x, layer)
    idx, _ = gpu.select_filters(st.out, 4)
    rg = gpu.backward(st, idx, mode=mode).cpu()
    # the CPU backward on the GPU's discrete decisions and seed activations (fp32 arithmetic)
    stc = ForwardState(layer, st.out.float().cpu(), {k: v.cpu() for k, v in st.codes.items()})
    rc = cpu.backward(stc, idx.cpu(), mode=mode)
    assert rg.shape == rc.shape == (1, 4, 224, 224, 3)
    n = 0
    for k in range(4):
        if int(idx[0, k]) < 0 or float(rc[0, k].abs().max()) == 0.0:
            continue  # no positive filter / an all-zero reconstruction (nothing to compare)
        c = _cos(rg[0, k], rc[0, k])
        assert c >= 0.999, (layer, mode, k, c)
        n += 1
    assert n >= 1, (layer, mode, idx)
    mg = ops.deprocess_mosaic(rg.reshape(4, 224, 224, 3))
    mc = ops.deprocess_mosaic(rc.reshape(4, 224, 224, 3))
    assert _psnr(mg, mc) >= 30.0, (layer, mode, _psnr(mg, mc))


# ---- B > 1: cross-image indexing of the folded B*K backward (code_div / unpool_div = K) ----

B3_LAYERS = ["block1_pool", "block2_conv2", "block3_conv3", "block4_pool", "block5_conv3", "block5_pool", "fc1",
             "predictions"]


@pytest.fixture(scope="module")
def x3(native_lib):
    g = torch.Generator().manual_seed(5)
    img = torch.randint(0, 256, (3, 224, 224, 3), generator=g, dtype=torch.uint8)
    img[1] = img[1].flip(0) // 2  # three different images (different switches and top filters)
    img[2] = (img[2].float() * 0.6 + 80).to(torch.uint8)
    x = torch.empty(3, 224, 224, 8, dtype=torch.bfloat16, device="cuda")
    for b in range(3):
        ops.resize_preprocess(img[b].cuda(), x[b])
    return x


def _cpu_state(st, layer):
    return ForwardState(layer, st.out.float().cpu(), {k: v.cpu() for k, v in st.codes.items()},
                        {k: v.float().cpu() for k, v in st.outputs.items()})


@pytest.mark.parametrize("batch_topk", ["per_image", "global"])
@pytest.mark.parametrize("mode", ["all", "max"])
@pytest.mark.parametrize("layer", B3_LAYERS)
def test_strict_backward_parity_batch3(engines, x3, layer, mode, batch_topk):
    """B = 3 different images, K = 4: image b's chains must use image b's switches (a wrong
    ``b // K`` would pair reconstructions with another image's codes); per-image and the
    reference's across-batch ('global', app/deepdream.py:369-380) filter selection."""
    gpu, cpu, _ = engines
    st = gpu.forward(x3, layer)
    idx, _ = gpu.select_filters(st.out, 4, batch_topk)
    rg = gpu.backward(st, idx, mode=mode, batch_topk=batch_topk).cpu()
    rc = cpu.backward(_cpu_state(st, layer), idx.cpu(), mode=mode, batch_topk=batch_topk)
    assert rg.shape == rc.shape == (3, 4, 224, 224, 3)
    n = 0
    for b in range(3):
        for k in range(4):
            if int(idx[b, k]) < 0 or float(rc[b, k].abs().max()) == 0.0:
                continue
            c = _cos(rg[b, k], rc[b, k])
            assert c >= 0.999, (layer, mode, batch_topk, b, k, c)
            n += 1
    assert n >= 3, (layer, mode, batch_topk, idx)


@pytest.mark.parametrize("target", ["block3_conv3", "block5_pool", "fc1"])
def test_visualize_all_layers_k8_parity(engines, target):
    """The library API (app/deepdream.py:383-476: every named layer <= target, top-8 filters,
    across-batch sums) on the GPU engine, each of its reconstructions vs the fp32 CPU backward fed
    the same forward state and filters."""
    from deconv_api_amd.engine.deconvnet import visualize_all_layers

    gpu, cpu, x = engines
    res = visualize_all_layers(gpu, x, target, "all", all_layers=True, top=8)
    st = gpu.forward(x, target, fuse_pools=False, keep_all=True)
    stc = _cpu_state(st, target)
    ti = gpu.names.index(target)
    want_layers = [s.name for s in gpu.specs[1: ti + 1] if s.kind in ("conv", "pool", "flatten", "dense")]
    assert sorted(res) == sorted(want_layers)
    checked = 0
    for name, lst in res.items():
        out = st.outputs[name]
        idx, _ = gpu.select_filters(out, 8, "global")
        nsel = int((idx[0] >= 0).sum())
        assert len(lst) == nsel, (name, len(lst), nsel)
        sub = ForwardState(name, stc.outputs[name], stc.codes, stc.outputs)
        rc = cpu.backward(sub, idx.cpu(), "all", "global", layer=name)
        for kk in range(nsel):
            got = torch.from_numpy(lst[kk])
            if float(rc[0, kk].abs().max()) == 0.0:
                continue
            c = _cos(got, rc[0, kk])
            assert c >= 0.999, (target, name, kk, c)
            checked += 1
    assert checked >= 8 * len(want_layers) // 2, checked


# ---- strict FORWARD parity: the GPU's discrete decisions (switch codes, top-k) ----

POOL_CONVS = [("block1_conv2", "block1_conv1"), ("block2_conv2", "block2_conv1"), ("block3_conv3", "block3_conv2"),
              ("block4_conv3", "block4_conv2"), ("block5_conv3", "block5_conv2")]


@pytest.fixture(scope="module")
def cpu_bf16w(native_lib):
    """CPU fp32 engine on the bf16-ROUNDED weights the GPU uses: per layer, only accumulation order
    and the output rounding differ between the two."""
    m = VGG16.random(0, include_top=False)
    sd = {k: (v.to(torch.bfloat16).float() if v.is_floating_point() else v) for k, v in m.state_dict().items()}
    return DeconvNet(VGG16.from_state_dict(sd, specs=m.specs).build("cpu", torch.float32)), \
        DeconvNet(VGG16.from_state_dict(sd, specs=m.specs).build("cuda", torch.bfloat16))


@pytest.mark.parametrize("conv,prev", POOL_CONVS)
def test_strict_forward_switch_codes(cpu_bf16w, x3, conv, prev):
    """Each fused conv + 2x2 max-pool epilogue, fed the CPU forward's own (bf16-rounded) input of
    that layer: GPU switch codes == the fp32 CPU first-max codes on >= 99.9 % of the windows whose
    best and second-best differ by more than 1 % (all-zero windows, exact ties, must give code 0
    on both: first max in row-major order, app/deepdream.py:170-187)."""
    cpu, gpu = cpu_bf16w
    xc = x3.float().cpu()
    stc = cpu.forward(xc, prev, fuse_pools=False, keep_all=True)
    inp = stc.outputs[prev].to(torch.bfloat16)
    act = ops.conv2d(inp.float(), cpu.rt.convs[conv].fwd, relu=True)  # [N, H, W, C] fp32
    _, want = ops.maxpool2x2(act)
    _, got = ops.conv2d(inp.cuda(), gpu.rt.convs[conv].fwd, relu=True, epilogue="pool")
    got = got.cpu()
    assert got.shape == want.shape
    N, H, W, C = act.shape
    win = act.reshape(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, C, 4)
    top2 = win.topk(2, dim=-1).values
    zero = top2[..., 0] == 0
    clear = (top2[..., 0] - top2[..., 1]) > 1e-2 * top2[..., 0]
    assert torch.equal(got[zero], want[zero]) and not bool(got[zero].any())
    agree = float((got[clear] == want[clear]).double().mean())
    assert int(clear.sum()) > 0.2 * clear.numel(), (conv, int(clear.sum()))
    assert agree >= 0.999, (conv, agree, int(clear.sum()))


@pytest.mark.parametrize("layer", ["block1_pool", "block3_conv3", "block4_pool", "block5_conv3"])
def test_strict_forward_topk(cpu_bf16w, x3, layer):
    """Top-4 filter selection from the whole bf16 GPU forward vs the fp32 CPU forward on the same
    input: every GPU-selected filter's CPU channel sum is within 2 % of the CPU's 4th best, and the
    sets are equal whenever the CPU's 4th and 5th sums are more than 2 % apart."""
    cpu, gpu = cpu_bf16w
    st = gpu.forward(x3, layer)
    idx, _ = gpu.select_filters(st.out, 4)
    sums = ops.channel_sum(cpu.forward(x3.float().cpu(), layer).out)
    for b in range(x3.shape[0]):
        srt = torch.sort(sums[b], descending=True).values
        got = sums[b, idx[b].long().cpu()]
        assert float(got.min()) >= float(srt[3]) * 0.98, (layer, b, idx[b].tolist())
        if float(srt[3] - srt[4]) > 0.02 * float(srt[3]):
            want = set(torch.topk(sums[b], 4).indices.tolist())
            assert set(idx[b].tolist()) == want, (layer, b, idx[b].tolist(), sorted(want))
