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
