"""GPU: the bf16 HIP engine vs the fp32 CPU engine (which itself matches the float64 oracle,
tests/test_oracle_engine.py), on a scaled VGG16 and on the full-size VGG16."""
import numpy as np
import pytest
import torch

from deconv_api_amd import ops
from deconv_api_amd.engine.deconvnet import DeconvNet
from deconv_api_amd.models.vgg16 import VGG16

pytestmark = pytest.mark.gpu


def _x8(B, hw, seed=0):
    g = torch.Generator().manual_seed(seed)
    img = torch.randint(0, 256, (B, hw, hw, 3), generator=g).float()
    x8 = torch.zeros(B, hw, hw, 8)
    x8[..., :3] = img - torch.tensor(ops.CAFFE_MEAN)
    return x8


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a @ b) / (a.norm() * b.norm() + 1e-30))


def _compare(model, B, hw, layers, seed=0):
    cpu = DeconvNet(model.build("cpu", torch.float32))
    gpu = DeconvNet(model.build("cuda", torch.bfloat16))
    x = _x8(B, hw, seed).to(torch.bfloat16).float()
    for layer in layers:
        st_g = gpu.forward(x.to(torch.bfloat16).cuda(), layer)
        st_c = cpu.forward(x, layer)
        rel = float((st_g.out.float().cpu() - st_c.out).abs().max() / st_c.out.abs().max())
        assert rel < 5e-2, (layer, rel)
        idx, _ = gpu.select_filters(st_g.out, 4)
        rg = gpu.backward(st_g, idx).cpu()
        rc = cpu.backward(st_c, idx.cpu())
        assert rg.shape == rc.shape == (B, 4, hw, hw, 3)
        for b in range(B):
            for k in range(4):
                if idx[b, k] < 0:
                    continue
                c = _cos(rg[b, k], rc[b, k])
                assert c > 0.98, (layer, b, k, c)


def test_engine_small_all_targets(native_lib, small_specs):
    m = VGG16.random(0, specs=small_specs)
    _compare(m, 3, 32, ["block1_conv1", "block1_pool", "block2_conv2", "block3_conv3", "block5_conv3",
                        "block5_pool", "flatten", "fc1", "predictions"])


def test_engine_full_vgg16_block5_conv3(native_lib):
    m = VGG16.random(0)
    _compare(m, 2, 224, ["block5_conv3", "block2_pool"], seed=1)


def test_engine_mosaic_and_run(native_lib):
    m = VGG16.random(0, include_top=False)
    gpu = DeconvNet(m.build("cuda", torch.bfloat16))
    x = _x8(4, 224, 2).to(torch.bfloat16).cuda()
    res = gpu.run(x, "block5_conv3", k=4)
    assert res.mosaic.shape == (4, 448, 448, 3) and res.mosaic.dtype == torch.uint8
    assert (res.filters >= 0).all()
    # same mosaic from the CPU deprocess of the GPU reconstructions
    ref = ops.deprocess_mosaic(res.recon.reshape(16, 224, 224, 3).cpu())
    d = (res.mosaic.cpu().int() - ref.int()).abs()
    assert d.max() <= 1
