"""CPU: the engine's decomposition (fused pools, B*K batched backward, seeded first step) equals
the float64 oracle of the reference semantics; the oracle equals naive loops. (BASELINE config 1
is the block1_conv1 case below on the full-size VGG16.)"""
import numpy as np
import pytest
import torch

from deconv_api_amd import ops
from deconv_api_amd.engine.deconvnet import DeconvNet, UnknownLayerError, visualize_all_layers
from deconv_api_amd.models.vgg16 import VGG16, VGG16_LAYER_NAMES
from deconv_api_amd.oracle import deconv_ref, naive

LAYERS = ["block1_conv1", "block1_conv2", "block1_pool", "block2_conv2", "block3_conv3", "block4_pool",
          "block5_conv3", "block5_pool", "flatten", "fc1", "fc2", "predictions"]


def _inputs(B, hw, seed=1):
    g = torch.Generator().manual_seed(seed)
    img = torch.randint(0, 256, (B, hw, hw, 3), generator=g).float()
    x3 = img - torch.tensor(ops.CAFFE_MEAN)
    x8 = torch.zeros(B, hw, hw, 8)
    x8[..., :3] = x3
    return x3, x8


@pytest.fixture(scope="module")
def small(small_specs):
    m = VGG16.random(0, specs=small_specs)
    return m, DeconvNet(m.build("cpu", torch.float32))


@pytest.mark.parametrize("layer", LAYERS)
@pytest.mark.parametrize("mode", ["all", "max"])
def test_target_matches_oracle(small, layer, mode):
    m, eng = small
    x3, x8 = _inputs(2, 32)
    ref = deconv_ref.visualize_all_layers(m, x3.double().numpy(), layer, mode, only_target=True)[layer]
    got = visualize_all_layers(eng, x8, layer, mode, all_layers=False)[layer]
    assert len(ref) == len(got) > 0
    for a, b in zip(ref, got):
        assert a.shape == b.shape
        np.testing.assert_allclose(b, a, rtol=1e-4, atol=1e-4 * np.abs(a).max())


def test_all_layers_parity(small):
    m, eng = small
    x3, x8 = _inputs(1, 32, seed=3)
    ref = deconv_ref.visualize_all_layers(m, x3.double().numpy(), "block3_conv2", "all")
    got = visualize_all_layers(eng, x8, "block3_conv2", "all", all_layers=True)
    assert list(ref.keys()) == list(got.keys())
    assert list(got.keys())[0] == "block3_conv2" and "block1_conv1" in got
    for k in ref:
        assert len(ref[k]) == len(got[k])
        for a, b in zip(ref[k], got[k]):
            assert a.shape == (32, 32, 3)
            np.testing.assert_allclose(b, a, rtol=1e-4, atol=1e-4 * np.abs(a).max())


def test_batched_equals_single(small):
    """B x K batched backward == K separate B=1 runs (per-image selection)."""
    _, eng = small
    _, x8 = _inputs(3, 32, seed=5)
    res = eng.run(x8, "block4_conv2", k=4, mosaic=False)
    for b in range(3):
        one = eng.run(x8[b:b + 1], "block4_conv2", k=4, mosaic=False)
        assert torch.equal(one.filters[0], res.filters[b])
        torch.testing.assert_close(one.recon[0], res.recon[b], rtol=1e-4, atol=1e-4 * float(res.recon[b].abs().max()))


def test_reconstructions_nonnegative(small):
    _, eng = small
    _, x8 = _inputs(2, 32)
    res = eng.run(x8, "fc2", k=4, mosaic=False)
    assert (res.recon >= 0).all()


def test_illegal_mode_and_unknown_layer(small):
    _, eng = small
    _, x8 = _inputs(1, 32)
    with pytest.raises(ValueError):
        eng.run(x8, "block1_conv1", mode="bogus")
    with pytest.raises(UnknownLayerError):
        eng.run(x8, "block9_conv1")
    with pytest.raises(UnknownLayerError):
        eng.run(x8, "input_1")


def test_naive_pool_and_topk_match_oracle():
    rng = np.random.default_rng(0)
    # tie-heavy post-ReLU input
    x = np.maximum(rng.integers(-3, 3, size=(2, 8, 8, 5)).astype(np.float64), 0)
    p_ref, s_ref = naive.maxpool_with_switch(x)
    dp = deconv_ref.DPooling("p")
    p = dp.up(torch.as_tensor(x))
    np.testing.assert_array_equal(p.numpy(), p_ref)
    np.testing.assert_array_equal(dp.switch.numpy(), s_ref)
    y = rng.standard_normal((2, 4, 4, 5))
    np.testing.assert_allclose(dp.down(torch.as_tensor(y)).numpy(), naive.unpool(y, s_ref))
    out = np.maximum(rng.integers(-2, 3, size=(1, 3, 3, 40)).astype(np.float64), 0)
    assert deconv_ref.find_top_filters(torch.as_tensor(out)) == naive.top_filters(out)
    # the op-level pool agrees too (first-max ties)
    v, c = ops.maxpool_switch_ref(torch.as_tensor(x))
    np.testing.assert_array_equal(v.numpy(), p_ref)
    recon = ops.unpool_ref(torch.as_tensor(y), c)
    np.testing.assert_allclose(recon.numpy(), naive.unpool(y, s_ref))


def test_naive_conv_matches_oracle_conv():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((1, 6, 7, 4))
    w = rng.standard_normal((3, 3, 4, 5))
    b = rng.standard_normal(5)
    dc = deconv_ref.DConv("c", torch.as_tensor(w), torch.as_tensor(b))
    np.testing.assert_allclose(dc.up(torch.as_tensor(x)).numpy(), np.maximum(naive.conv3x3_same(x, w, b), 0),
                               rtol=1e-10, atol=1e-10)
    y = rng.standard_normal((1, 6, 7, 5))
    wd = w.transpose(0, 1, 3, 2)[::-1, ::-1]
    np.testing.assert_allclose(dc.down(torch.as_tensor(y)).numpy(), np.maximum(naive.conv3x3_same(y, wd), 0),
                               rtol=1e-10, atol=1e-10)


def test_topk_positive_stable_ties():
    v = torch.tensor([[0.0, 3.0, 3.0, -1.0, 2.0, 3.0, 0.5]])
    idx, val = ops.topk_positive(v, 8)
    assert idx[0].tolist() == [1, 2, 5, 4, 6, -1, -1, -1]
    assert val[0, :5].tolist() == [3.0, 3.0, 3.0, 2.0, 0.5]


def test_full_vgg16_block1_conv1_cpu():
    """BASELINE config 1: VGG16 block1_conv1 deconvnet on one 224x224 image, CPU reference."""
    m = VGG16.random(0, include_top=False)
    assert VGG16_LAYER_NAMES[1] == "block1_conv1" and len(VGG16_LAYER_NAMES) == 23
    eng = DeconvNet(m.build("cpu", torch.float32))
    x3, x8 = _inputs(1, 224, seed=7)
    ref = deconv_ref.visualize_all_layers(m, x3.double().numpy(), "block1_conv1", "all", only_target=True)
    res = eng.run(x8, "block1_conv1", k=4)
    for k in range(4):
        np.testing.assert_allclose(res.recon[0, k].numpy(), ref["block1_conv1"][k], rtol=1e-4,
                                   atol=1e-4 * np.abs(ref["block1_conv1"][k]).max())
    mos = deconv_ref.deprocess_image(deconv_ref.mosaic(ref["block1_conv1"][:4]))[..., ::-1]
    diff = np.abs(res.mosaic[0].numpy().astype(int) - mos.astype(int))
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-3


def test_vgg16_param_count():
    m = VGG16.random(0)
    assert m.num_params() == 138357544  # Keras VGG16(include_top=True)
