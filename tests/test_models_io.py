"""CPU: checkpoint import/export (Keras .h5 layout mapping, safetensors round trip)."""
import numpy as np
import pytest
import torch

from deconv_api_amd.models.keras_import import keras_state_from_h5_like
from deconv_api_amd.models.vgg16 import VGG16, VGG16_SPECS


class FakeNode(dict):
    def __init__(self, *a, attrs=None, **k):
        super().__init__(*a, **k)
        self.attrs = attrs or {}


def _fake_h5(model: VGG16):
    """Mimic vgg16_weights_tf_dim_ordering_tf_kernels.h5: group/<layer>/<layer>/{kernel:0,bias:0}."""
    root = FakeNode(attrs={"layer_names": [s.name.encode() for s in VGG16_SPECS]})
    for s in VGG16_SPECS:
        if s.name in model.params:
            k, b = model.params[s.name]
            inner = FakeNode({"kernel:0": k.numpy(), "bias:0": b.numpy()})
            root[s.name] = FakeNode({s.name: inner}, attrs={"weight_names": [f"{s.name}/kernel:0".encode(),
                                                                                f"{s.name}/bias:0".encode()]})
        else:
            root[s.name] = FakeNode(attrs={"weight_names": []})
    return root


def test_keras_h5_mapping_roundtrip():
    m = VGG16.random(3)
    sd = keras_state_from_h5_like(_fake_h5(m))
    m2 = VGG16.from_state_dict(sd)
    for name, (k, b) in m.params.items():
        assert torch.equal(m2.params[name][0], k) and torch.equal(m2.params[name][1], b)


def test_keras_h5_shape_check():
    m = VGG16.random(3)
    f = _fake_h5(m)
    f["fc2"]["fc2"]["kernel:0"] = np.zeros((10, 10), np.float32)
    with pytest.raises(ValueError):
        keras_state_from_h5_like(f)


def test_safetensors_roundtrip(tmp_path):
    m = VGG16.random(5, include_top=False)
    p = str(tmp_path / "w.safetensors")
    m.save(p)
    m2 = VGG16.load(p)
    assert set(m2.params) == set(m.params)
    for n in m.params:
        assert torch.equal(m.params[n][0], m2.params[n][0])


def _fake_keras_dream_h5(model, kind, tf2_names=False, bn_scale=False):
    """Keras HDF5 layout of InceptionV3 (conv2d_N + batch_normalization_N, scale=False) or
    ResNet-50 (convS_blockB_K_conv + _bn) built from random BN statistics; returns (file, the
    expected folded state)."""
    from deconv_api_amd.models.inception_v3 import fold_bn

    g = torch.Generator().manual_seed(7)
    root = FakeNode(attrs={"layer_names": []})
    expect = {}

    def add(lname, arrays):
        root.attrs["layer_names"].append(lname.encode())
        names = [f"{lname}/w{i}:0".encode() for i in range(len(arrays))]
        root[lname] = FakeNode({lname: FakeNode({f"w{i}:0": a for i, a in enumerate(arrays)})},
                               attrs={"weight_names": names})

    units = list(model.units.items())
    for i, (n, u) in enumerate(units):
        w = torch.randn(u.w.shape, generator=g) * 0.1
        co = u.cout
        beta, mean = torch.randn(co, generator=g), torch.randn(co, generator=g) * 0.1
        var = torch.rand(co, generator=g) + 0.5
        gamma = torch.rand(co, generator=g) + 0.5 if (kind == "resnet" or bn_scale) else None
        hwio = w.permute(2, 3, 1, 0).numpy()
        if kind == "inception":
            sfx = "" if (tf2_names and i == 0) else f"_{i if tf2_names else i + 1}"
            add(f"conv2d{sfx}", [hwio])
            bn = [beta, mean, var] if gamma is None else [gamma, beta, mean, var]
            add(f"batch_normalization{sfx}", [t.numpy() for t in bn])
            expect[n] = fold_bn(w, gamma, beta, mean, var, 1e-3)
        else:
            cb = torch.randn(co, generator=g) * 0.1
            add(n, [hwio, cb.numpy()])
            add(n[:-5] + "_bn", [t.numpy() for t in (gamma, beta, mean, var)])
            expect[n] = fold_bn(w, gamma, beta, mean, var, 1.001e-5, cb)
    return root, expect


@pytest.mark.parametrize("tf2_names", [False, True])
def test_inception_keras_import(tf2_names, tmp_path):
    from deconv_api_amd.models import dream_import as di
    from deconv_api_amd.models.inception_v3 import InceptionV3

    m = InceptionV3(1)
    f, expect = _fake_keras_dream_h5(m, "inception", tf2_names=tf2_names)
    di.apply_state(m, di.state_from_h5_like(f, m))
    for n, (w, b) in expect.items():
        torch.testing.assert_close(m.units[n].w, w)
        torch.testing.assert_close(m.units[n].b, b)
    # folded safetensors round trip, then a CPU forward runs on the imported weights
    p = str(tmp_path / "iv3.safetensors")
    di.save(m, p)
    m2 = di.load_weights(InceptionV3(2), p).build("cpu")
    for n in expect:
        assert torch.equal(m2.units[n].w, m.units[n].w)
    out = m2.forward(torch.rand(1, 75, 75, 3), ["mixed2"])["mixed2"]
    assert out.shape[-1] == 288 and torch.isfinite(out).all()


def test_resnet50_keras_import_and_shape_check():
    from deconv_api_amd.models import dream_import as di
    from deconv_api_amd.models.resnet50 import ResNet50

    m = ResNet50(1)
    f, expect = _fake_keras_dream_h5(m, "resnet")
    di.apply_state(m, di.state_from_h5_like(f, m))
    for n, (w, b) in expect.items():
        torch.testing.assert_close(m.units[n].w, w)
        torch.testing.assert_close(m.units[n].b, b)
    f["conv2_block1_2_conv"]["conv2_block1_2_conv"]["w0:0"] = np.zeros((3, 3, 64, 65), np.float32)
    with pytest.raises(ValueError):
        di.state_from_h5_like(f, ResNet50(1))
