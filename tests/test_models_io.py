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
