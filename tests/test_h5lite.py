"""CPU: the dependency-free HDF5 reader (models/h5lite.py) against files written by a REAL h5py.

The fixtures (tests/fixtures/keras_tiny_{earliest,latest}.h5) were written by h5py 3.3 / HDF5 1.10.6
(tools/make_h5_fixtures.py, run with this container's conda Python 3.9, the only interpreter here
that has h5py); every array in them is ``_vals(shape)``, recomputed below. The full-size VGG16 test
writes a keras-applications-layout file with that same h5py when it is available (skipped
otherwise) and loads it through ``VGG16.load`` without h5py. Parity against the real ImageNet
weight file stays unpinned: no copy of it exists in this image.
"""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from deconv_api_amd.models import h5lite

FIX = os.path.join(os.path.dirname(__file__), "fixtures")
FILES = ["keras_tiny_earliest.h5", "keras_tiny_latest.h5"]
CONDA_PY = "/opt/conda/bin/python3.9"


def _vals(shape, dtype="float32"):
    n = int(np.prod(shape))
    return ((np.arange(n, dtype=np.float64) * 0.37) % 7.0 - 3.0).reshape(shape).astype(dtype)


LAYERS = [("input_1", None), ("block1_conv1", ((3, 3, 3, 4), (4,))), ("block1_pool", None),
          ("block2_conv1", ((3, 3, 4, 6), (6,))), ("fc1", ((24, 5), (5,)))]


@pytest.mark.parametrize("fn", FILES)
def test_h5lite_keras_layout(fn):
    with h5lite.File(os.path.join(FIX, fn)) as f:
        assert [n.decode() for n in f.attrs["layer_names"]] == [n for n, _ in LAYERS]
        assert f.attrs["layer_names"].dtype.kind == "S"  # fixed-length strings, as Keras writes them
        assert f.attrs["backend"] in (b"tensorflow", "tensorflow")
        assert f.attrs["note"] == "vlen string attribute"  # variable-length string (global heap)
        assert float(f.attrs["scalar_f64"]) == 2.5
        assert set(f.keys()) == {n for n, _ in LAYERS} | {"extras"}
        for name, shapes in LAYERS:
            g = f[name]
            wn = g.attrs["weight_names"]
            if shapes is None:
                assert len(wn) == 0
                continue
            assert [w.decode() for w in wn] == [f"{name}/kernel:0", f"{name}/bias:0"]
            assert f"{name}/kernel:0" in g and "nope" not in g
            k = np.asarray(g[f"{name}/kernel:0"], dtype=np.float32)
            b = np.asarray(f[f"{name}/{name}/bias:0"])
            assert k.shape == shapes[0] and np.array_equal(k, _vals(shapes[0]))
            assert b.dtype == np.float32 and np.array_equal(b, _vals(shapes[1]) * np.float32(0.1))
        x = f["extras"]
        be = np.asarray(x["be_f32"])
        assert be.dtype.isnative and np.array_equal(be, _vals((5, 3)))
        assert np.array_equal(np.asarray(x["i32"]), np.arange(-6, 6, dtype=np.int32).reshape(3, 4))
        assert np.array_equal(np.asarray(x["f16"]), _vals((7,), "float16"))
        assert np.array_equal(np.asarray(x["compact_f32"]), _vals((4, 2)))
        assert x["i32"].shape == (3, 4) and x["i32"][1, 2] == 0


def test_h5lite_header_continuation():
    """40 attributes on one group: v1 object header continuation blocks (earliest format)."""
    with h5lite.File(os.path.join(FIX, FILES[0])) as f:
        a = f["extras/many_attrs"].attrs
        assert len(a) == 40
        for i in range(40):
            assert np.array_equal(a[f"a{i:02d}"], np.arange(i + 1))


def test_h5lite_unsupported_is_named():
    """The latest format moves > 8 attributes to dense (fractal-heap) storage: outside the Keras
    subset, refused with an error that names it (never silently wrong)."""
    with h5lite.File(os.path.join(FIX, FILES[1])) as f:
        with pytest.raises(h5lite.H5Unsupported, match="dense attribute"):
            f["extras/many_attrs"]


def test_h5lite_not_hdf5(tmp_path):
    p = tmp_path / "x.h5"
    p.write_bytes(b"not an hdf5 file" * 64)
    with pytest.raises(h5lite.H5Error):
        h5lite.File(str(p))


_WRITE_VGG = r"""
import sys, h5py, numpy as np
d = np.load(sys.argv[1])
names = [n for n in d.files if n.endswith('.kernel')]
layers = ['input_1'] + [n[:-7] for n in names]
with h5py.File(sys.argv[2], 'w') as f:
    f.attrs['layer_names'] = np.array([n.encode() for n in layers])
    f.attrs['backend'] = np.bytes_('tensorflow')
    f.create_group('input_1').attrs['weight_names'] = np.array([])
    for n in names:
        l = n[:-7]
        g = f.create_group(l)
        g.attrs['weight_names'] = np.array([f'{l}/kernel:0'.encode(), f'{l}/bias:0'.encode()])
        s = g.create_group(l)
        s.create_dataset('kernel:0', data=d[n])
        s.create_dataset('bias:0', data=d[l + '.bias'])
"""


@pytest.mark.skipif(not os.path.exists(CONDA_PY), reason="no interpreter with h5py to write the file")
@pytest.mark.parametrize("whole_file", [True, False])
def test_vgg16_load_keras_h5_without_h5py(tmp_path, monkeypatch, whole_file):
    """VGG16.load on a notop keras-applications-layout file (59 MB, written by real h5py): every
    kernel and bias equal to the source weights. ``whole_file=False`` forces the per-dataset
    ``np.fromfile`` path used for files over ``h5lite.SMALL_BYTES`` (the 553 MB ImageNet file)."""
    from deconv_api_amd.models.vgg16 import VGG16

    probe = subprocess.run([CONDA_PY, "-c", "import h5py"], capture_output=True)
    if probe.returncode != 0:
        pytest.skip("conda python without h5py")
    m = VGG16.random(7, include_top=False)
    npz = tmp_path / "w.npz"
    np.savez(npz, **{k: v.numpy() for k, v in m.state_dict().items()})
    h5 = tmp_path / "vgg16_notop.h5"
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "PYTHONHOME")}
    subprocess.run([CONDA_PY, "-c", _WRITE_VGG, str(npz), str(h5)], check=True, env=env, cwd=str(tmp_path))
    if not whole_file:
        monkeypatch.setattr(h5lite, "SMALL_BYTES", 1 << 20)
    monkeypatch.setitem(sys.modules, "h5py", None)  # as in the shipped container: h5py not importable
    m2 = VGG16.load(str(h5))
    assert set(m2.params) == set(m.params)
    for n, (k, b) in m.params.items():
        assert torch.equal(m2.params[n][0], k) and torch.equal(m2.params[n][1], b), n
