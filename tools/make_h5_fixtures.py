"""Writes the HDF5 fixtures of tests/test_h5lite.py with a REAL h5py (not importable by the framework's
interpreter; this container's conda Python 3.9 has h5py 3.3 / HDF5 1.10.6):

    /opt/conda/bin/python3.9 tools/make_h5_fixtures.py tests/fixtures

Two files with the same content, one in HDF5's earliest format (superblock 0, v1 object headers,
symbol-table groups: what keras-applications weight files are) and one in the latest (superblock 3,
v2 object headers, compact link messages). The content mimics a Keras 2 ``save_weights`` file
(root ``layer_names`` / ``backend`` / ``keras_version`` attributes, one group per layer with a
``weight_names`` attribute, datasets under ``<layer>/<layer>/kernel:0``) plus format corner cases:
an empty ``weight_names`` (layers without weights), a big-endian float dataset, an int32 dataset,
a compact-layout dataset, a variable-length string attribute, a scalar attribute, and one object
with enough attributes to need header continuation blocks. Every array is a closed-form function of
its shape (``_vals``), so the test recomputes the expected values without this script.
"""
import sys

import h5py
import numpy as np


def _vals(shape, dtype="float32"):
    n = int(np.prod(shape))
    return ((np.arange(n, dtype=np.float64) * 0.37) % 7.0 - 3.0).reshape(shape).astype(dtype)


LAYERS = [("input_1", None), ("block1_conv1", ((3, 3, 3, 4), (4,))), ("block1_pool", None),
          ("block2_conv1", ((3, 3, 4, 6), (6,))), ("fc1", ((24, 5), (5,)))]


def write(path, libver):
    with h5py.File(path, "w", libver=libver) as f:
        f.attrs["layer_names"] = np.array([n.encode("utf8") for n, _ in LAYERS])
        f.attrs["backend"] = b"tensorflow"
        f.attrs["keras_version"] = b"2.2.4"
        f.attrs["note"] = "vlen string attribute"  # h5py stores str as a variable-length string
        f.attrs["scalar_f64"] = np.float64(2.5)
        for name, shapes in LAYERS:
            g = f.create_group(name)
            if shapes is None:
                g.attrs["weight_names"] = np.array([])  # what Keras writes for a weightless layer
                continue
            g.attrs["weight_names"] = np.array([f"{name}/kernel:0".encode(), f"{name}/bias:0".encode()])
            sub = g.create_group(name)
            sub.create_dataset("kernel:0", data=_vals(shapes[0]))
            sub.create_dataset("bias:0", data=_vals(shapes[1]) * 0.1)
        x = f.create_group("extras")
        x.create_dataset("be_f32", data=_vals((5, 3), ">f4"))
        x.create_dataset("i32", data=np.arange(-6, 6, dtype=np.int32).reshape(3, 4))
        x.create_dataset("f16", data=_vals((7,), "float16"))
        # compact layout (raw data inside the object header)
        space = h5py.h5s.create_simple((4, 2))
        dcpl = h5py.h5p.create(h5py.h5p.DATASET_CREATE)
        dcpl.set_layout(h5py.h5d.COMPACT)
        dsid = h5py.h5d.create(x.id, b"compact_f32", h5py.h5t.IEEE_F32LE, space, dcpl=dcpl)
        dsid.write(h5py.h5s.ALL, h5py.h5s.ALL, _vals((4, 2)))
        many = x.create_group("many_attrs")
        for i in range(40):
            many.attrs[f"a{i:02d}"] = np.arange(i + 1, dtype=np.int64)


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else "tests/fixtures"
    write(f"{out}/keras_tiny_earliest.h5", "earliest")
    write(f"{out}/keras_tiny_latest.h5", "latest")
    print("wrote", out)
