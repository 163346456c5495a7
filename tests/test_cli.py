"""python -m deconv_api_amd.cli (CPU engine): deconv mosaics and DeepDream outputs written as JPEG files, the
same images the HTTP routes return; an unknown layer fails before any compute."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np
import pytest
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cli(*args, timeout=600):
    env = dict(os.environ, DV_DEVICE="cpu", DV_HIP_GRAPHS="0", DV_LOG_JSON="0", OMP_NUM_THREADS="4", PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "deconv_api_amd.cli", *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.timeout(600)
def test_cli_deconv_and_dream(tmp_path):
    rng = np.random.default_rng(4)
    a, b = tmp_path / "a.png", tmp_path / "b.jpg"
    Image.fromarray(rng.integers(0, 256, (50, 70, 3), dtype=np.uint8)).save(a)
    Image.fromarray(rng.integers(0, 256, (80, 80, 3), dtype=np.uint8)).save(b, quality=90)
    out = tmp_path / "out"
    r = _cli("deconv", str(a), str(b), "--layer", "block1_conv1", "--out-dir", str(out))
    assert r.returncode == 0, r.stderr[-2000:]
    for stem in ("a", "b"):
        with Image.open(out / f"{stem}_block1_conv1.jpg") as im:
            assert im.format == "JPEG" and im.size == (448, 448)
    # the same mosaic as the service's for that image (the API's data URL holds the same JPEG bytes)
    from deconv_api_amd.codec import encode_data_url, read_data_url
    from deconv_api_amd.codec.image import make_data_url
    from deconv_api_amd.config import Config
    from deconv_api_amd.serve.service import DeconvService

    svc = DeconvService(Config.from_env(device="cpu", hip_graphs=False))
    try:
        want = svc.run_batch("block1_conv1", [read_data_url(make_data_url(np.asarray(Image.open(a).convert("RGB"))))])
    finally:
        svc.close()
    import base64
    from urllib.parse import unquote

    url = encode_data_url(np.ascontiguousarray(want[0]), 95)
    jpeg = base64.b64decode(unquote(url.split(",", 1)[1]))
    assert (out / "a_block1_conv1.jpg").read_bytes() == jpeg

    r = _cli("dream", str(b), "--octaves", "1", "--steps", "1", "--out-dir", str(out))
    assert r.returncode == 0, r.stderr[-2000:]
    with Image.open(out / "b_dream_inception_v3.jpg") as im:
        assert im.size == (80, 80)

    r = _cli("deconv", str(a), "--layer", "nope", "--out-dir", str(out))
    assert r.returncode == 2 and r.stderr.startswith("error: unknown layer"), r.stderr[-500:]


def test_cli_layers():
    r = _cli("layers", timeout=120)
    names = r.stdout.split()
    assert r.returncode == 0 and names[0] == "block1_conv1" and "predictions" in names and "input_1" not in names


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_cli_deconv_on_gpu(tmp_path, native_lib):
    """The CLI on the HIP engine (bf16, hipGraph batch path) writes the mosaic of each file."""
    rng = np.random.default_rng(6)
    paths = []
    for i, shape in enumerate([(224, 224, 3), (300, 200, 3)]):
        pth = tmp_path / f"g{i}.png"
        Image.fromarray(rng.integers(0, 256, shape, dtype=np.uint8)).save(pth)
        paths.append(str(pth))
    env_dev = {"DV_DEVICE": "cuda", "DV_HIP_GRAPHS": "1"}
    r = subprocess.run([sys.executable, "-m", "deconv_api_amd.cli", "deconv", *paths, "--layer", "block5_conv3",
                        "--out-dir", str(tmp_path)], cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, DV_LOG_JSON="0", PYTHONPATH=ROOT, **env_dev))
    assert r.returncode == 0, r.stderr[-2000:]
    for i in range(2):
        with Image.open(tmp_path / f"g{i}_block5_conv3.jpg") as im:
            assert im.size == (448, 448) and np.asarray(im).std() > 1.0
