"""CPU: HTTP surface parity with app/main.py (routes, form fields, CORS, response format)."""
import base64
import io
import json
from urllib.parse import quote

import numpy as np
import pytest
import torch
from PIL import Image

from deconv_api_amd import ops
from deconv_api_amd.api.app import create_app
from deconv_api_amd.api.forms import encode_multipart, parse_form, parse_multipart, parse_urlencoded
from deconv_api_amd.codec import DATA_URL_PREFIX, make_data_url, parse_result_data_url, read_data_url
from deconv_api_amd.config import Config
from deconv_api_amd.engine.deconvnet import DeconvNet
from deconv_api_amd.models.vgg16 import VGG16
from deconv_api_amd.serve.service import DeconvService

pytestmark = pytest.mark.filterwarnings("ignore::DeprecationWarning")


@pytest.fixture(scope="module")
def client(small_specs):
    from fastapi.testclient import TestClient

    cfg = Config.from_env(device="cpu", image_size=32, max_batch=8, batch_timeout_ms=1.0, codec_workers=2)
    eng = DeconvNet(VGG16.random(0, specs=small_specs).build("cpu", torch.float32))
    svc = DeconvService(cfg, engine=eng)
    app = create_app(svc, cfg)
    with TestClient(app) as c:
        yield c, svc
    svc.close()


def _img(h=40, w=50, seed=0):
    return np.random.default_rng(seed).integers(0, 256, size=(h, w, 3), dtype=np.uint8)


def test_health_check(client):
    c, _ = client
    r = c.get("/health-check")
    assert r.status_code == 200 and r.json() == {"healthy": "true"}


def test_cors(client):
    c, _ = client
    r = c.get("/health-check", headers={"Origin": "http://example.com"})
    assert r.headers["access-control-allow-origin"] == "*"
    pre = c.options("/", headers={"Origin": "http://x.y", "Access-Control-Request-Method": "POST",
                                  "Access-Control-Request-Headers": "content-type"})
    assert pre.status_code == 200 and pre.headers["access-control-allow-origin"] == "*"


def _check_url(s, size=64):
    assert isinstance(s, str) and s.startswith(DATA_URL_PREFIX)
    payload = s[len(DATA_URL_PREFIX):]
    assert "+" not in payload and "=" not in payload  # quote() escapes them (quirk Q3)
    rgb = parse_result_data_url(s)
    assert rgb.shape == (size, size, 3)
    return rgb


def test_post_urlencoded_and_multipart(client):
    c, _ = client
    url = make_data_url(_img(), "PNG")
    r = c.post("/", data={"file": url, "layer": "block3_conv1"})
    assert r.status_code == 200 and r.headers["content-type"].startswith("application/json")
    a = _check_url(r.json())
    body, ct = encode_multipart({"file": url, "layer": "block3_conv1"})
    r2 = c.post("/", content=body, headers={"content-type": ct})
    assert r2.status_code == 200
    b = _check_url(r2.json())
    assert np.array_equal(a, b)


def test_post_matches_engine(client):
    """The HTTP result equals the engine's mosaic for the same image (up to JPEG)."""
    c, svc = client
    img = _img(32, 32, seed=3)
    r = c.post("/", data={"file": make_data_url(img, "PNG"), "layer": "block2_pool"})
    got = _check_url(r.json()).astype(int)
    x = svc.preprocess([img])
    want = svc.engine.run(x, "block2_pool", k=4).mosaic[0].numpy()
    from deconv_api_amd.codec import encode_data_url

    assert np.array_equal(got, parse_result_data_url(encode_data_url(want)).astype(int))


def test_errors(client):
    c, _ = client
    r = c.post("/", data={"layer": "block1_conv1"})
    assert r.status_code == 422 and r.json()["detail"][0]["loc"] == ["body", "file"]
    r = c.post("/", data={"file": make_data_url(_img(), "PNG"), "layer": "nope"})
    assert r.status_code == 400 and "unknown layer" in r.json()["detail"]
    r = c.post("/", data={"file": "no-comma-here", "layer": "block1_conv1"})
    assert r.status_code == 400
    r = c.post("/", data={"file": "data:image/png;base64," + base64.b64encode(b"junk").decode(), "layer": "fc1"})
    assert r.status_code == 400
    r = c.post("/", data={"file": make_data_url(_img(), "PNG"), "layer": "input_1"})
    assert r.status_code == 400


def test_openapi_form_schema(client):
    c, _ = client
    spec = c.get("/openapi.json").json()
    body = spec["paths"]["/"]["post"]["requestBody"]["content"]
    for ct in ("application/x-www-form-urlencoded", "multipart/form-data"):
        assert sorted(body[ct]["schema"]["required"]) == ["file", "layer"]
    assert "/health-check" in spec["paths"]
    assert c.get("/docs").status_code == 200


def test_metrics_ready_layers(client):
    c, _ = client
    c.post("/", data={"file": make_data_url(_img(), "JPEG"), "layer": "block1_conv1"})
    m = c.get("/metrics").text
    assert "dv_requests_total" in m and "dv_request_latency_seconds_bucket" in m
    rd = c.get("/ready")
    assert rd.status_code == 200 and rd.json()["ready"] is True
    assert "block5_conv3" in c.get("/layers").json()["layers"]


def test_concurrent_requests_batch(client):
    """Concurrent requests are coalesced into engine batches and each gets its own answer."""
    import concurrent.futures as cf

    c, svc = client
    before = svc.batches
    imgs = [_img(30 + i, 30, seed=i) for i in range(6)]
    with cf.ThreadPoolExecutor(6) as ex:
        rs = list(ex.map(lambda im: c.post("/", data={"file": make_data_url(im, "PNG"), "layer": "block4_conv1"}), imgs))
    assert all(r.status_code == 200 for r in rs)
    outs = [_check_url(r.json()) for r in rs]
    assert not np.array_equal(outs[0], outs[1])
    assert svc.batches - before <= 6


def test_form_parsers():
    assert parse_urlencoded(b"a=1+2&b=%2B%3D&a=3") == {"a": "1 2", "b": "+="}
    body, ct = encode_multipart({"file": "data:x;base64,AAA+/=", "layer": "fc1"})
    assert parse_multipart(body, ct) == {"file": "data:x;base64,AAA+/=", "layer": "fc1"}
    assert parse_form(body, ct)["layer"] == "fc1"
    raw = (b"--B\r\nContent-Disposition: form-data; name=\"layer\"\r\n\r\nblock1_pool\r\n"
           b"--B\r\nContent-Disposition: form-data; name=\"file\"; filename=\"x.txt\"\r\nContent-Type: text/plain\r\n\r\n"
           b"abc\r\n--B--\r\n")
    assert parse_form(raw, 'multipart/form-data; boundary="B"') == {"layer": "block1_pool", "file": "abc"}


def test_codec_quirks():
    img = _img(10, 12)
    url = make_data_url(img, "PNG")
    # lenient base64: characters outside the alphabet are dropped like base64.b64decode does
    assert np.array_equal(read_data_url(url.replace("base64,", "base64,\n")), img)
    gray = Image.fromarray(img[..., 0])
    buf = io.BytesIO()
    gray.save(buf, "PNG")
    g3 = read_data_url("data:image/png;base64," + base64.b64encode(buf.getvalue()).decode())
    assert g3.shape == (10, 12, 3)
    rgba = Image.fromarray(np.dstack([img, np.full((10, 12), 7, np.uint8)]), "RGBA")
    buf = io.BytesIO()
    rgba.save(buf, "PNG")
    assert np.array_equal(read_data_url("data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()), img)
    assert quote("ab+c/d=") == "ab%2Bc/d%3D"
    from deconv_api_amd.codec.image import quote_b64

    for n in (0, 1, 2, 3, 1000, 4097):
        b = base64.b64encode(np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8).tobytes()).decode()
        assert quote_b64(b) == quote(b)


def test_resize_oracle_properties():
    img = _img(448, 448)
    r = ops.resize_u8_ref(img)  # exact 2x: INTER_AREA fast path
    ref = ((img[0::2, 0::2].astype(int) + img[0::2, 1::2] + img[1::2, 0::2] + img[1::2, 1::2] + 2) >> 2)
    assert np.array_equal(r, ref)
    const = np.full((300, 500, 3), 77, np.uint8)
    assert (ops.resize_u8_ref(const) == 77).all()
    up = ops.resize_u8_ref(_img(100, 57))
    assert up.shape == (224, 224, 3) and up.dtype == np.uint8


def _native_or_skip():
    from deconv_api_amd.ops import native

    if not native.available():
        pytest.skip("native extension not built")
    return native.lib()


def test_native_jpeg_encoder():
    """csrc/jpeg_enc.cpp: a standard baseline JPEG (PIL decodes it), close to PIL's q95 4:2:0
    encode of the same image, restart-segmented scans decode identically, and the data URL is
    exactly prefix + quote(base64(jpeg))."""
    lib = _native_or_skip()
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:96, 0:120].astype(np.float32)
    base = 128 + 60 * np.sin(xx / 7) * np.cos(yy / 11) + rng.normal(0, 8, (96, 120))
    img = np.clip(np.stack([base, base[::-1], 255 - base], -1), 0, 255).astype(np.uint8)
    for im in (img, np.ascontiguousarray(img[:37, :53])):
        jb = lib.jpeg_encode(torch.from_numpy(im), 95)
        assert jb[:2] == b"\xff\xd8" and jb[-2:] == b"\xff\xd9"
        dec = np.asarray(Image.open(io.BytesIO(jb)).convert("RGB")).astype(int)
        buf = io.BytesIO()
        Image.fromarray(im).save(buf, "JPEG", quality=95, subsampling=2)
        ref = np.asarray(Image.open(io.BytesIO(buf.getvalue())).convert("RGB")).astype(int)
        assert dec.shape == im.shape and np.abs(dec - ref).mean() < 2.0
        for threads in (1, 3, 7):
            url = lib.jpeg_data_urls(torch.from_numpy(im[None].copy()), 95, DATA_URL_PREFIX, threads)[0]
            assert np.array_equal(parse_result_data_url(url).astype(int), dec)  # restart segments
    url = lib.jpeg_data_urls(torch.from_numpy(img[None].copy()), 95, DATA_URL_PREFIX, 1)[0]
    assert url == DATA_URL_PREFIX + quote(base64.b64encode(lib.jpeg_encode(torch.from_numpy(img), 95)).decode())


def test_deepdream_bad_inputs_are_400(client):
    """/deepdream: malformed body, unknown charset and non-numeric fields are client errors."""
    from deconv_api_amd.api.forms import encode_multipart

    client, _ = client
    r = client.post("/deepdream", content=b"--x\r\n", headers={"content-type": "multipart/form-data"})
    assert r.status_code == 400, r.text
    body = (b'--bb\r\nContent-Disposition: form-data; name="file"\r\nContent-Type: text/plain; charset=nope-9\r\n\r\n'
            b'data:,x\r\n--bb--\r\n')
    r = client.post("/deepdream", content=body, headers={"content-type": "multipart/form-data; boundary=bb"})
    assert r.status_code == 400 and "charset" in r.json()["detail"], r.text
    b, ct = encode_multipart({"file": "data:image/png;base64,AAAA", "octaves": "x"})
    r = client.post("/deepdream", content=b, headers={"content-type": ct})
    assert r.status_code == 400, r.text
    r = client.post("/", content=body, headers={"content-type": "multipart/form-data; boundary=bb"})
    assert r.status_code == 400, r.text


def test_decoded_pixel_cap(client, monkeypatch):
    """Images above the service's pixel cap are rejected as 400 before they are decoded."""
    import numpy as np

    client, _ = client
    from deconv_api_amd.codec import image as ci
    from deconv_api_amd.codec import make_data_url

    monkeypatch.setattr(ci, "MAX_PIXELS", 1000)
    url = make_data_url(np.zeros((40, 40, 3), np.uint8), "PNG")
    r = client.post("/", data={"file": url, "layer": "block1_conv1"})
    assert r.status_code == 400 and "too large" in r.json()["detail"], r.text


def test_deepdream_requests_are_batched():
    """Concurrent same-shape /deepdream requests run as ONE engine batch (padded to a power of two);
    a different shape runs in its own batch; batched outputs match single-image runs."""
    import asyncio

    from deconv_api_amd.codec import encode_data_url, read_data_url
    from deconv_api_amd.config import Config
    from deconv_api_amd.serve.dream_service import DreamService

    ds = DreamService(Config.from_env(device="cpu", dream_max_batch=4, dream_window_ms=300.0, hip_graphs=False))
    rng = np.random.default_rng(0)
    from urllib.parse import unquote

    shapes = [(80, 80, 3)] * 3 + [(96, 88, 3)]
    urls = [unquote(encode_data_url(rng.integers(0, 256, s, dtype=np.uint8), 95)) for s in shapes]

    async def go():
        return await asyncio.gather(*[ds.dream(u, "inception_v3", 1, 1) for u in urls])

    try:
        outs = asyncio.run(go())
        assert sorted(ds.batches) == [1, 3]
        for u, o in zip(urls, outs):
            assert o.startswith("data:image/")  # the reference labels JPEG bytes as webp
        # exactness of batching: the engine output of an image inside a batch == alone
        imgs = [ds.prepare(read_data_url(u), 1) for u in urls[:3]]
        both = ds.run_batch(imgs, "inception_v3", 1, 1)
        alone = ds.run_batch(imgs[1:2], "inception_v3", 1, 1)
        assert both.shape == (3, 80, 80, 3)
        d = np.abs(both[1].astype(int) - alone[0].astype(int))
        assert d.max() <= 2 and d.mean() < 0.05
        with pytest.raises(ValueError):
            ds.prepare(np.zeros((40, 40, 3), np.uint8), 4)
    finally:
        ds.close()


def test_asyncio_debug_mode_enables_loop_debug():
    """DV_ASYNCIO_DEBUG: the app's startup hook puts the event loop in debug mode (slow-callback
    logging at cfg.slow_callback_ms)."""
    from fastapi.testclient import TestClient

    from deconv_api_amd.api.app import create_app
    from deconv_api_amd.config import Config

    cfg = Config(asyncio_debug=True, slow_callback_ms=20.0, log_json=False)
    app = create_app(service=object(), cfg=cfg)
    with TestClient(app) as c:
        assert c.get("/health-check").json() == {"healthy": "true"}
        assert getattr(app.state, "loop_debug", False) is True


def test_scale_sweep_efficiency_and_parsing():
    """tools/scale_sweep.py: JSON-line parsing of bench output and weak-scaling efficiency."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location(
        "scale_sweep", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "scale_sweep.py"))
    sw = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sw)
    out = 'noise\n{"metric": "m", "value": 100.0, "unit": "images/s"}\n'
    assert sw.parse_json_line(out)["value"] == 100.0
    rows = sw.efficiency([{"n": 1, "value": 100.0}, {"n": 2, "value": 190.0}, {"n": 4, "value": None}])
    assert rows[0]["efficiency"] == 1.0 and rows[1]["efficiency"] == 0.95 and rows[2]["efficiency"] is None
    assert sw.bench_cmd(2, type("A", (), dict(steps=3, warmup=1, device="cpu", tiny=True, batch=0))())[1:3] == \
        ["-m", "torch.distributed.run"]


def test_native_data_url_b64decode_matches_python():
    """csrc/jpeg_enc.cpp:data_url_b64decode == base64.b64decode(uri.split(',')[1]) (non-strict:
    junk skipped, a completed pad ends the input) with the same error messages, on fuzzed payloads."""
    import base64 as b64
    import binascii

    lib = _native_or_skip()
    rng = np.random.default_rng(0)
    alpha = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"
    pool = alpha * 3 + "==== \n\t!-_.:;"
    cases = ["YQ==", "YQ==YQ==", "YQ=", "YQ", "Y", "YW Jj!", "YW=Jj", "=YWJj", "YQ=a=", "YWJjZA===",
             "YWJjZA", "YQ===", "Y===", "YWI=YQ", "YW=JjZA=", "YW=JjZA==", ""]
    cases += ["".join(rng.choice(list(pool), int(rng.integers(0, 40)))) for _ in range(3000)]
    cases += [b64.b64encode(rng.bytes(int(n))).decode() for n in rng.integers(0, 5000, 50)]
    for payload in cases:
        for uri in ("data:image/png;base64," + payload, "x," + payload + ",tail,more"):
            try:
                want, werr = b64.b64decode(uri.split(",")[1]), None
            except (binascii.Error, ValueError) as e:
                want, werr = None, str(e)
            try:
                got, gerr = lib.data_url_b64decode(uri), None
            except ValueError as e:
                got, gerr = None, str(e)
            assert (got, gerr) == (want, werr), (uri, got, gerr, want, werr)
    from deconv_api_amd.codec.image import ImageDecodeError, read_data_url

    for bad in ("no comma here", "data:x;base64,YQ=", "data:x;base64,Y"):
        with pytest.raises(ImageDecodeError):
            read_data_url(bad)
