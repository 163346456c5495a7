"""Multi-process serving: HTTP front ends (serve/frontend.py) feeding their rank's GPU owner over the
ingest socket (serve/ingest.py), launched by serve/launch.py; CPU engine here (the same processes run
the HIP engine on a GPU box). Reference surface: app/main.py:19-78."""
from __future__ import annotations

import base64
import io
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.error
import urllib.request
from urllib.parse import quote_plus

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _png_url(h=40, w=56, seed=0) -> str:
    from PIL import Image

    rng = np.random.default_rng(seed)
    buf = io.BytesIO()
    Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(buf, format="PNG")
    return "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()


def _post(base, fields, multipart=False, timeout=120):
    """Fresh connection per call (urllib): SO_REUSEPORT hashes each one to some front end."""
    if multipart:
        from deconv_api_amd.api.forms import encode_multipart

        body, ct = encode_multipart(fields)
    else:
        body = "&".join(f"{k}={quote_plus(v)}" for k, v in fields.items()).encode()
        ct = "application/x-www-form-urlencoded"
    req = urllib.request.Request(base + "/", data=body, headers={"Content-Type": ct})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def _get(base, path, timeout=30):
    with urllib.request.urlopen(base + path, timeout=timeout) as r:
        return r.status, r.read()


def _wait_ready(base, proc, timeout=240):
    t0 = time.time()
    while time.time() - t0 < timeout:
        assert proc.poll() is None, f"server exited with {proc.returncode}"
        try:
            if _get(base, "/ready", 5)[0] == 200:
                return
        except OSError:
            pass
        time.sleep(0.3)
    raise TimeoutError("server not ready")


def _start(cmd, port, frontends, extra_env=None):
    env = dict(os.environ, DV_DEVICE="cpu", DV_PORT=str(port), DV_HOST="127.0.0.1", DV_FRONTENDS=str(frontends),
               DV_HIP_GRAPHS="0", DV_CODEC_WORKERS="2", DV_LOG_JSON="1", OMP_NUM_THREADS="1",
               DV_INGEST_DIR="/tmp", PYTHONPATH=ROOT)
    env.update(extra_env or {})
    return subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            start_new_session=True)


def _stop(p):
    if p.poll() is None:
        os.killpg(p.pid, signal.SIGTERM)
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()


@pytest.mark.timeout(300)
def test_frontends_serve_reference_surface():
    """Two front ends + one CPU owner: the reference's routes behave as in single-process mode."""
    port = _free_port()
    base = f"http://127.0.0.1:{port}"
    p = _start([sys.executable, "-m", "deconv_api_amd.serve.launch"], port, 2)
    try:
        _wait_ready(base, p)
        assert json.loads(_get(base, "/health-check")[1]) == {"healthy": "true"}
        layers = json.loads(_get(base, "/layers")[1])["layers"]
        assert layers[0] == "block1_conv1" and "block5_conv3" in layers
        url = _png_url()
        outs = []
        for mp in (False, True):
            st, out = _post(base, {"file": url, "layer": "block1_conv1"}, multipart=mp)
            assert st == 200 and out.startswith("data:image/webp;base64,")
            outs.append(out)
        assert outs[0] == outs[1]  # same image, same layer: same bytes through either body encoding
        from deconv_api_amd.codec.image import parse_result_data_url

        assert parse_result_data_url(outs[0]).shape == (448, 448, 3)
        st, out = _post(base, {"file": url, "layer": "nope"})
        assert st == 400 and "unknown layer" in out["detail"]
        st, out = _post(base, {"file": "data:image/png;base64,AAAA", "layer": "block1_conv1"})
        assert st == 400
        st, out = _post(base, {"layer": "block1_conv1"})
        assert st == 422
        st, out = _post(base, {"file": url, "layer": "input_1"})  # the owner's check, relayed
        assert st == 400 and "no filters" in out["detail"]
        st, body = _get(base, "/ready")
        rd = json.loads(body)
        assert rd["ready"] and rd["ingest"]["connections"] == 2 and rd["frontend"]["pid"] != rd["ingest"]["pid"]
        m = _get(base, "/metrics")[1].decode()
        assert "dv_requests_total" in m and "dv_batch_size_count" in m and 'stage="decode"' in m
        assert m.count("# TYPE dv_uptime_seconds") == 1
    finally:
        _stop(p)
    assert p.returncode is not None


@pytest.mark.timeout(300)
def test_frontends_relay_deepdream():
    """POST /deepdream through a front end runs on the owner's DreamService (CPU InceptionV3 here);
    its 400 for an image too small for the octaves comes back unchanged."""
    port = _free_port()
    base = f"http://127.0.0.1:{port}"
    p = _start([sys.executable, "-m", "deconv_api_amd.serve.launch"], port, 1)
    try:
        _wait_ready(base, p)

        def dream(fields):
            body = "&".join(f"{k}={quote_plus(v)}" for k, v in fields.items()).encode()
            req = urllib.request.Request(base + "/deepdream", data=body,
                                         headers={"Content-Type": "application/x-www-form-urlencoded"})
            try:
                with urllib.request.urlopen(req, timeout=240) as r:
                    return r.status, json.loads(r.read())
            except urllib.error.HTTPError as e:
                return e.code, json.loads(e.read())

        st, out = dream({"file": _png_url(80, 80, seed=9), "octaves": "1", "steps": "1"})
        assert st == 200 and out.startswith("data:image/"), (st, out if st != 200 else "")
        from deconv_api_amd.codec.image import parse_result_data_url

        assert parse_result_data_url(out).shape == (80, 80, 3)
        st, out = dream({"file": _png_url(40, 40, seed=9), "octaves": "4", "steps": "1"})
        assert st == 400 and out["detail"], (st, out)
    finally:
        _stop(p)


@pytest.mark.timeout(300)
def test_frontend_restarted_after_it_dies():
    """The rank's supervisor (serve/supervisor.py) starts a front end again when one is killed; the
    service keeps answering through the survivor meanwhile and through both afterwards."""
    port = _free_port()
    base = f"http://127.0.0.1:{port}"
    p = _start([sys.executable, "-m", "deconv_api_amd.serve.launch"], port, 2)
    try:
        _wait_ready(base, p)
        url = _png_url(seed=5)
        assert _post(base, {"file": url, "layer": "block1_conv1"})[0] == 200
        pids = set()
        for _ in range(200):  # fresh connections reach both front ends sooner or later
            pids.add(json.loads(_get(base, "/ready")[1])["frontend"]["pid"])
            if len(pids) == 2:
                break
        assert len(pids) == 2, pids
        victim = sorted(pids)[0]
        os.kill(victim, signal.SIGKILL)  # our own child process, by its exact pid
        t0 = time.time()
        conns, seen = 0, set()
        while time.time() - t0 < 120:
            try:
                rd = json.loads(_get(base, "/ready")[1])
            except OSError:
                continue  # a connection the kernel had queued on the dead listener
            conns = rd["ingest"]["connections"]
            seen.add(rd["frontend"]["pid"])
            if conns >= 3 and len(seen - {victim}) == 2:
                break
            time.sleep(0.2)
        assert conns >= 3 and victim not in seen and len(seen) == 2, (conns, seen, victim)
        for i in range(6):
            st, out = _post(base, {"file": url, "layer": "block1_conv1"}, multipart=bool(i % 2))
            assert st == 200 and out.startswith("data:image/webp;base64,")
    finally:
        _stop(p)


@pytest.mark.timeout(420)
def test_frontends_per_rank_ingest_world3():
    """torchrun world 3 (Gloo, CPU): every rank runs its own front end on the shared port
    (SO_REUSEPORT) and decodes / computes only what its own front end accepted. Requests are spread
    over the ranks by the kernel; each rank's owner counts exactly the requests its front end
    shipped (no rank-0 decode, resize or scatter on the POST path)."""
    port = _free_port()
    mport = _free_port()
    base = f"http://127.0.0.1:{port}"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={mport}", "-m", "deconv_api_amd.serve.launch"]
    p = _start(cmd, port, 1)
    try:
        _wait_ready(base, p, 300)
        url = _png_url(seed=3)
        n = 36
        for i in range(n):
            st, out = _post(base, {"file": url, "layer": "block1_conv1"}, multipart=bool(i % 2))
            assert st == 200 and out.startswith("data:image/webp;base64,")
        seen = {}
        for _ in range(200):  # fresh connections land on every rank's front end sooner or later
            rd = json.loads(_get(base, "/ready")[1])
            seen[rd["ingest"]["rank"]] = (rd["ingest"]["requests"], rd["frontend"]["pid"], rd["ingest"]["pid"])
            if len(seen) == 3:
                break
        assert sorted(seen) == [0, 1, 2], seen
        assert sum(v[0] for v in seen.values()) == n  # every request was decoded and run by exactly one rank
        assert all(v[0] > 0 for v in seen.values()), seen  # ... and every rank took a share
        assert len({v[2] for v in seen.values()}) == 3 and len({v[1] for v in seen.values()}) == 3
    finally:
        _stop(p)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_frontends_on_gpu_match_the_engine(native_lib):
    """Two front ends + the GPU owner (HIP engine, GPU JPEG): a response equals the engine's own mosaic
    for the same image (up to the q95 JPEG round trip), through urlencoded and multipart bodies."""
    import torch

    from deconv_api_amd import ops
    from deconv_api_amd.codec.image import decode_image, encode_jpeg, parse_result_data_url
    from deconv_api_amd.engine.deconvnet import DeconvNet
    from deconv_api_amd.models.vgg16 import VGG16

    port = _free_port()
    base = f"http://127.0.0.1:{port}"
    p = _start([sys.executable, "-m", "deconv_api_amd.serve.launch"], port, 2,
               extra_env={"DV_DEVICE": "cuda", "DV_HIP_GRAPHS": "1"})
    try:
        _wait_ready(base, p, 240)
        rd = json.loads(_get(base, "/ready")[1])
        assert rd["device"].startswith("cuda") and rd["native"] is True, rd
        rng = np.random.default_rng(7)
        img = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
        from deconv_api_amd.codec import make_data_url

        url = make_data_url(img, "PNG")
        outs = [_post(base, {"file": url, "layer": "block4_pool"}, multipart=mp) for mp in (False, True)]
        assert all(st == 200 for st, _ in outs), outs[0][1] if outs[0][0] != 200 else outs[1][1]
        assert outs[0][1] == outs[1][1]
        got = parse_result_data_url(outs[0][1])
    finally:
        _stop(p)
    eng = DeconvNet(VGG16.random(0).build("cuda", torch.bfloat16))  # the launcher's weights (seed 0)
    x = torch.empty(1, 224, 224, 8, dtype=torch.bfloat16, device="cuda")
    ops.resize_preprocess(torch.from_numpy(img).cuda()[None], x)
    want = eng.run(x, "block4_pool").mosaic[0].cpu().numpy()
    ref = decode_image(encode_jpeg(want, 95))
    mse = float(((got.astype(np.float64) - ref.astype(np.float64)) ** 2).mean())
    assert mse == 0 or 10 * np.log10(255.0 ** 2 / mse) >= 35.0, mse


def test_supervisor_restart_budget(monkeypatch):
    """supervise(): a dead front end is restarted at most RESTARTS_PER_MIN times a minute, never while the
    owner's socket is absent, and the pass reports 'all down for good' only when nothing is alive."""
    from deconv_api_amd.config import Config
    from deconv_api_amd.serve import supervisor as S

    class P:
        def __init__(self, code=None):
            self.returncode = code

        def poll(self):
            return self.returncode

    spawned = []

    def fake_spawn(cfg, path, i):
        spawned.append(i)
        return P(code=1)  # dies again at once

    monkeypatch.setattr(S, "spawn_frontend", fake_spawn)
    cfg = Config(log_json=False)
    fes, hist = [P(), P(code=9)], {}
    assert S.supervise(cfg, "/x", fes, hist, 0.0, can_restart=False) is True  # #0 alive, #1 not restarted
    assert spawned == []
    t = 1.0
    for _ in range(S.RESTARTS_PER_MIN + 3):
        assert S.supervise(cfg, "/x", fes, hist, t, can_restart=True) is True
        t += 1.0
    assert spawned == [1] * S.RESTARTS_PER_MIN  # budget spent within the minute
    fes[0] = P(code=0)  # the survivor goes too
    assert S.supervise(cfg, "/x", fes, hist, t, can_restart=True) is True  # #0 gets its own budget
    assert spawned[-1] == 0
    assert S.supervise(cfg, "/x", fes, hist, t + 61.0, can_restart=True) is True  # a minute later: #1 again
    assert spawned[-1] in (0, 1)


def test_supervisor_reports_all_down(monkeypatch):
    from deconv_api_amd.config import Config
    from deconv_api_amd.serve import supervisor as S

    class P:
        returncode = 1

        def poll(self):
            return 1

    monkeypatch.setattr(S, "spawn_frontend", lambda cfg, path, i: P())
    cfg, fes, hist = Config(log_json=False), [P(), P()], {}
    results = [S.supervise(cfg, "/x", fes, hist, 10.0 + 0.1 * k, can_restart=True) for k in range(2 * S.RESTARTS_PER_MIN)]
    assert results[:S.RESTARTS_PER_MIN] == [True] * S.RESTARTS_PER_MIN and results[-1] is False
