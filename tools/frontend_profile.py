"""CPU profile of ONE HTTP front end (serve/frontend.py) under load, with a stub GPU owner that answers
every request at once with a realistic ~100 KB data URL: where a front end's per-request CPU goes
(h11 / uvicorn / starlette / form parsing / base64 + PIL decode / ingest IPC / response). No GPU needed.

    python tools/frontend_profile.py --seconds 8 --clients 32 [--png-every 0] [--top 35]
"""
from __future__ import annotations

import argparse
import json
import os
import pstats
import signal
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from deconv_api_amd.serve import ingest  # noqa: E402


class _Cfg:
    jpeg_quality = 95


class _Engine:
    names = ["input_1", "block1_conv1", "block5_conv3"]


class StubService:
    """DeconvService surface the IngestServer uses; answers with a fixed data URL."""

    cfg = _Cfg()
    engine = _Engine()

    def __init__(self, body: bytes):
        self.body = body

    def submit(self, layer, img, done):
        done(self.body, None)

    def status(self):
        return {"ready": True, "worker_alive": True, "device": "stub"}

    def layer_names(self):
        return ["block1_conv1", "block5_conv3"]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--png-every", type=int, default=4)
    ap.add_argument("--top", type=int, default=35)
    ap.add_argument("--out", default=None, help="write the pstats text here")
    a = ap.parse_args()

    import numpy as np

    from deconv_api_amd.codec import encode_data_url

    y, x = np.mgrid[0:448, 0:448].astype(np.float32)
    mosaic = np.stack([128 + 90 * np.sin(x / (9 + 4 * c) + y / (13 + 3 * c)) for c in range(3)], -1)
    mosaic += np.random.default_rng(0).normal(0, 12, mosaic.shape)
    mosaic = np.clip(mosaic, 0, 255).astype(np.uint8)
    body = encode_data_url(mosaic, 95).encode()  # textured mosaic: a response of the served size class
    d = tempfile.mkdtemp(prefix="dv-feprof-")
    sock_path = os.path.join(d, "owner.sock")
    srv = ingest.IngestServer(sock_path, StubService(body))
    port = _free_port()
    prof = os.path.join(d, "fe.prof")
    env = dict(os.environ, DV_LOG_JSON="1", PYTHONPATH=ROOT, DV_CODEC_WORKERS=os.environ.get("DV_CODEC_WORKERS", "4"))
    fe = subprocess.Popen([sys.executable, "-m", "cProfile", "-o", prof, "-m", "deconv_api_amd.serve.frontend",
                           "--sock", sock_path, "--host", "127.0.0.1", "--port", str(port)],
                          cwd=ROOT, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, start_new_session=True)
    base = f"http://127.0.0.1:{port}"
    import urllib.request

    t0 = time.time()
    while True:
        try:
            with urllib.request.urlopen(base + "/health-check", timeout=2) as r:
                if r.status == 200:
                    break
        except OSError:
            pass
        if fe.poll() is not None or time.time() - t0 > 60:
            raise SystemExit(f"front end did not start: {fe.stderr.read().decode()[-2000:]}")
        time.sleep(0.2)
    import psutil

    p = psutil.Process(fe.pid)
    cpu0 = p.cpu_times()
    load = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "http_load.py"), "--url", base,
                           "--clients", str(a.clients), "--procs", str(a.procs), "--seconds", str(a.seconds),
                           "--warmup", "1", "--png-every", str(a.png_every), "--layer", "block5_conv3"],
                          capture_output=True, text=True, timeout=600)
    cpu1 = p.cpu_times()
    os.killpg(fe.pid, signal.SIGINT)  # uvicorn shuts down; cProfile writes its file
    fe.wait(timeout=60)
    srv.close()
    res = json.loads(load.stdout.strip().splitlines()[-1])
    run = res["runs"][0]
    n = run["responses"]
    cpu = (cpu1.user + cpu1.system) - (cpu0.user + cpu0.system)
    head = {"responses": n, "req_per_s": run["req_per_s"], "fe_cpu_s": round(cpu, 2),
            "fe_cpu_ms_per_req": round(1e3 * cpu / max(n, 1), 3), "response_bytes": len(body)}
    print(json.dumps(head), flush=True)
    import io

    buf = io.StringIO()
    st = pstats.Stats(prof, stream=buf)
    st.sort_stats("tottime").print_stats(a.top)
    txt = buf.getvalue()
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(head) + "\n" + txt)


if __name__ == "__main__":
    main()
