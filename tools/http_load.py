"""HTTP load generator for the reference's only workload, ``POST /`` (app/main.py:45-78).

Drives a running server (or one it starts itself with ``--spawn``) through real sockets: P client
processes x C keep-alive connections each, every connection sending complete HTTP/1.1 requests whose
``file`` field is a data-URL JPEG or PNG of mixed sizes (224x224 .. 1024x768), half of them
urlencoded (percent-encoded like a browser form) and half multipart/form-data. Per client count it
reports requests/s, p50/p90/p99 latency, error counts and the server's per-stage breakdown from the
deltas of its ``/metrics`` histograms (decode, queue, GPU stages, encode).

    python tools/http_load.py --spawn --frontends 4 --clients 64,256 --seconds 10
    python tools/http_load.py --url http://127.0.0.1:8080 --clients 64

The clients are non-blocking sockets under one ``selectors`` loop per process (no HTTP library on
the client's hot path), request bytes prebuilt, so a client process sustains several thousand
responses/s of ~80 KB each. Prints one JSON object (and writes it to ``--out``).
"""
from __future__ import annotations

import argparse
import base64
import io
import json
import multiprocessing as mp
import os
import selectors
import signal
import socket
import subprocess
import sys
import time
import urllib.request
from urllib.parse import quote_plus

import numpy as np

SIZES = [(224, 224), (320, 240), (500, 375), (640, 480), (375, 500), (1024, 768)]
WEIGHTS = [0.2, 0.2, 0.25, 0.2, 0.1, 0.05]


def _image(rng, w, h):
    """A photo-like image: smooth gradients + a few shapes + mild noise (compresses like a photo,
    not like white noise)."""
    y, x = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.stack([128 + 100 * np.sin(x / (17 + 7 * c) + y / (23 + 5 * c) + rng.uniform(0, 6)) for c in range(3)], -1)
    for _ in range(6):
        cx, cy, r = rng.uniform(0, w), rng.uniform(0, h), rng.uniform(10, max(w, h) / 4)
        m = (x - cx) ** 2 + (y - cy) ** 2 < r * r
        img[m] = rng.uniform(0, 255, 3)
    img += rng.normal(0, 6, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def corpus(n: int, seed: int = 0, png_every: int = 4):
    """n (data URL, kind) pairs: mixed sizes, JPEG (q90) and every ``png_every``-th one PNG."""
    from PIL import Image

    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        w, h = SIZES[rng.choice(len(SIZES), p=WEIGHTS)]
        fmt = "PNG" if png_every and i % png_every == png_every - 1 else "JPEG"
        buf = io.BytesIO()
        kw = {"quality": 90} if fmt == "JPEG" else {"compress_level": 1}
        Image.fromarray(_image(rng, w, h)).save(buf, format=fmt, **kw)
        out.append((f"data:image/{fmt.lower()};base64," + base64.b64encode(buf.getvalue()).decode(), f"{fmt}{w}x{h}"))
    return out


def build_requests(urls, layer: str, host: str):
    """Prebuilt HTTP/1.1 request bytes: even indices urlencoded, odd multipart."""
    reqs = []
    for i, (u, _) in enumerate(urls):
        if i % 2 == 0:
            body = f"file={quote_plus(u)}&layer={quote_plus(layer)}".encode()
            ct = "application/x-www-form-urlencoded"
        else:
            b = "dvload7MA4YWxkTrZu0gW"
            body = (f"--{b}\r\nContent-Disposition: form-data; name=\"file\"\r\n\r\n{u}\r\n"
                    f"--{b}\r\nContent-Disposition: form-data; name=\"layer\"\r\n\r\n{layer}\r\n--{b}--\r\n").encode()
            ct = f"multipart/form-data; boundary={b}"
        head = (f"POST / HTTP/1.1\r\nHost: {host}\r\nContent-Type: {ct}\r\n"
                f"Content-Length: {len(body)}\r\nConnection: keep-alive\r\n\r\n").encode()
        reqs.append(head + body)
    return reqs


class _Conn:
    __slots__ = ("sock", "out", "buf", "t0", "need", "hdr_end", "status", "ok")

    def __init__(self, sock):
        self.sock = sock
        self.out = memoryview(b"")
        self.buf = bytearray()
        self.t0 = 0.0
        self.need = -1
        self.hdr_end = -1
        self.status = 0


def _client(addr, conns, reqs, t_warm, t_end, seed, q):
    """One client process: ``conns`` keep-alive connections, each sending the next request as soon
    as its previous response is complete. Latencies (ms) of responses that finished inside
    [t_warm, t_end] go back through ``q`` with error counts."""
    sel = selectors.DefaultSelector()
    rng = np.random.default_rng(seed)
    lat, errs, bad, n_out = [], 0, 0, 0
    cs = []

    def connect():
        s = socket.create_connection(addr)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 20)
        s.setblocking(False)
        c = _Conn(s)
        return c

    def send_next(c):
        c.out = memoryview(reqs[int(rng.integers(len(reqs)))])
        c.buf = bytearray()
        c.need, c.hdr_end, c.status = -1, -1, 0
        c.t0 = time.perf_counter()
        sel.register(c.sock, selectors.EVENT_WRITE | selectors.EVENT_READ, c)

    for _ in range(conns):
        c = connect()
        cs.append(c)
        send_next(c)
    cpu0 = None
    while True:
        now = time.perf_counter()
        if cpu0 is None and now >= t_warm:
            cpu0 = time.process_time()
        if now > t_end:
            break
        for key, ev in sel.select(timeout=0.05):
            c = key.data
            if ev & selectors.EVENT_WRITE and len(c.out):
                try:
                    k = c.sock.send(c.out)
                except BlockingIOError:
                    k = 0
                c.out = c.out[k:]
                if not len(c.out):
                    sel.modify(c.sock, selectors.EVENT_READ, c)
            if ev & selectors.EVENT_READ:
                try:
                    chunk = c.sock.recv(1 << 20)
                except BlockingIOError:
                    continue
                except ConnectionError:
                    chunk = b""
                if not chunk:  # server closed: count and reconnect
                    errs += 1
                    sel.unregister(c.sock)
                    c.sock.close()
                    nc = connect()
                    cs[cs.index(c)] = nc
                    send_next(nc)
                    continue
                c.buf += chunk
                if c.hdr_end < 0:
                    e = c.buf.find(b"\r\n\r\n")
                    if e < 0:
                        continue
                    c.hdr_end = e + 4
                    head = bytes(c.buf[:e]).decode("latin-1").split("\r\n")
                    c.status = int(head[0].split()[1])
                    c.need = 0
                    for h in head[1:]:
                        k_, _, v = h.partition(":")
                        if k_.strip().lower() == "content-length":
                            c.need = int(v)
                if len(c.buf) - c.hdr_end < c.need:
                    continue
                t1 = time.perf_counter()
                body = bytes(c.buf[c.hdr_end:c.hdr_end + 32])
                n_out += 1
                if c.status != 200:
                    errs += 1
                elif not body.startswith(b'"data:image/webp;base64,'):
                    bad += 1
                elif t_warm <= t1 <= t_end:
                    lat.append((t1 - c.t0) * 1e3)
                sel.unregister(c.sock)
                send_next(c)
    for c in cs:
        try:
            c.sock.close()
        except OSError:
            pass
    q.put((lat, errs, bad, n_out, time.process_time() - (cpu0 or 0.0)))


def scrape(base: str) -> dict:
    """/metrics -> {series: value} for the histogram sums/counts the breakdown needs."""
    try:
        txt = urllib.request.urlopen(base + "/metrics", timeout=10).read().decode()
    except OSError:
        return {}
    out = {}
    for line in txt.splitlines():
        if line.startswith("#") or " " not in line:
            continue
        k, v = line.rsplit(" ", 1)
        if "_sum" in k or "_count" in k:
            try:
                out[k] = float(v)
            except ValueError:
                pass
    return out


def breakdown(m0: dict, m1: dict) -> dict:
    """Mean seconds per observation -> ms, per histogram series, over the run (metric deltas)."""
    out = {}
    for k, v in m1.items():
        if "_seconds_sum" not in k:
            continue
        ck = k.replace("_sum", "_count")
        dn = m1.get(ck, 0) - m0.get(ck, 0)
        if dn > 0:
            name = k.replace("dv_", "").replace("_seconds_sum", "")
            out[name] = {"mean_ms": round(1e3 * (v - m0.get(k, 0)) / dn, 3), "n": int(dn)}
    return out


def _tree_cpu(pid):
    """{"frontend"|"owner"|"other": CPU seconds} of a process tree (psutil), by command line."""
    import psutil

    out = {}
    try:
        root = psutil.Process(pid)
        procs = [root] + root.children(recursive=True)
    except psutil.Error:
        return out
    for p in procs:
        try:
            t = p.cpu_times()
            cmd = " ".join(p.cmdline())
        except psutil.Error:
            continue
        kind = "frontend" if "serve.frontend" in cmd else ("owner" if "serve.launch" in cmd else "other")
        out[kind] = out.get(kind, 0.0) + t.user + t.system
    return out


def run_load(base, reqs, clients, procs, seconds, warmup, server_pid=None):
    host, port = base.split("://")[1].split(":")
    addr = (host, int(port))
    procs = max(1, min(procs, clients))
    per = [clients // procs + (1 if i < clients % procs else 0) for i in range(procs)]
    t_start = time.perf_counter() + 0.5
    t_warm = t_start + warmup
    t_end = t_warm + seconds
    q = mp.get_context("fork").Queue()
    m0 = None
    ps = [mp.get_context("fork").Process(target=_client, args=(addr, per[i], reqs, t_warm, t_end, 1000 + i, q))
          for i in range(procs)]
    for p in ps:
        p.start()
    time.sleep(max(0.0, t_warm - time.perf_counter()))
    c0 = _tree_cpu(server_pid) if server_pid else {}
    m0 = scrape(base)
    time.sleep(max(0.0, t_end - time.perf_counter()))
    c1 = _tree_cpu(server_pid) if server_pid else {}
    res = [q.get(timeout=seconds + warmup + 120) for _ in ps]
    m1 = scrape(base)
    for p in ps:
        p.join(timeout=30)
    lat = sorted(x for r in res for x in r[0])
    n = len(lat)

    def pct(f):
        return round(lat[min(n - 1, int(f * n))], 2) if n else None

    out = {"clients": clients, "client_procs": procs, "seconds": seconds, "responses": n,
           "req_per_s": round(n / seconds, 1), "p50_ms": pct(0.5), "p90_ms": pct(0.9), "p99_ms": pct(0.99),
           "errors": sum(r[1] for r in res), "bad_bodies": sum(r[2] for r in res),
           "client_cpu_s": round(sum(r[4] for r in res), 2), "server_stages": breakdown(m0, m1)}
    if c1:  # CPU-seconds the server spent in the window, per process kind, and per response
        out["server_cpu_s"] = {k: round(c1.get(k, 0.0) - c0.get(k, 0.0), 2) for k in c1}
        tot = sum(out["server_cpu_s"].values())
        out["server_cpu_ms_per_req"] = round(1e3 * tot / max(n, 1), 3)
        out["cpus_busy"] = round((tot + out["client_cpu_s"]) / seconds, 2)
    return out


def wait_ready(base: str, timeout: float, proc=None) -> None:
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc is not None and proc.poll() is not None:
            raise RuntimeError(f"server exited with {proc.returncode}")
        try:
            r = urllib.request.urlopen(base + "/ready", timeout=5)
            if r.status == 200:
                return
        except OSError:
            pass
        time.sleep(0.5)
    raise TimeoutError("server not ready")


def warm_layer(base: str, url: str, layer: str, n: int = 4) -> None:
    """A few sequential requests so graph capture for small batch buckets is out of the window."""
    body = f"file={quote_plus(url)}&layer={quote_plus(layer)}".encode()
    for _ in range(n):
        req = urllib.request.Request(base + "/", data=body,
                                     headers={"Content-Type": "application/x-www-form-urlencoded"})
        urllib.request.urlopen(req, timeout=300).read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="http://127.0.0.1:8080")
    ap.add_argument("--layer", default="block5_conv3")
    ap.add_argument("--clients", default="64,256")
    ap.add_argument("--procs", type=int, default=4, help="client processes")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--warmup", type=float, default=3.0)
    ap.add_argument("--corpus", type=int, default=64)
    ap.add_argument("--png-every", type=int, default=4, help="every n-th corpus image is a PNG (0: JPEG only)")
    ap.add_argument("--spawn", action="store_true", help="start `python -m deconv_api_amd.serve.launch` as a child")
    ap.add_argument("--frontends", type=int, default=None, help="DV_FRONTENDS for the spawned server")
    ap.add_argument("--env", action="append", default=[], help="extra KEY=VALUE for the spawned server")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    urls = corpus(a.corpus, png_every=a.png_every)
    host = a.url.split("://")[1]
    reqs = build_requests(urls, a.layer, host)
    srv = None
    if a.spawn:
        env = dict(os.environ, DV_PORT=host.split(":")[1], DV_HOST=host.split(":")[0], DV_LOG_JSON="1")
        if a.frontends is not None:
            env["DV_FRONTENDS"] = str(a.frontends)
        for kv in a.env:
            k, _, v = kv.partition("=")
            env[k] = v
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        log = open(os.environ.get("DV_LOAD_SERVER_LOG", "/tmp/dv_http_server.log"), "w")
        srv = subprocess.Popen([sys.executable, "-m", "deconv_api_amd.serve.launch"], cwd=root, env=env,
                               stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    res = {"layer": a.layer, "url": a.url, "corpus": {}, "runs": []}
    for _, kind in urls:
        res["corpus"][kind] = res["corpus"].get(kind, 0) + 1
    res["mean_request_kb"] = round(sum(len(r) for r in reqs) / len(reqs) / 1024, 1)
    try:
        wait_ready(a.url, 600, srv)
        warm_layer(a.url, urls[0][0], a.layer)
        try:
            res["server"] = json.loads(urllib.request.urlopen(a.url + "/ready", timeout=10).read())
        except OSError:
            pass
        for c in [int(x) for x in a.clients.split(",")]:
            r = run_load(a.url, reqs, c, a.procs, a.seconds, a.warmup, srv.pid if srv is not None else None)
            print(json.dumps(r), flush=True)
            res["runs"].append(r)
    finally:
        if srv is not None:
            os.killpg(srv.pid, signal.SIGTERM)
            try:
                srv.wait(timeout=30)
            except subprocess.TimeoutExpired:
                os.killpg(srv.pid, signal.SIGKILL)
    print(json.dumps(res))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
