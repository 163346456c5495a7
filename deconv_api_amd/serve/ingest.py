"""Front-end <-> GPU-owner transport for multi-process serving (``DV_FRONTENDS`` > 0).

One Python process cannot keep an MI355X busy through HTTP: h11 parsing, form parsing and the
JSON response hold its GIL for every request, and the reference's workload is exactly that, one
small HTTP request per image (app/main.py:45-78). So each rank runs:

  * ``frontends`` front-end processes (serve/frontend.py): uvicorn + the same FastAPI app, all
    bound to the serving port with SO_REUSEPORT (the kernel spreads connections over every
    front-end of every rank on the node). Each parses the form, base64- and PIL-decodes the image
    on its own threads (its own GIL), and ships the decoded uint8 pixels to its rank's GPU owner;
  * one GPU-owner process (serve/launch.py): the batching service (serve/service.py) on this
    rank's GPU behind an ``IngestServer`` on a Unix socket. A reader thread per front-end
    connection ``recv_into``s each image straight into a numpy array (GIL released during the
    copy) and enqueues it; the response (data URL, JPEG-encoded on the GPU and base64'd natively)
    is sent back by the encode thread that produced it.

Every rank decodes only the requests its own front-ends accepted: there is no rank-0 decode,
resize or scatter on the ``POST /`` path, so HTTP throughput scales with ranks.

Wire format (little endian), both directions over one SOCK_STREAM Unix socket per front-end:
  request   <I rid, B kind, B pad, H layer_len, I h, I w, Q nbytes, I decode_us> + layer utf-8 + payload
  response  <I rid, H status, Q nbytes> + payload
kinds: DECONV (payload = h*w*3 uint8 RGB pixels), STATUS / METRICS / LAYERS (no payload; JSON or
text back), DREAM (payload = JSON header line + the data URL). status: HTTP-like (200, 400, 503,
500); non-200 payloads are the error message. ``decode_us``: the front end's base64 + PIL decode time,
recorded by the owner, whose /metrics therefore cover every front end of the rank.
"""
from __future__ import annotations

import asyncio
import json
import os
import socket
import struct
import threading
import time
from typing import Callable, Dict, Optional

import numpy as np

from ..codec.image import MAX_PIXELS
from ..utils import metrics as M
from ..utils.logging import get_logger

log = get_logger("deconv_api_amd.ingest")

REQ = struct.Struct("<IBBHIIQI")
RESP = struct.Struct("<IHQ")
DECONV, STATUS, METRICS, LAYERS, DREAM = 1, 2, 3, 4, 5
SOCK_BUF = 8 << 20
MAX_DREAM_BODY = 256 << 20  # JSON header + data URL of one /deepdream request


def socket_path(port: int, rank: int) -> str:
    base = os.environ.get("DV_INGEST_DIR") or os.environ.get("TMPDIR") or "/tmp"
    return os.path.join(base, f"dv-ingest-{port}-r{rank}-{os.getpid()}.sock")


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray(n)
    _recv_into(sock, memoryview(buf))
    return bytes(buf)


def _recv_into(sock: socket.socket, mv: memoryview) -> None:
    got = 0
    n = len(mv)
    while got < n:
        k = sock.recv_into(mv[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed")
        got += k


def _tune(sock: socket.socket) -> None:
    for opt in (socket.SO_SNDBUF, socket.SO_RCVBUF):
        try:
            sock.setsockopt(socket.SOL_SOCKET, opt, SOCK_BUF)
        except OSError:
            pass


def _status_of(e: BaseException) -> int:
    from ..codec import ImageDecodeError
    from ..engine.deconvnet import UnknownLayerError
    from .service import ServiceOverloaded

    if isinstance(e, (ImageDecodeError, UnknownLayerError, ValueError)):
        return 400
    if isinstance(e, ServiceOverloaded):
        return 503
    return 500


class IngestServer:
    """GPU-owner side: accepts front-end connections on ``path`` and feeds the batching service.

    ``svc``: serve.service.DeconvService (``submit`` entry); ``dream``: serve.dream_service.
    DreamService or None (its coroutines run on one private event loop thread)."""

    def __init__(self, path: str, svc, dream=None, rank: int = 0):
        self.path = path
        self.svc = svc
        self.dream = dream
        self.rank = rank
        self.conns = 0
        self.requests = 0
        self._stop = threading.Event()
        self._threads = []
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        if os.path.exists(path):
            os.unlink(path)
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.bind(path)
        self.sock.listen(64)
        self._acceptor = threading.Thread(target=self._accept, name="dv-ingest-accept", daemon=True)
        self._acceptor.start()

    # ------------------------------------------------------------------ connections
    def _accept(self) -> None:
        while not self._stop.is_set():
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            _tune(c)
            self.conns += 1
            t = threading.Thread(target=self._serve, args=(c,), name=f"dv-ingest-{self.conns}", daemon=True)
            t.start()
            self._threads.append(t)

    def _serve(self, c: socket.socket) -> None:
        lock = threading.Lock()

        def reply(rid: int, status: int, payload: bytes) -> None:
            with lock:  # responses come from encode threads, the reader and the dream loop
                try:
                    c.sendall(RESP.pack(rid, status, len(payload)))
                    if payload:
                        c.sendall(payload)
                except OSError:
                    pass  # the front-end is gone; its requests die with its connections

        try:
            while not self._stop.is_set():
                rid, kind, _, llen, h, w, nbytes, dec_us = REQ.unpack(_recv_exact(c, REQ.size))
                layer = _recv_exact(c, llen).decode() if llen else ""
                if kind == DECONV:
                    if nbytes != h * w * 3 or h * w > MAX_PIXELS:
                        # the front ends enforce the same cap before decoding; a frame that breaks it is not
                        # worth draining (up to 2^64 bytes): answer and drop the connection
                        reply(rid, 400, b"pixel payload does not match its shape or exceeds DV_MAX_PIXELS")
                        return
                    img = np.empty((h, w, 3), np.uint8)
                    _recv_into(c, memoryview(img).cast("B"))
                    self.requests += 1
                    M.HOST_STAGE.observe(dec_us * 1e-6, stage="decode")
                    self._deconv(rid, layer, img, reply)
                elif kind == DREAM:
                    if nbytes > MAX_DREAM_BODY:
                        reply(rid, 413, b"dream request too large")
                        return
                    body = _recv_exact(c, nbytes)
                    self._dream(rid, body, reply)
                else:
                    if nbytes:  # info requests carry no payload
                        reply(rid, 400, b"unexpected payload")
                        return
                    reply(rid, *self._info(kind))
        except (ConnectionError, OSError, struct.error):
            pass
        finally:
            try:
                c.close()
            except OSError:
                pass

    # ------------------------------------------------------------------ request kinds
    def _deconv(self, rid: int, layer: str, img: np.ndarray, reply) -> None:
        def done(value, exc):
            if exc is None:
                if isinstance(value, np.ndarray):  # CPU / PIL path: raw mosaic, encode here
                    from ..codec import encode_data_url

                    value = encode_data_url(value, self.svc.cfg.jpeg_quality)
                reply(rid, 200, value.encode() if isinstance(value, str) else value)
            else:
                reply(rid, _status_of(exc), str(exc).strip('"').encode())

        try:
            self.svc.submit(layer, img, done)
        except Exception as e:  # noqa: BLE001 - unknown layer, queue full: answered at once
            done(None, e)

    def _dream(self, rid: int, body: bytes, reply) -> None:
        if self.dream is None:
            reply(rid, 404, b"/deepdream is not served by this process")
            return
        head, _, uri = body.partition(b"\n")
        try:
            p = json.loads(head)
        except ValueError:
            reply(rid, 400, b"bad dream header")
            return
        loop = self._dream_loop()
        fut = asyncio.run_coroutine_threadsafe(
            self.dream.dream(uri.decode("ascii", errors="replace"), p["model"], int(p["octaves"]), int(p["steps"])), loop)

        def done(f):
            e = f.exception()
            if e is None:
                reply(rid, 200, f.result().encode())
            else:
                reply(rid, _status_of(e), str(e).encode())

        fut.add_done_callback(done)

    def _dream_loop(self) -> asyncio.AbstractEventLoop:
        if self._loop is None:
            loop = asyncio.new_event_loop()
            threading.Thread(target=loop.run_forever, name="dv-ingest-dream", daemon=True).start()
            self._loop = loop
        return self._loop

    def _info(self, kind: int):
        try:
            if kind == STATUS:
                st = self.svc.status()
                st["ingest"] = {"rank": self.rank, "pid": os.getpid(), "connections": self.conns,
                                "requests": self.requests}
                if self.dream is not None:
                    st["deepdream"] = self.dream.status()
                return 200, json.dumps(st).encode()
            if kind == METRICS:
                return 200, M.REGISTRY.render().encode()
            if kind == LAYERS:
                return 200, json.dumps({"layers": self.svc.layer_names(), "names": list(self.svc.engine.names)}).encode()
        except Exception as e:  # noqa: BLE001
            return 500, repr(e).encode()
        return 400, b"unknown request kind"

    def close(self) -> None:
        self._stop.set()
        try:
            self.sock.close()
        finally:
            if os.path.exists(self.path):
                os.unlink(self.path)
        if self._loop is not None:
            self._loop.call_soon_threadsafe(self._loop.stop)


class IngestClient:
    """Front-end side: one connection to the rank's GPU owner, shared by the event loop and the
    decode threads. Requests are written by the thread that produced them (under a send lock);
    one reader thread completes them (``concurrent.futures``-style callbacks)."""

    def __init__(self, path: str, connect_timeout: float = 900.0, on_lost: Optional[Callable[[], None]] = None):
        t0 = time.time()
        while True:
            try:
                s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
                s.connect(path)
                break
            except OSError:
                s.close()
                if time.time() - t0 > connect_timeout:
                    raise
                time.sleep(0.2)
        _tune(s)
        self.sock = s
        self._send = threading.Lock()
        self._pend: Dict[int, Callable[[int, bytes], None]] = {}
        self._plock = threading.Lock()
        self._rid = 0
        self.on_lost = on_lost
        self._reader = threading.Thread(target=self._read, name="dv-ingest-reader", daemon=True)
        self._reader.start()

    def _next(self, cb) -> int:
        with self._plock:
            self._rid = (self._rid + 1) & 0xFFFFFFFF
            self._pend[self._rid] = cb
            return self._rid

    def send(self, kind: int, cb: Callable[[int, bytes], None], layer: str = "", h: int = 0, w: int = 0,
             payload=b"", decode_s: float = 0.0) -> None:
        """Queue one request; ``cb(status, payload)`` runs on the reader thread."""
        mv = memoryview(payload).cast("B") if not isinstance(payload, (bytes, bytearray)) else payload
        lb = layer.encode()
        rid = self._next(cb)
        head = REQ.pack(rid, kind, 0, len(lb), h, w, len(mv), min(int(decode_s * 1e6), 0xFFFFFFFF))
        with self._send:
            self.sock.sendall(head + lb)
            if len(mv):
                self.sock.sendall(mv)

    def call(self, kind: int, layer: str = "", payload=b"", timeout: float = 30.0):
        """Blocking request (status / metrics / layers) -> (status, payload)."""
        ev = threading.Event()
        box = {}

        def cb(st, data):
            box["r"] = (st, data)
            ev.set()

        self.send(kind, cb, layer, payload=payload)
        if not ev.wait(timeout):
            raise TimeoutError("GPU owner did not answer")
        return box["r"]

    def _read(self) -> None:
        try:
            while True:
                rid, st, n = RESP.unpack(_recv_exact(self.sock, RESP.size))
                data = _recv_exact(self.sock, n) if n else b""
                with self._plock:
                    cb = self._pend.pop(rid, None)
                if cb is not None:
                    cb(st, data)
        except (ConnectionError, OSError, struct.error):
            with self._plock:
                pend, self._pend = self._pend, {}
            for cb in pend.values():
                cb(500, b"GPU owner connection lost")
            if self.on_lost is not None:
                self.on_lost()

    def close(self) -> None:
        self.on_lost = None  # a deliberate close is not a lost owner
        try:
            self.sock.shutdown(socket.SHUT_RDWR)
            self.sock.close()
        except OSError:
            pass
