"""Front-end <-> GPU-owner wire protocol (serve/ingest.py) against a stand-in batching service:
request kinds, status mapping, and the owner's guards on malformed frames (CPU only)."""
from __future__ import annotations

import json
import os
import socket
import tempfile
import threading

import numpy as np
import pytest

from deconv_api_amd.serve import ingest as I


class _Cfg:
    jpeg_quality = 95


class _Engine:
    names = ["input_1", "block1_conv1"]


class _Svc:
    """submit() answers on another thread, as the encode pool does."""

    cfg = _Cfg()
    engine = _Engine()

    def __init__(self):
        self.seen = []

    def submit(self, layer, img, done):
        if layer != "block1_conv1":
            from deconv_api_amd.engine.deconvnet import UnknownLayerError

            raise UnknownLayerError(f"unknown layer {layer!r}")
        self.seen.append((layer, img.shape, int(img.sum())))
        threading.Thread(target=done, args=(f"data:image/jpeg;base64,{img.shape[0]}x{img.shape[1]}", None)).start()

    def status(self):
        return {"ready": True}

    def layer_names(self):
        return ["block1_conv1"]


@pytest.fixture()
def server():
    d = tempfile.mkdtemp(prefix="dv-ingest-test-")
    path = os.path.join(d, "s.sock")
    svc = _Svc()
    srv = I.IngestServer(path, svc, rank=3)
    yield path, svc, srv
    srv.close()
    os.rmdir(d)


def _call(cli, kind, **kw):
    ev, box = threading.Event(), {}

    def cb(st, data):
        box["r"] = (st, data)
        ev.set()

    cli.send(kind, cb, **kw)
    assert ev.wait(10)
    return box["r"]


def test_ingest_request_kinds(server):
    path, svc, _ = server
    cli = I.IngestClient(path, connect_timeout=10)
    try:
        img = np.arange(5 * 7 * 3, dtype=np.uint8).reshape(5, 7, 3)
        st, body = _call(cli, I.DECONV, layer="block1_conv1", h=5, w=7, payload=img, decode_s=0.002)
        assert st == 200 and body == b"data:image/jpeg;base64,5x7"
        assert svc.seen == [("block1_conv1", (5, 7, 3), int(img.sum()))]  # pixels arrive intact
        st, body = _call(cli, I.DECONV, layer="nope", h=1, w=1, payload=np.zeros((1, 1, 3), np.uint8))
        assert st == 400 and b"unknown layer" in body
        st, body = cli.call(I.STATUS)
        rd = json.loads(body)
        assert st == 200 and rd["ready"] and rd["ingest"]["rank"] == 3 and rd["ingest"]["requests"] == 2
        st, body = cli.call(I.LAYERS)
        assert st == 200 and json.loads(body) == {"layers": ["block1_conv1"], "names": ["input_1", "block1_conv1"]}
        st, body = cli.call(I.METRICS)
        assert st == 200 and b'stage="decode"' in body
        st, body = cli.call(I.DREAM, payload=b'{"model": "x"}\n')
        assert st == 404  # no DreamService in this owner
    finally:
        cli.close()


@pytest.mark.parametrize("frame", ["shape", "pixels", "info_payload"])
def test_ingest_rejects_malformed_frames(server, frame):
    """A frame that lies about its size is answered and its connection dropped (never drained)."""
    path, svc, _ = server
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.connect(path)
    try:
        if frame == "shape":  # nbytes != h * w * 3
            s.sendall(I.REQ.pack(7, I.DECONV, 0, 0, 4, 4, 10, 0))
        elif frame == "pixels":  # over the decoded-pixel cap
            side = int(I.MAX_PIXELS ** 0.5) + 1
            s.sendall(I.REQ.pack(7, I.DECONV, 0, 0, side, side, side * side * 3, 0))
        else:
            s.sendall(I.REQ.pack(7, I.STATUS, 0, 0, 0, 0, 5, 0) + b"extra")
        rid, st, n = I.RESP.unpack(I._recv_exact(s, I.RESP.size))
        msg = I._recv_exact(s, n)
        assert rid == 7 and st == 400 and msg
        s.settimeout(10)
        try:  # the owner closed the connection (reset when unread bytes were left behind)
            assert s.recv(1) == b""
        except ConnectionResetError:
            pass
    finally:
        s.close()
    assert svc.seen == []


def test_ingest_client_fails_pending_on_owner_loss(server):
    path, _, srv = server
    lost = threading.Event()
    cli = I.IngestClient(path, connect_timeout=10, on_lost=lost.set)
    ev, box = threading.Event(), {}
    # a request that is never answered: the owner's service holds it
    srv.svc.submit = lambda layer, img, done: None

    def cb(st, data):
        box["r"] = (st, data)
        ev.set()

    cli.send(I.DECONV, cb, layer="block1_conv1", h=1, w=1, payload=np.zeros((1, 1, 3), np.uint8))
    srv.close()  # stops accepting; the live connection is closed from this side below
    cli.sock.shutdown(socket.SHUT_RD)
    assert ev.wait(10) and box["r"][0] == 500
    assert lost.wait(10)
