"""HTTP front-end process of a rank (``DV_FRONTENDS`` > 0; transport and design: serve/ingest.py).

    python -m deconv_api_amd.serve.frontend --sock /tmp/dv-ingest-80-r0-123.sock --index 0

Started (and restarted when it dies) by the rank's front-end supervisor (serve/supervisor.py), which
serve/launch.py starts before the GPU owner touches the GPU (so no process with a GPU context starts
another program); never touches the GPU itself. It runs the same FastAPI app as the
single-process server (api/app.py, the reference's surface app/main.py:19-78) on a listening
socket bound with SO_REUSEPORT to the serving port, next to every other front end of every rank
on the node. A request is parsed and decoded here (native base64, PIL on the codec threads), its
pixels go to the GPU owner over the Unix socket, and the owner's data URL is the response.
The process exits when its owner goes away (the connection drops).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import time

from ..codec import CodecPool, read_data_url
from ..config import Config
from ..engine.deconvnet import UnknownLayerError
from ..utils import metrics as M
from ..utils.logging import get_logger, setup
from . import ingest

log = get_logger("deconv_api_amd.frontend")


class RemoteError(RuntimeError):
    """A non-200 answer of the GPU owner, carried to the HTTP response unchanged."""

    def __init__(self, status: int, msg: str):
        super().__init__(msg)
        self.status = status
        self.msg = msg


def _settle(fut: asyncio.Future, st: int, data: bytes) -> None:
    if not fut.done():
        fut.set_result((st, data))


class _Remote:
    def __init__(self, client: ingest.IngestClient, cfg: Config):
        self.client = client
        self.cfg = cfg

    async def _request(self, send, raw: bool = False):
        """``send(cb)`` queues the request (on a codec thread); -> the owner's 200 payload (bytes when
        ``raw``: the data URL goes into the HTTP body as is, api/app.py)."""
        loop = asyncio.get_running_loop()
        fut = loop.create_future()

        def cb(st, data):  # the client's reader thread
            loop.call_soon_threadsafe(_settle, fut, st, data)

        await send(cb)
        st, data = await asyncio.wait_for(fut, timeout=self.cfg.request_timeout_s)
        if st != 200:
            raise RemoteError(st, data.decode("utf-8", errors="replace"))
        return data if raw else data.decode("ascii", errors="replace")


class RemoteService(_Remote):
    """The ``DeconvService`` surface api/app.py uses, answered by the rank's GPU owner."""

    def __init__(self, client: ingest.IngestClient, cfg: Config):
        super().__init__(client, cfg)
        st, data = client.call(ingest.LAYERS, timeout=600)
        if st != 200:
            raise RuntimeError(f"GPU owner refused the layer list: {data!r}")
        info = json.loads(data)
        self.layers = info["layers"]
        self._names = set(info["names"])  # every engine name: the owner answers e.g. input_1 itself
        self.codec = CodecPool(cfg.codec_workers)

    def layer_names(self):
        return list(self.layers)

    def validate_layer(self, layer: str) -> None:
        if layer not in self._names:  # same message as DeconvNet._check_layer; the rest is the owner's
            raise UnknownLayerError(f"unknown layer {layer!r}; valid: {self.layers}")

    def _decode_send(self, uri: str, layer: str, cb) -> None:
        t0 = time.perf_counter()
        img = read_data_url(uri)  # ImageDecodeError -> 400 in the app
        # the owner records it (its /metrics then cover every front end of the rank)
        self.client.send(ingest.DECONV, cb, layer, img.shape[0], img.shape[1], img,
                         decode_s=time.perf_counter() - t0)

    async def deconv(self, uri: str, layer: str) -> str:
        self.validate_layer(layer)
        loop = asyncio.get_running_loop()

        async def send(cb):
            await loop.run_in_executor(self.codec.ex, self._decode_send, uri, layer, cb)

        return await self._request(send, raw=True)

    def status(self) -> dict:
        try:
            st, data = self.client.call(ingest.STATUS, timeout=10)
        except (OSError, TimeoutError) as e:
            return {"worker_alive": False, "last_error": repr(e)}
        out = json.loads(data) if st == 200 else {"worker_alive": False, "last_error": data.decode()}
        out["frontend"] = {"pid": os.getpid()}
        return out

    def metrics_text(self) -> str:
        try:
            st, data = self.client.call(ingest.METRICS, timeout=10)
        except (OSError, TimeoutError):
            return M.REGISTRY.render()
        return M.merge_text(M.REGISTRY.render(), data.decode() if st == 200 else "")

    def close(self) -> None:
        self.codec.shutdown()


class RemoteDream(_Remote):
    """``DreamService.dream`` forwarded to the GPU owner (which validates and decodes)."""

    async def dream(self, uri: str, model: str = "inception_v3", octaves: int = 4, steps: int = 20) -> str:
        body = json.dumps({"model": model, "octaves": octaves, "steps": steps}).encode() + b"\n" + uri.encode()
        loop = asyncio.get_running_loop()

        async def send(cb):
            await loop.run_in_executor(None, lambda: self.client.send(ingest.DREAM, cb, payload=body))

        return await self._request(send)


def listen_socket(host: str, port: int, backlog: int = 4096) -> socket.socket:
    """TCP listener sharing ``port`` with every other front end on the node (SO_REUSEPORT: the
    kernel hashes each new connection to one of the listeners)."""
    fam = socket.AF_INET6 if ":" in host else socket.AF_INET
    s = socket.socket(fam, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(backlog)
    s.set_inheritable(True)
    return s


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sock", required=True, help="the GPU owner's ingest socket")
    ap.add_argument("--index", type=int, default=0)
    ap.add_argument("--host", default=None)
    ap.add_argument("--port", type=int, default=None)
    a = ap.parse_args(argv)
    overrides = {k: v for k, v in (("host", a.host), ("port", a.port)) if v is not None}
    cfg = Config.from_env(**overrides)
    setup(cfg.log_json)
    import sys

    if cfg.gil_switch_us > 0:
        sys.setswitchinterval(cfg.gil_switch_us / 1e6)
    client = ingest.IngestClient(a.sock, on_lost=lambda: os._exit(3))
    svc = RemoteService(client, cfg)
    import uvicorn

    from ..api.app import create_app

    app = create_app(svc, cfg, dream_service=RemoteDream(client, cfg))
    sock = listen_socket(cfg.host, cfg.port)
    log.info("front end serving", extra={"fields": {"index": a.index, "port": cfg.port, "pid": os.getpid()}})
    server = uvicorn.Server(uvicorn.Config(app, log_level="warning", access_log=False, timeout_keep_alive=30))
    try:
        server.run(sockets=[sock])
    finally:
        svc.close()
        client.close()


if __name__ == "__main__":
    main()
