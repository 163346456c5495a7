"""Server launcher: one GPU-owner process per GPU (reference: a single uvicorn worker, Dockerfile:15).

    python -m torch.distributed.run --standalone --nproc-per-node 8 -m deconv_api_amd.serve.launch
    python -m deconv_api_amd.serve.launch            # single GPU / CPU

Rank 0 creates (or loads) the VGG16 weights and broadcasts them over RCCL; every rank builds the
same engine on its GPU. Two serving layouts:

  * ``DV_FRONTENDS=N`` (default 4): each rank starts a front-end supervisor (serve/supervisor.py)
    BEFORE touching its GPU; it runs N HTTP front-end processes (serve/frontend.py, restarted when
    one dies), all bound to the port with SO_REUSEPORT, and the rank serves what they decode through
    an ``IngestServer`` (serve/ingest.py). Ranks are independent on the request path:
    every rank parses, decodes, batches and encodes only its own front ends' requests, so HTTP
    throughput scales with the ranks (no rank-0 decode / resize / scatter). ``/deepdream`` runs on
    the receiving rank's GPU (tiled on that GPU above ``dream_tile``).
  * ``DV_FRONTENDS=0``: rank 0 runs uvicorn in-process and shards every batch across the ranks
    (parallel/sharded.py: scatter / gather, failover re-forming the group over the survivors,
    ``/deepdream`` tiled across every rank); the followers serve rank 0's command stream.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import threading

import torch

from ..config import Config
from ..engine.deconvnet import DeconvNet
from ..parallel import dist as pdist
from ..parallel.sharded import ShardedRunner
from ..utils.logging import get_logger, setup
from .service import DeconvService, load_model

log = get_logger("deconv_api_amd.launch")


def build_engine(cfg: Config, info: pdist.DistInfo) -> DeconvNet:
    model = load_model(cfg)
    if info.world > 1:
        sd = pdist.broadcast_state(model.state_dict(), info)
        model = type(model).from_state_dict(sd)
    return DeconvNet(model.build(info.device, cfg.torch_dtype(info.device)))


def spawn_frontends(cfg: Config, path: str, n: int) -> subprocess.Popen:
    """Start the rank's front-end supervisor (serve/supervisor.py), which starts the ``n`` front ends
    for the ingest socket ``path`` and restarts one that dies. Called before this process initialises
    the GPU: the children are fresh interpreters that never open it, and this process never starts
    another program after that."""
    return subprocess.Popen([sys.executable, "-m", "deconv_api_amd.serve.supervisor", "--sock", path, "--n", str(n),
                             "--owner-pid", str(os.getpid())],
                            env=dict(os.environ, DV_HOST=cfg.host, DV_PORT=str(cfg.port)))


def serve_frontends(cfg: Config, info: pdist.DistInfo, eng: DeconvNet, path: str, sup: subprocess.Popen,
                    stop: threading.Event) -> None:
    """This rank's GPU owner: the batching service + /deepdream behind the ingest socket, until
    ``stop`` is set or the front-end supervisor has exited (every front end down for good)."""
    from .dream_service import DreamService
    from .ingest import IngestServer

    svc = DeconvService(cfg, engine=eng)
    dream = DreamService(cfg)
    srv = IngestServer(path, svc, dream, rank=info.rank)
    log.info("serving through front ends", extra={"fields": {"rank": info.rank, "world": info.world,
                                                             "frontends": cfg.frontends, "port": cfg.port}})
    try:
        while not stop.wait(0.5):
            if sup.poll() is not None:
                log.error("front-end supervisor exited", extra={"fields": {"code": sup.returncode}})
                break
    finally:
        srv.close()
        if sup.poll() is None:
            sup.terminate()  # it terminates the front ends
        try:
            sup.wait(timeout=30)
        except subprocess.TimeoutExpired:
            sup.kill()
        svc.close()
        dream.close()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default=None)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--frontends", type=int, default=None, help="HTTP front-end processes per rank (0: in-process)")
    a = ap.parse_args(argv)
    overrides = {k: v for k, v in (("host", a.host), ("port", a.port), ("frontends", a.frontends)) if v is not None}
    cfg = Config.from_env(**overrides)
    setup(cfg.log_json)
    stop = threading.Event()
    sup, path = None, None
    if cfg.frontends > 0:
        from .ingest import socket_path

        # before pdist.init(): nothing that touches the GPU has run in this process yet
        path = socket_path(cfg.port, int(os.environ.get("RANK", "0")))
        sup = spawn_frontends(cfg, path, cfg.frontends)
        for sig in (signal.SIGTERM, signal.SIGINT):
            signal.signal(sig, lambda *_: stop.set())
    info = pdist.init()
    eng = build_engine(cfg, info)
    if cfg.frontends > 0:
        try:
            serve_frontends(cfg, info, eng, path, sup, stop)
        finally:
            if torch.distributed.is_initialized():  # ranks are independent here: no exit barrier
                torch.distributed.destroy_process_group()
        return
    runner = ShardedRunner(eng, info, cfg.image_size, cfg.filters, cfg.mode, cfg=cfg) if info.world > 1 else None
    if not info.is_main:
        n = runner.follow()
        log.info("follower done", extra={"fields": {"rank": info.rank, "batches": n}})
        pdist.shutdown()
        return
    import uvicorn

    from ..api.app import create_app

    from .dream_service import DreamService

    svc = DeconvService(cfg, engine=eng, runner=runner)
    # /deepdream: tiled across every rank when there are several (the same control plane)
    dream = DreamService(cfg, runner=runner)
    app = create_app(svc, cfg, dream_service=dream)
    log.info("serving", extra={"fields": {"world": info.world, "device": str(info.device), "port": cfg.port}})
    try:
        uvicorn.run(app, host=cfg.host, port=cfg.port, log_level="info")
    finally:
        if runner is not None:
            runner.stop()
        svc.close()
        dream.close()
        pdist.shutdown()


if __name__ == "__main__":
    main()
