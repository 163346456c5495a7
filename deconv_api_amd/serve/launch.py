"""Server launcher: one process per GPU (reference: a single uvicorn worker, Dockerfile:15).

    python -m torch.distributed.run --standalone --nproc-per-node 8 -m deconv_api_amd.serve.launch
    python -m deconv_api_amd.serve.launch            # single GPU / CPU

Rank 0 creates (or loads) the VGG16 weights and broadcasts them over RCCL, then runs uvicorn
with the batching service; every other rank builds the same engine on its GPU and serves rank
0's shards (parallel/sharded.py) until shutdown.
"""
from __future__ import annotations

import argparse
import os

import torch

from ..config import Config
from ..engine.deconvnet import DeconvNet
from ..parallel import dist as pdist
from ..parallel.sharded import ShardedRunner
from ..utils.logging import get_logger, setup
from .service import DeconvService, load_model

log = get_logger("deconv_api_amd.launch")


def build_engine(cfg: Config, info: pdist.DistInfo) -> DeconvNet:
    model = load_model(cfg) if info.is_main else load_model(Config(**{**cfg.__dict__, "seed": cfg.seed}))
    if info.world > 1:
        sd = pdist.broadcast_state(model.state_dict(), info)
        model = type(model).from_state_dict(sd)
    dtype = torch.bfloat16 if info.device.type == "cuda" else torch.float32
    return DeconvNet(model.build(info.device, dtype))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default=None)
    ap.add_argument("--port", type=int, default=None)
    a = ap.parse_args(argv)
    overrides = {k: v for k, v in (("host", a.host), ("port", a.port)) if v is not None}
    cfg = Config.from_env(**overrides)
    setup(cfg.log_json)
    info = pdist.init()
    eng = build_engine(cfg, info)
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
