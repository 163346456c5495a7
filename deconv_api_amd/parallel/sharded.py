"""Data-parallel deconvnet serving across ranks, with failover that re-forms the group over the
surviving GPUs (the reference is one blocking worker, app/main.py:46 and
Dockerfile:15).

Planes:
  * control (parallel/elastic.py): the job's TCPStore. Rank 0 posts a command per batch; every
    collective is entered only after rank 0 has seen every member acknowledge the step before it
    and released a "go" key, so no rank ever waits in a collective on a dead peer. Followers
    publish heartbeats; a missing ack plus a stale heartbeat marks a peer dead;
  * data (RCCL over xGMI; Gloo on CPU): rank 0 resizes the whole batch on its GPU from one staged
    upload (runtime/staging.py) into uint8 224x224x3 (150 KB/image) and ``scatter``s each rank
    only its shard; every rank preprocesses its shard and runs the engine from a captured hipGraph
    per (layer, shard bucket); the uint8 mosaics are ``gather``ed to rank 0 only (1/N of the bytes
    of an all-gather; rank 0 is the only rank that answers HTTP).

Per batch (epoch e, sequence s):
  rank 0:   cmd -> wait ready(all) -> go1 -> scatter -> compute -> wait done(all) -> go2 -> gather
  follower: wait cmd -> ready -> wait go1 -> scatter -> compute -> done -> wait go2 -> gather

Failure: a follower that dies (or stops heartbeating) is detected while rank 0 waits for an ack.
Rank 0 then publishes ``reform`` on the keys the survivors wait on, the survivors and rank 0
tear down the process group and build a new one over the survivors (renumbered, new store
prefix), and the batch is recomputed on the new world. A local error on rank 0 (bad input,
kernel check) fails only that batch; it never degrades the group.
"""
from __future__ import annotations

import json
import time
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..utils.faults import FaultInjector
from ..utils.logging import get_logger
from .dist import DistInfo, shard_sizes
from .elastic import Control, PeerLost

log = get_logger("deconv_api_amd.sharded")


class ShardedRunner:
    def __init__(self, engine, info: DistInfo, image_size: int = 224, k: int = 4, mode: str = "all",
                 use_graphs: bool = True, hb_timeout: float = 3.0, ack_timeout: float = 600.0):
        self.engine = engine
        self.info = info
        self.S = image_size
        self.k = k
        self.mode = mode
        self.batches = 0
        self.reforms = 0
        self.last_error: Optional[str] = None
        self.faults = FaultInjector.from_env(info.rank)
        self.ctl = Control(info, hb_timeout=hb_timeout, ack_timeout=ack_timeout) if info.world > 1 else None
        self.graphs = None
        if use_graphs and info.device.type == "cuda":
            from ..engine.graphs import GraphedDeconv

            self.graphs = GraphedDeconv(engine, image_size, k, mode)
        self.ring = None
        if info.device.type == "cuda" and info.rank == 0:
            from ..runtime.staging import StagingRing

            self.ring = StagingRing(info.device)

    @property
    def world(self) -> int:
        return self.info.world

    @property
    def degraded(self) -> bool:
        """True once the group lost a member (it keeps serving on the survivors)."""
        return self.reforms > 0

    # ----------------------------------------------------------------- shared compute
    def _resize_u8(self, images: List[np.ndarray], npad: int) -> torch.Tensor:
        """rank 0: all images -> uint8 [npad, S, S, 3] (zero rows pad to npad) on this rank's device."""
        S = self.S
        if self.ring is not None:
            out = torch.zeros(npad, S, S, 3, dtype=torch.uint8, device=self.info.device)
            self.ring.stage(images, out)
            return out
        out = torch.zeros(npad, S, S, 3, dtype=torch.uint8)
        for b, img in enumerate(images):
            out[b] = torch.from_numpy(ops.resize_u8_ref(img, S, S))
        return out

    def _preprocess(self, u8: torch.Tensor) -> torch.Tensor:
        if u8.is_cuda:
            x = torch.empty(*u8.shape[:3], 8, dtype=torch.bfloat16, device=u8.device)
            ops.native.lib().preprocess_u8(u8, x)
            return x
        return torch.stack([ops.preprocess_ref(u8[b].numpy(), 8, torch.float32) for b in range(u8.shape[0])]) \
            if u8.shape[0] else torch.empty(0, self.S, self.S, 8)

    def _engine(self, x: torch.Tensor, layer: str) -> torch.Tensor:
        if self.graphs is not None:
            return self.graphs.run(x, layer).mosaic[: x.shape[0]]
        return self.engine.run(x, layer, k=self.k, mode=self.mode).mosaic

    def _local(self, layer: str, images: List[np.ndarray]) -> torch.Tensor:
        """Single-process reference of a batch (tests, and the world-1 path)."""
        u8 = self._resize_u8(images, len(images))
        return self._engine(self._preprocess(u8), layer)

    # ----------------------------------------------------------------- rank 0
    def run(self, layer: str, images: List[np.ndarray]) -> np.ndarray:
        return self.finish(self.launch(layer, images))

    def launch(self, layer: str, images: List[np.ndarray]):
        """rank 0: run the batch's control steps and collectives and enqueue the mosaics' copy to
        pinned host memory; returns a handle for ``finish`` (the D2H may still be in flight, so
        the service's worker can start the next batch while this one drains)."""
        assert self.info.rank == 0
        self.batches += 1
        while True:
            if self.world == 1:
                self.faults.on_batch()
                return self._to_host(self._local(layer, images), len(images))
            try:
                return self._run_group(layer, images)
            except PeerLost as e:
                self.last_error = repr(e)
                log.error("peer lost, re-forming over the survivors", extra={"fields": {"dead": e.dead}})
                self.ctl.reform(e.dead)
                self.reforms += 1

    @staticmethod
    def _to_host(mos: torch.Tensor, n: int):
        if not mos.is_cuda:
            return ("host", mos[:n].numpy())
        host = torch.empty((n, *mos.shape[1:]), dtype=mos.dtype, pin_memory=True)
        host.copy_(mos[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ("event", ev, host)

    @staticmethod
    def finish(handle) -> np.ndarray:
        if handle[0] == "host":
            return handle[1]
        handle[1].synchronize()
        return handle[2].numpy()

    def _run_group(self, layer: str, images: List[np.ndarray]):
        n = len(images)
        per = shard_sizes(n, self.world)[0]
        ctl = self.ctl
        seq = ctl.post_cmd({"op": "run", "layer": layer, "n": n, "per": per})
        u8 = self._resize_u8(images, per * self.world)  # overlaps the followers' acks
        ctl.wait_acks("ready", seq)
        ctl.go("go1", seq)
        shard = torch.empty(per, self.S, self.S, 3, dtype=torch.uint8, device=u8.device)
        dist.scatter(shard, scatter_list=list(u8.chunk(self.world)), src=0)
        self.faults.on_batch()
        mos = self._engine(self._preprocess(shard), layer).contiguous()
        ctl.wait_acks("done", seq)
        ctl.go("go2", seq)
        parts = [torch.empty_like(mos) for _ in range(self.world)]
        dist.gather(mos, gather_list=parts, dst=0)
        return self._to_host(torch.cat(parts), n)

    def ping(self) -> bool:
        """Idle liveness check: re-forms the group if a follower stopped heartbeating."""
        if self.world == 1 or self.ctl is None:
            return True
        dead = self.ctl.stale()
        if dead:
            self.ctl.reform(dead)
            self.reforms += 1
            return False
        return True

    def stop(self):
        if self.ctl is not None and self.info.rank == 0:
            if self.world > 1:
                self.ctl.post_cmd({"op": "stop"})
            self.ctl.close()

    # ----------------------------------------------------------------- followers
    def follow(self) -> int:
        """Serve rank 0's batches until 'stop' (or until dropped from the group). Returns the
        number of batches run."""
        assert self.info.rank != 0
        ctl = self.ctl
        done = 0
        while True:
            seq, msg = ctl.wait_cmd()
            if msg["op"] == "stop":
                ctl.close()
                return done
            if msg["op"] == "reform":
                if not ctl.follow_reform(msg):
                    return done
                continue
            per = msg["per"]
            dev = self.info.device
            ctl.ack("ready", seq)
            r = ctl.wait_go("go1", seq)
            if r is not None:  # reform announced instead of go
                if not ctl.follow_reform(r):
                    return done
                continue
            shard = torch.empty(per, self.S, self.S, 3, dtype=torch.uint8, device=dev)
            dist.scatter(shard, scatter_list=None, src=0)
            self.faults.on_batch()
            mos = self._engine(self._preprocess(shard), msg["layer"]).contiguous()
            if mos.is_cuda:
                torch.cuda.current_stream(dev).synchronize()
            ctl.ack("done", seq)
            r = ctl.wait_go("go2", seq)
            if r is not None:
                if not ctl.follow_reform(r):
                    return done
                continue
            dist.gather(mos, gather_list=None, dst=0)
            done += 1
