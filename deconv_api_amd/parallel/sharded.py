"""Data-parallel deconvnet execution across ranks (one process per GPU).

Rank 0 owns the request batch. Per batch:
  1. control plane (Gloo side group): rank 0 broadcasts {layer, n, per-rank size} plus the
     decoded uint8 images; every rank takes its contiguous shard (zero images pad the last
     shard so every rank runs the same static shape);
  2. every rank preprocesses its shard on its own GPU and runs the engine (B_r x 4 chains);
  3. data plane (RCCL over xGMI): one ``all_gather_into_tensor`` of the uint8 mosaics
     (602 KB per image) returns the whole batch in rank order; rank 0 drops the padding.
Followers sit in ``follow()`` until rank 0 sends ``stop``.

Failure handling: the per-batch control broadcast doubles as a heartbeat
(``ping()`` when idle). If a control or gather collective fails (a follower died: Gloo reports the
closed peer, or the group timeout fires), rank 0 marks the runner degraded, stops using the
process group and recomputes the batch - and every later one - on its own GPU, so requests keep
being answered while the pool is re-formed by the orchestrator.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..utils.faults import FaultInjector
from ..utils.logging import get_logger
from .dist import DistInfo, all_gather_rows, shard_sizes

log = get_logger("deconv_api_amd.sharded")


class ShardedRunner:
    def __init__(self, engine, info: DistInfo, image_size: int = 224, k: int = 4, mode: str = "all"):
        self.engine = engine
        self.info = info
        self.S = image_size
        self.k = k
        self.mode = mode
        self.group = info.ctrl_group  # gloo side group (None -> default group, e.g. gloo on CPU)
        self.batches = 0
        self.degraded = False
        self.last_error: Optional[str] = None
        self.faults = FaultInjector.from_env(info.rank)

    @property
    def world(self) -> int:
        return 1 if self.degraded else self.info.world

    # ----------------------------------------------------------------- shared compute
    def _prep(self, images: List[np.ndarray]) -> torch.Tensor:
        dev = self.info.device
        B, S = len(images), self.S
        if dev.type == "cuda":
            x = torch.empty(B, S, S, 8, dtype=torch.bfloat16, device=dev)
            for b, img in enumerate(images):
                ops.resize_preprocess(torch.from_numpy(np.ascontiguousarray(img)).to(dev, non_blocking=True), x[b])
            return x
        x = torch.empty(B, S, S, 8)
        for b, img in enumerate(images):
            x[b] = ops.preprocess_ref(ops.resize_u8_ref(img, S, S), 8, torch.float32)
        return x

    def _local(self, layer: str, images: List[np.ndarray]) -> torch.Tensor:
        return self.engine.run(self._prep(images), layer, k=self.k, mode=self.mode).mosaic

    def _compute(self, layer: str, images: List[np.ndarray], n: int, per: int) -> torch.Tensor:
        self.faults.on_batch()
        r = self.info.rank
        shard = images[r * per:(r + 1) * per]
        pad = per - len(shard)
        if pad:
            shard = list(shard) + [np.zeros((self.S, self.S, 3), np.uint8)] * pad
        mos = self._local(layer, shard)
        return all_gather_rows(mos.contiguous(), self.info)

    # ----------------------------------------------------------------- rank 0
    def run(self, layer: str, images: List[np.ndarray]) -> np.ndarray:
        assert self.info.rank == 0
        n = len(images)
        self.batches += 1
        if not self.degraded and self.info.world > 1:
            per = shard_sizes(n, self.info.world)[0]
            try:
                dist.broadcast_object_list([{"op": "run", "layer": layer, "n": n, "per": per}, images], src=0,
                                           group=self.group)
                out = self._compute(layer, images, n, per)
                return out[:n].cpu().numpy()
            except RuntimeError as e:  # a peer died / the group timed out
                self._degrade(e)
        self.faults.on_batch() if self.info.world == 1 else None
        return self._local(layer, images).cpu().numpy()

    def ping(self) -> bool:
        """Heartbeat over the control group; False (and degraded) if any follower is gone."""
        if self.degraded or self.info.world == 1:
            return not self.degraded
        try:
            dist.broadcast_object_list([{"op": "ping"}, None], src=0, group=self.group)
            return True
        except RuntimeError as e:
            self._degrade(e)
            return False

    def _degrade(self, e: BaseException) -> None:
        self.degraded = True
        self.last_error = repr(e)
        log.error("follower failure, continuing on rank 0 only", extra={"fields": {"error": repr(e)}})

    def stop(self):
        if self.info.world > 1 and self.info.rank == 0 and not self.degraded:
            try:
                dist.broadcast_object_list([{"op": "stop"}, None], src=0, group=self.group)
            except RuntimeError as e:
                self._degrade(e)

    # ----------------------------------------------------------------- followers
    def follow(self) -> int:
        """Serve rank 0's batches until 'stop'. Returns the number of batches run."""
        assert self.info.rank != 0
        done = 0
        while True:
            box = [None, None]
            dist.broadcast_object_list(box, src=0, group=self.group)
            msg, images = box
            if msg["op"] == "stop":
                return done
            if msg["op"] == "ping":
                continue
            self._compute(msg["layer"], images, msg["n"], msg["per"])
            done += 1
