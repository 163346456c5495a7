"""Data-parallel deconvnet execution across ranks (one process per GPU).

Rank 0 owns the request batch. Per batch:
  1. control plane (Gloo side group): rank 0 broadcasts {layer, n, per-rank size} plus the
     decoded uint8 images; every rank takes its contiguous shard (zero images pad the last
     shard so every rank runs the same static shape);
  2. every rank preprocesses its shard on its own GPU and runs the engine (B_r x 4 chains);
  3. data plane (RCCL over xGMI): one ``all_gather_into_tensor`` of the uint8 mosaics
     (602 KB per image) returns the whole batch in rank order; rank 0 drops the padding.
Followers sit in ``follow()`` until rank 0 sends ``stop``.
"""
from __future__ import annotations

import time
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from .dist import DistInfo, all_gather_rows, shard_sizes


class ShardedRunner:
    def __init__(self, engine, info: DistInfo, image_size: int = 224, k: int = 4, mode: str = "all"):
        self.engine = engine
        self.info = info
        self.S = image_size
        self.k = k
        self.mode = mode
        self.group = info.ctrl_group  # gloo side group (None -> default group, e.g. gloo on CPU)
        self.batches = 0

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

    def _compute(self, layer: str, images: List[np.ndarray], n: int, per: int) -> torch.Tensor:
        r = self.info.rank
        shard = images[r * per:(r + 1) * per]
        pad = per - len(shard)
        if pad:
            shard = list(shard) + [np.zeros((self.S, self.S, 3), np.uint8)] * pad
        x = self._prep(shard)
        res = self.engine.run(x, layer, k=self.k, mode=self.mode)
        return all_gather_rows(res.mosaic.contiguous(), self.info)

    # ----------------------------------------------------------------- rank 0
    def run(self, layer: str, images: List[np.ndarray]) -> np.ndarray:
        assert self.info.rank == 0
        n = len(images)
        per = shard_sizes(n, self.info.world)[0]
        if self.info.world > 1:
            dist.broadcast_object_list([{"op": "run", "layer": layer, "n": n, "per": per}, images], src=0,
                                       group=self.group)
        out = self._compute(layer, images, n, per)
        self.batches += 1
        return out[:n].cpu().numpy()

    def stop(self):
        if self.info.world > 1 and self.info.rank == 0:
            dist.broadcast_object_list([{"op": "stop"}, None], src=0, group=self.group)

    # ----------------------------------------------------------------- followers
    def follow(self, poll_timeout: Optional[float] = None) -> int:
        """Serve rank 0's batches until 'stop'. Returns the number of batches run."""
        assert self.info.rank != 0
        done = 0
        while True:
            box = [None, None]
            dist.broadcast_object_list(box, src=0, group=self.group)
            msg, images = box
            if msg["op"] == "stop":
                return done
            self._compute(msg["layer"], images, msg["n"], msg["per"])
            done += 1
