"""hipGraph capture of the whole deconvnet step (forward -> top-k -> B x K backward -> mosaic)
per (layer, batch bucket). At serving batch sizes the step is launch-bound (~40 kernels plus
torch glue per batch); replaying one graph removes the per-launch host cost. Batches are padded
up to the next bucket so a handful of graphs cover every size."""
from __future__ import annotations

import threading
from typing import Dict, Tuple

import torch

from ..runtime.capture import capture
from .deconvnet import DeconvNet

BUCKETS = (1, 2, 4, 8, 16, 32, 64, 128, 256)


def bucket_for(n: int) -> int:
    for b in BUCKETS:
        if n <= b:
            return b
    return ((n + 255) // 256) * 256


class GraphedDeconv:
    def __init__(self, engine: DeconvNet, image_size: int = 224, k: int = 4, mode: str = "all"):
        self.engine = engine
        self.S = image_size
        self.k = k
        self.mode = mode
        self.device = engine.rt.device
        self._cache: Dict[Tuple[str, int], tuple] = {}
        self._lock = threading.Lock()

    def _capture(self, layer: str, B: int):
        x = torch.zeros(B, self.S, self.S, 8, dtype=self.engine.rt.dtype, device=self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up kernels/allocator off the capture stream
                self.engine.run(x, layer, k=self.k, mode=self.mode)
        torch.cuda.current_stream(self.device).wait_stream(s)
        # thread-local (runtime/capture.py): the service's completion thread keeps synchronizing on
        # earlier batches' events while the worker captures a new (layer, bucket) graph
        g, res = capture(lambda: self.engine.run(x, layer, k=self.k, mode=self.mode))
        return g, x, res

    def get(self, layer: str, B: int):
        key = (layer, B)
        with self._lock:
            if key not in self._cache:
                self._cache[key] = self._capture(layer, B)
            return self._cache[key]

    def input(self, layer: str, n: int) -> torch.Tensor:
        """The static input of the (layer, bucket(n)) graph, for a producer that writes straight
        into it (runtime/staging.py); follow with ``replay``."""
        return self.get(layer, bucket_for(n))[1]

    def replay(self, layer: str, n: int):
        B = bucket_for(n)
        g, xs, res = self.get(layer, B)
        if n < B:
            xs[n:].zero_()
        g.replay()
        return res

    def run(self, x: torch.Tensor, layer: str):
        """x: [n, S, S, 8] bf16 on device (n <= bucket). Returns the (graph-owned) result whose
        first n rows are valid until the next replay of the same (layer, bucket)."""
        n = x.shape[0]
        B = bucket_for(n)
        g, xs, res = self.get(layer, B)
        xs[:n].copy_(x)
        if n < B:
            xs[n:].zero_()
        g.replay()
        return res

    @property
    def captured(self):
        return sorted(self._cache)
