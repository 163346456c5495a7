"""Service behind the ``POST /deepdream`` extension route (not in the reference): decode ->
DeepDream (InceptionV3 or ResNet-50) on the GPU worker -> JPEG data URL (same conventions as
``POST /``).

Engines: images up to ``dream_tile`` per side on one GPU run the untiled engine (one hipGraph per
octave); larger ones run TiledDeepDream (rolled tiles as one batch). With several
ranks (``runner``: parallel/sharded.py) every batch runs TILED ACROSS ALL RANKS: rank 0 posts a
``dream`` command on the control plane, broadcasts the images over RCCL, and every rank runs its
share of the (tile, image) units with the packs all-gathered each step; every rank ends with the
same result and rank 0 answers.

Requests are batched: a request joins the pending list after decode + size validation; the GPU
worker takes the oldest request and every pending one with the same (model, octaves, steps,
H, W) key (waiting up to ``dream_window_ms`` for more, at most ``dream_max_batch``) and runs them
as ONE DeepDream batch. Every image's loss, gradient normalisation and max-loss flag are per
image (engine/deepdream.py), so batching is exact; the batch is padded to a power of two by
repeating the last image so the per-(B, H, W) hipGraph cache sees few distinct batch sizes."""
from __future__ import annotations

import asyncio
import collections
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Deque, Dict, List, Optional, Tuple

import numpy as np
import torch

from ..codec import encode_data_url, read_data_url
from ..config import Config
from ..engine.deepdream import RESNET_LAYERS, DeepDream, DreamSettings, TiledDeepDream
from ..utils import metrics as M

MAX_SIDE = 1024
MODELS = ("inception_v3", "resnet50")


@dataclass
class _Req:
    img: torch.Tensor  # u8 [H, W, 3], already resized to <= MAX_SIDE
    key: Tuple[Any, ...]  # (model, octaves, steps, H, W)
    fut: asyncio.Future
    loop: asyncio.AbstractEventLoop
    t0: float = field(default_factory=time.perf_counter)


def _bucket(n: int, cap: int) -> int:
    b = 1
    while b < n:
        b *= 2
    return max(n, min(b, cap))


def _resolve(fut: asyncio.Future, value=None, exc: Optional[BaseException] = None) -> None:
    if fut.done():
        return
    if exc is not None:
        fut.set_exception(exc)
    else:
        fut.set_result(value)


def make_dream_net(cfg: Config, model: str, device):
    """The /deepdream network on ``device``: seeded random init or the configured weights. Every
    rank builds it from the same seed / file, so the replicas are identical without a broadcast."""
    from ..models.dream_import import load_weights, new_model

    net = new_model(model, cfg.seed)
    path = cfg.inception_weights if model == "inception_v3" else cfg.resnet_weights
    if path:
        load_weights(net, path)
    return net.build(device)


def dream_settings(model: str, octaves: int, steps: int) -> DreamSettings:
    s = DreamSettings() if model == "inception_v3" else DreamSettings(layers=dict(RESNET_LAYERS))
    s.octaves, s.iterations = octaves, steps
    return s


def tiled_engine(cache: Dict[Tuple[str, int, int], TiledDeepDream], nets: Dict[str, Any], cfg: Config, model: str,
                 octaves: int, steps: int, device, info=None) -> TiledDeepDream:
    """One TiledDeepDream per (model, octaves, steps) with its own settings (no shared mutable
    settings between batches of different keys); the shift generator is re-seeded per batch by the
    caller so every rank rolls identically."""
    key = (model, octaves, steps)
    if key not in cache:
        if model not in nets:
            nets[model] = make_dream_net(cfg, model, device)
        cache[key] = TiledDeepDream(nets[model], dream_settings(model, octaves, steps), tile=cfg.dream_tile,
                                    info=info, seed=cfg.seed, use_graphs=cfg.hip_graphs)
    return cache[key]


class DreamService:
    def __init__(self, cfg: Optional[Config] = None, runner=None):
        """``runner``: parallel.sharded.ShardedRunner of a multi-rank service: every /deepdream batch
        then runs tiled across all ranks (its control plane and process group)."""
        self.cfg = cfg or Config.from_env()
        self.runner = runner
        self.device = torch.device(self.cfg.resolve_device() if runner is None else str(runner.info.device))
        self._engines: Dict[str, DeepDream] = {}
        self._tiled: Dict[Tuple[str, int, int], TiledDeepDream] = {}
        self._nets: Dict[str, Any] = {}
        self._lock = threading.Lock()
        self._run_lock = threading.RLock()  # one batch at a time (engine settings are per batch)
        self._cv = threading.Condition()
        self._pending: List[_Req] = []
        self._stop = False
        self._worker: Optional[threading.Thread] = None
        self.max_batch = max(1, self.cfg.dream_max_batch)
        self.window_s = max(0.0, self.cfg.dream_window_ms) / 1e3
        # real (unpadded) sizes of the most recent batches, for tests (bounded: a long-running
        # service must not grow it; M.BATCH_SIZE keeps the full histogram)
        self.batches: Deque[int] = collections.deque(maxlen=1024)

    # ------------------------------------------------------------------ engines
    @staticmethod
    def validate(model: str, octaves: int, steps: int) -> None:
        if model not in MODELS:
            raise ValueError("model must be inception_v3 or resnet50")
        if not (1 <= octaves <= 6 and 1 <= steps <= 100):
            raise ValueError("octaves must be 1..6 and steps 1..100")

    def engine(self, model: str, octaves: int, steps: int) -> DeepDream:
        """The untiled engine of ``model``. Its settings are set per batch, so it is only handed out
        under ``_run_lock``, which ``run_batch`` holds for the whole batch (a second thread's batch
        waits instead of changing octaves / steps under a running one)."""
        self.validate(model, octaves, steps)
        assert self._run_lock._is_owned(), "DreamService.engine: hold _run_lock (run_batch does)"
        with self._lock:
            if model not in self._engines:
                if model not in self._nets:
                    self._nets[model] = make_dream_net(self.cfg, model, self.device)
                s = dream_settings(model, octaves, steps)
                self._engines[model] = DeepDream(self._nets[model], s, use_graphs=self.cfg.hip_graphs)
            e = self._engines[model]
        e.s.octaves, e.s.iterations = octaves, steps
        return e

    def tiled(self, model: str, octaves: int, steps: int) -> TiledDeepDream:
        self.validate(model, octaves, steps)
        with self._lock:
            return tiled_engine(self._tiled, self._nets, self.cfg, model, octaves, steps, self.device)

    @property
    def world(self) -> int:
        return self.runner.world if self.runner is not None else 1

    def status(self) -> dict:
        return {"world": self.world, "tile": self.cfg.dream_tile, "models": sorted(self._nets),
                "batches": len(self.batches)}

    # ------------------------------------------------------------------ request prep (codec pool)
    def prepare(self, img: np.ndarray, octaves: int) -> torch.Tensor:
        """Decoded RGB -> u8 [H, W, 3] at most MAX_SIDE per side; rejects images whose smallest
        octave would be under 75 px (the InceptionV3 minimum)."""
        h, w = img.shape[:2]
        scale = min(1.0, MAX_SIDE / max(h, w))
        t = torch.from_numpy(np.ascontiguousarray(img))
        if scale < 1.0:
            from ..engine.deepdream import resize

            t = resize(t.unsqueeze(0).float(), (int(h * scale), int(w * scale)))[0]
            t = t.round().clamp(0, 255).to(torch.uint8)
        small = min(t.shape[:2]) / (DreamSettings().octave_scale ** (octaves - 1))
        if small < 75:
            raise ValueError(f"image too small for {octaves} octaves (smallest octave side {small:.0f} < 75)")
        return t.contiguous()

    # ------------------------------------------------------------------ batching worker
    def _ensure_worker(self) -> None:
        with self._cv:
            if self._worker is None or not self._worker.is_alive():
                self._stop = False
                self._worker = threading.Thread(target=self._loop, name="dv-dream", daemon=True)
                self._worker.start()

    def _take(self) -> Optional[List[_Req]]:
        """Oldest pending request plus every same-key one (after up to ``window_s`` of waiting)."""
        with self._cv:
            while not self._pending and not self._stop:
                self._cv.wait()
            if not self._pending:
                return None
            key = self._pending[0].key
            deadline = time.monotonic() + self.window_s
            while True:
                n = sum(1 for r in self._pending if r.key == key)
                left = deadline - time.monotonic()
                if n >= self.max_batch or left <= 0 or self._stop:
                    break
                self._cv.wait(left)
            batch = [r for r in self._pending if r.key == key][: self.max_batch]
            taken = {id(r) for r in batch}
            self._pending = [r for r in self._pending if id(r) not in taken]
            M.QUEUE_DEPTH.set(len(self._pending), route="/deepdream")
            return batch

    def run_batch(self, imgs: List[torch.Tensor], model: str, octaves: int, steps: int) -> np.ndarray:
        """u8 [H, W, 3] images of one shape -> dreamed u8 [n, H, W, 3] (one engine batch): across
        every rank when the service has several, tiled on this GPU for sides > dream_tile, else the
        untiled engine."""
        with self._run_lock:
            return self._run_batch(imgs, model, octaves, steps)

    def _run_batch(self, imgs: List[torch.Tensor], model: str, octaves: int, steps: int) -> np.ndarray:
        n = len(imgs)
        t0 = time.perf_counter()
        H, W = imgs[0].shape[:2]
        if self.world > 1:
            out = self.runner.dream(torch.stack(imgs), model, octaves, steps)
        elif max(H, W) > self.cfg.dream_tile:
            e = self.tiled(model, octaves, steps)
            e.gen.manual_seed(self.cfg.seed)  # same rolls as the multi-rank path for the same input
            out = e.dream_u8(torch.stack(imgs)).cpu().numpy()
        else:
            e = self.engine(model, octaves, steps)
            pad = _bucket(n, self.max_batch) - n
            x = torch.stack(imgs + [imgs[-1]] * pad)
            out = e.dream_u8(x)[:n].cpu().numpy()
        M.ENGINE_TIME.observe(time.perf_counter() - t0, stage="deepdream")
        M.BATCH_SIZE.observe(n, route="/deepdream")
        M.IMAGES.inc(n, route="/deepdream")
        return out

    def _loop(self) -> None:
        while True:
            batch = self._take()
            if batch is None:
                return
            model, octaves, steps = batch[0].key[:3]
            self.batches.append(len(batch))
            try:
                out = self.run_batch([r.img for r in batch], model, octaves, steps)
            except Exception as exc:  # noqa: BLE001 - delivered to every request of the batch
                for r in batch:
                    r.loop.call_soon_threadsafe(_resolve, r.fut, None, exc)
                continue
            for r, o in zip(batch, out):
                r.loop.call_soon_threadsafe(_resolve, r.fut, o)

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        if self._worker is not None:
            self._worker.join(timeout=30)

    # ------------------------------------------------------------------ request entry
    async def dream(self, uri: str, model: str = "inception_v3", octaves: int = 4, steps: int = 20) -> str:
        self.validate(model, octaves, steps)
        loop = asyncio.get_running_loop()
        img = await loop.run_in_executor(None, read_data_url, uri)
        t = await loop.run_in_executor(None, self.prepare, img, octaves)
        fut = loop.create_future()
        self._ensure_worker()
        with self._cv:
            self._pending.append(_Req(t, (model, octaves, steps, t.shape[0], t.shape[1]), fut, loop))
            M.QUEUE_DEPTH.set(len(self._pending), route="/deepdream")
            self._cv.notify_all()
        out = await fut
        return await loop.run_in_executor(None, encode_data_url, out, self.cfg.jpeg_quality)
