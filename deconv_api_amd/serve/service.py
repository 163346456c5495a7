"""Request batching service: async front end -> GPU worker thread -> host codec pool.

The reference runs each request to completion on the event-loop thread (``async def`` with
blocking compute, app/main.py:46), so requests serialize and the server stalls. Here:
  * decode (PIL) and JPEG encode run on a thread pool (they release the GIL);
  * requests are queued and a single GPU worker thread drains them in batches (same target layer,
    up to ``max_batch``, waiting at most ``batch_timeout_ms`` for stragglers); one batch = one
    engine call over B images x 4 filters;
  * uploads use pinned host buffers + non_blocking copies on the compute stream; the GPU-side
    resize+preprocess kernel writes straight into the batch tensor;
  * backpressure: beyond ``max_queue`` pending requests new ones fail fast (HTTP 503).
"""
from __future__ import annotations

import asyncio
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from .. import ops
from ..codec import CodecPool, encode_data_url, read_data_url
from ..config import Config
from ..engine.deconvnet import DeconvNet, UnknownLayerError, VALID_MODES
from ..models.vgg16 import VGG16
from ..utils import metrics as M
from ..utils.faults import FaultInjector
from ..utils.logging import get_logger

log = get_logger("deconv_api_amd.serve")


class ServiceOverloaded(RuntimeError):
    pass


@dataclass
class _Job:
    layer: str
    image: np.ndarray
    loop: asyncio.AbstractEventLoop
    future: asyncio.Future
    t_enq: float = field(default_factory=time.perf_counter)


def load_model(cfg: Config) -> VGG16:
    if cfg.weights:
        if cfg.weights.endswith((".h5", ".hdf5")):
            from ..models.keras_import import load_keras_vgg16_h5

            return load_keras_vgg16_h5(cfg.weights)
        return VGG16.load(cfg.weights)
    return VGG16.random(cfg.seed)


class DeconvService:
    def __init__(self, cfg: Optional[Config] = None, engine: Optional[DeconvNet] = None, runner=None):
        """``runner``: optional parallel.sharded.ShardedRunner (world > 1): batches are then split
        across all ranks' GPUs and the mosaics all-gathered over RCCL."""
        self.cfg = cfg or Config.from_env()
        self.runner = runner
        dev = self.cfg.resolve_device() if runner is None else str(runner.info.device)
        self.device = torch.device(dev)
        if engine is None:
            model = load_model(self.cfg)
            dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
            engine = DeconvNet(model.build(self.device, dtype))
        self.engine = engine
        self.codec = CodecPool(self.cfg.codec_workers)
        self.q: "queue.Queue[_Job]" = queue.Queue()
        self.batches = 0
        self.images = 0
        self.last_error: Optional[str] = None
        self._stop = threading.Event()
        self.faults = FaultInjector.from_env()
        self._batch_t0: Optional[float] = None
        self.stalled = False
        self._thread = threading.Thread(target=self._worker, name="dv-gpu-worker", daemon=True)
        self._thread.start()
        self._watchdog = threading.Thread(target=self._watch, name="dv-watchdog", daemon=True)
        self._watchdog.start()

    def _watch(self):
        """Marks the service not-ready while a batch runs longer than the request timeout (a hung
        kernel or a dead peer); clears when batches complete again."""
        while not self._stop.wait(0.5):
            t0 = self._batch_t0
            self.stalled = t0 is not None and time.perf_counter() - t0 > self.cfg.request_timeout_s

    # ------------------------------------------------------------------ front end
    def validate_layer(self, layer: str) -> None:
        try:
            self.engine._check_layer(layer)
        except UnknownLayerError:
            raise

    async def deconv(self, uri: str, layer: str) -> str:
        """The reference's POST / pipeline for one request -> data URL string."""
        self.validate_layer(layer)
        if self.q.qsize() >= self.cfg.max_queue:
            raise ServiceOverloaded("request queue is full")
        loop = asyncio.get_running_loop()
        img = await loop.run_in_executor(self.codec.ex, read_data_url, uri)
        fut = loop.create_future()
        self.q.put(_Job(layer, img, loop, fut))
        M.QUEUE_DEPTH.set(self.q.qsize())
        mosaic = await asyncio.wait_for(fut, timeout=self.cfg.request_timeout_s)
        return await loop.run_in_executor(self.codec.ex, encode_data_url, mosaic, self.cfg.jpeg_quality)

    def status(self) -> dict:
        st = {"device": str(self.device), "worker_alive": self._thread.is_alive() and not self.stalled,
              "stalled": self.stalled, "queue_depth": self.q.qsize(),
              "batches": self.batches, "images": self.images, "last_error": self.last_error,
              "native": ops.native.available() if self.device.type == "cuda" else None}
        if self.runner is not None:
            st.update(world=self.runner.world, degraded=self.runner.degraded, runner_error=self.runner.last_error)
        if self.device.type == "cuda":
            st["gpu"] = torch.cuda.get_device_name(self.device)
        return st

    def close(self):
        self._stop.set()
        self._thread.join(timeout=5)
        self.codec.shutdown()

    # ------------------------------------------------------------------ GPU worker
    def _collect(self) -> List[_Job]:
        try:
            first = self.q.get(timeout=0.1)
        except queue.Empty:
            return []
        jobs = [first]
        deadline = time.perf_counter() + self.cfg.batch_timeout_ms / 1e3
        while len(jobs) < self.cfg.max_batch:
            rem = deadline - time.perf_counter()
            if rem <= 0:
                break
            try:
                jobs.append(self.q.get(timeout=rem))
            except queue.Empty:
                break
        return jobs

    def _worker(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        last_beat = time.perf_counter()
        while not self._stop.is_set():
            jobs = self._collect()
            if not jobs:
                if self.runner is not None and time.perf_counter() - last_beat > 10.0:
                    self.runner.ping()  # idle heartbeat to the follower ranks
                    last_beat = time.perf_counter()
                continue
            last_beat = time.perf_counter()
            M.QUEUE_DEPTH.set(self.q.qsize())
            by_layer = {}
            for j in jobs:
                by_layer.setdefault(j.layer, []).append(j)
            for layer, group in by_layer.items():
                try:
                    mos = self.run_batch(layer, [j.image for j in group])
                    for j, m in zip(group, mos):
                        _deliver(j.loop, _set_result, j.future, m)
                except Exception as e:  # noqa: BLE001 - delivered to every waiting request
                    self.last_error = repr(e)
                    log.exception("batch failed")
                    for j in group:
                        _deliver(j.loop, _set_exc, j.future, e)

    def preprocess(self, images: List[np.ndarray]) -> torch.Tensor:
        B, S = len(images), self.cfg.image_size
        if self.device.type == "cuda":
            x = torch.empty(B, S, S, 8, dtype=torch.bfloat16, device=self.device)
            for b, img in enumerate(images):
                h = torch.from_numpy(np.ascontiguousarray(img)).pin_memory()
                ops.resize_preprocess(h.to(self.device, non_blocking=True), x[b])
            return x
        x = torch.empty(B, S, S, 8, dtype=torch.float32)
        for b, img in enumerate(images):
            x[b] = ops.preprocess_ref(ops.resize_u8_ref(img, S, S), 8, torch.float32)
        return x

    def run_batch(self, layer: str, images: List[np.ndarray]) -> np.ndarray:
        t0 = time.perf_counter()
        self._batch_t0 = t0
        try:
            if self.runner is not None:
                mos = self.runner.run(layer, images)
            else:
                self.faults.on_batch()
                x = self.preprocess(images)
                res = self.engine.run(x, layer, k=self.cfg.filters, mode=self.cfg.mode)
                mos = res.mosaic.cpu().numpy()
        finally:
            self._batch_t0 = None
        dt = time.perf_counter() - t0
        self.batches += 1
        self.images += len(images)
        M.BATCH_SIZE.observe(len(images))
        M.ENGINE_TIME.observe(dt, stage="batch")
        M.IMAGES.inc(len(images), layer=layer)
        return mos


def _deliver(loop: asyncio.AbstractEventLoop, fn, fut, v):
    try:
        loop.call_soon_threadsafe(fn, fut, v)
    except RuntimeError:  # the requester's event loop is gone (client timed out / shut down)
        pass


def _set_result(fut: asyncio.Future, v):
    if not fut.done():
        fut.set_result(v)


def _set_exc(fut: asyncio.Future, e: BaseException):
    if not fut.done():
        fut.set_exception(e)
