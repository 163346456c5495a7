"""Request batching service: async front end -> GPU worker thread -> completion thread -> codec pool.

The reference runs each request to completion on the event-loop thread (``async def`` with
blocking compute, app/main.py:46), so requests serialize and the server stalls. Here:
  * decode (PIL, releases the GIL) runs on a thread pool; responses are JPEG-encoded by the
    native encoder (csrc/jpeg_enc.cpp) for a whole batch at once, GIL released, on native threads;
  * requests are queued and a single GPU worker thread drains them in batches (same target layer,
    up to ``max_batch``, waiting at most ``batch_timeout_ms`` for stragglers); one batch = one
    engine call over B images x 4 filters, replayed from a hipGraph per (layer, batch bucket);
  * the worker never waits for the GPU: the batch's decoded images go into one pinned staging
    slot, ONE H2D copy on the copy stream, ONE batched resize launch, the engine (graph replay) on
    the compute stream, and the mosaics' copy-back on a third stream (runtime/staging.py); a
    completion thread waits on the copy-back event and hands results to the requests, whose JPEG
    encode then overlaps the next batch's GPU work; per-stage hipEvent times go to /metrics;
  * backpressure: beyond ``max_queue`` pending requests new ones fail fast (HTTP 503);
  * a watchdog marks the service not-ready while a batch exceeds the request timeout.
"""
from __future__ import annotations

import asyncio
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import numpy as np
import torch

from .. import ops
from ..codec import CodecPool, encode_data_url, encode_data_urls, read_data_url
from ..codec.image import gpu_data_urls, gpu_jpeg_fits
from ..runtime.staging import GpuScans
from ..config import Config
from ..engine.deconvnet import DeconvNet, UnknownLayerError
from ..models.vgg16 import VGG16
from ..utils import metrics as M
from ..utils.faults import FaultInjector
from ..utils.logging import get_logger

log = get_logger("deconv_api_amd.serve")


class ServiceOverloaded(RuntimeError):
    pass


# batches above this size are trimmed to a full graph bucket (the rest waits for the next batch)
TRIM_MIN = 16


@dataclass
class _Job:
    """One request in the batcher. ``deliver(value, exc)`` hands the result back: for an HTTP
    request of this process it completes an asyncio future on the request's loop, for a request
    from a front-end process (serve/ingest.py) it writes the response to that front-end's socket."""
    layer: str
    image: np.ndarray
    deliver: Callable[[object, Optional[BaseException]], None]
    t_enq: float = field(default_factory=time.perf_counter)
    t_launch: float = 0.0
    t_gpu: float = 0.0
    t_enc: float = 0.0


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
        if self.cfg.gil_switch_us > 0:
            # many short GIL sections hop between ~6 threads per request (event loop, codec pool,
            # worker, completion); the default 5 ms switch interval turns each hop into a wait
            import sys

            sys.setswitchinterval(self.cfg.gil_switch_us / 1e6)
        dev = self.cfg.resolve_device() if runner is None else str(runner.info.device)
        self.device = torch.device(dev)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if engine is None:
            model = load_model(self.cfg)
            engine = DeconvNet(model.build(self.device, self.cfg.torch_dtype(self.device)))
        self.engine = engine
        self.graphs = None
        self.ring = None
        if self.device.type == "cuda" and runner is None:
            from ..runtime.staging import StagingRing

            # pinned staging ring + copy / compute / copy-back streams (runtime/staging.py)
            self.ring = StagingRing(self.device, max_images=max(self.cfg.max_batch, 1))
            if self.cfg.hip_graphs:
                from ..engine.graphs import GraphedDeconv

                self.graphs = GraphedDeconv(engine, self.cfg.image_size, self.cfg.filters, self.cfg.mode)
        elif runner is not None and runner.graphs is not None:
            self.graphs = runner.graphs  # the runner replays its own per-(layer, shard) graphs
        self.codec = CodecPool(self.cfg.codec_workers)
        from concurrent.futures import ThreadPoolExecutor

        self.enc_ex = ThreadPoolExecutor(max(1, self.cfg.encode_workers), thread_name_prefix="dv-encode")
        from ..codec.image import _native

        self.native_codec = bool(self.cfg.native_codec and _native() is not None)
        self.q: "queue.Queue[_Job]" = queue.Queue()
        self._carry: List[_Job] = []
        self.done_q: "queue.Queue" = queue.Queue()
        self.batches = 0
        self.images = 0
        self.last_error: Optional[str] = None
        self._stop = threading.Event()
        self.faults = FaultInjector.from_env()
        self._batch_t0: Optional[float] = None
        self.stalled = False
        self.trace: Optional[list] = None
        self._thread = threading.Thread(target=self._worker, name="dv-gpu-worker", daemon=True)
        self._thread.start()
        self._completer = threading.Thread(target=self._complete, name="dv-completion", daemon=True)
        self._completer.start()
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
        self.engine._check_layer(layer)  # raises UnknownLayerError

    def layer_names(self) -> List[str]:
        return [s.name for s in self.engine.specs[1:]]

    def submit(self, layer: str, img: np.ndarray, deliver) -> _Job:
        """Enqueue an already decoded HxWx3 uint8 image; ``deliver(value, exc)`` is called from a
        service thread with the response string (or the error). Raises at once for an unknown
        layer or a full queue."""
        self.validate_layer(layer)
        if self.q.qsize() >= self.cfg.max_queue:
            raise ServiceOverloaded("request queue is full")
        job = _Job(layer, img, deliver)
        self.q.put(job)
        M.QUEUE_DEPTH.set(self.q.qsize())
        return job

    async def deconv(self, uri: str, layer: str) -> str:
        """The reference's POST / pipeline for one request -> data URL string."""
        self.validate_layer(layer)
        if self.q.qsize() >= self.cfg.max_queue:
            raise ServiceOverloaded("request queue is full")
        loop = asyncio.get_running_loop()
        t0 = time.perf_counter()
        img = await loop.run_in_executor(self.codec.ex, read_data_url, uri)
        M.HOST_STAGE.observe(time.perf_counter() - t0, stage="decode")
        fut = loop.create_future()
        job = self.submit(layer, img, lambda v, e: _deliver(loop, _set_exc if e is not None else _set_result,
                                                            fut, e if e is not None else v))
        res = await asyncio.wait_for(fut, timeout=self.cfg.request_timeout_s)
        if self.trace is not None:  # per-request stage timestamps (tools/latency.py --trace)
            self.trace.append((t0, job.t_enq, job.t_launch, job.t_gpu, job.t_enc, time.perf_counter()))
        if isinstance(res, str):  # encoded natively, batch-wide, by the completion thread
            return res
        return await loop.run_in_executor(self.codec.ex, encode_data_url, res, self.cfg.jpeg_quality)

    def status(self) -> dict:
        st = {"device": str(self.device), "worker_alive": self._thread.is_alive() and not self.stalled,
              "stalled": self.stalled, "queue_depth": self.q.qsize(),
              "batches": self.batches, "images": self.images, "last_error": self.last_error,
              "native": ops.native.available() if self.device.type == "cuda" else None,
              "native_codec": self.native_codec,
              "graphs": [f"{l}:{b}" for l, b in self.graphs.captured] if self.graphs else None}
        if self.device.type == "cuda":
            st["gpu"] = torch.cuda.get_device_name(self.device)
        if self.runner is not None:
            st.update(world=self.runner.world, degraded=self.runner.degraded, runner_error=self.runner.last_error)
        return st

    def close(self):
        self._stop.set()
        self._thread.join(timeout=5)
        self.done_q.put(None)
        self._completer.join(timeout=5)
        self.enc_ex.shutdown(wait=True)
        self.codec.shutdown()

    # ------------------------------------------------------------------ GPU worker
    def _collect(self, wait_s: float = 0.1) -> List[_Job]:
        if self._carry:  # the tail of the previous collection, trimmed to a graph bucket (below)
            jobs, self._carry = self._carry, []
        else:
            try:
                first = self.q.get(timeout=wait_s) if wait_s > 0 else self.q.get_nowait()
            except queue.Empty:
                return []
            jobs = [first]
        # dynamic batching: wait for stragglers only while the GPU still has a batch in flight
        # (they would queue behind it anyway); an idle GPU starts the batch immediately
        busy = not self.done_q.empty() or self._batch_t0 is not None
        deadline = time.perf_counter() + (self.cfg.batch_timeout_ms / 1e3 if busy else 0.0)
        while len(jobs) < self.cfg.max_batch:
            if not busy:
                try:
                    jobs.append(self.q.get_nowait())
                    continue
                except queue.Empty:
                    break
            rem = deadline - time.perf_counter()
            if rem <= 0:
                break
            try:
                jobs.append(self.q.get(timeout=rem))
            except queue.Empty:
                break
        if self.graphs is not None and len(jobs) > TRIM_MIN:
            # a graph replays its whole batch bucket (engine/graphs.py BUCKETS): 46 images run the 64-image
            # graph. Under load run the largest bucket that is full now and carry the rest to the next batch
            from ..engine.graphs import BUCKETS

            fit = max(b for b in BUCKETS if b <= len(jobs))
            if fit < len(jobs):
                jobs, self._carry = jobs[:fit], jobs[fit:]
        return jobs

    def _worker(self):
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
            if self.ring is not None:  # all engine work of this thread on the ring's compute stream
                torch.cuda.set_stream(self.ring.compute_stream)
        last_beat = time.perf_counter()
        # multi-GPU: the batch launched last (scattered, engine enqueued on every rank) but not yet
        # gathered. It is gathered right after the NEXT batch is launched, or as soon as no batch is
        # queued, so every rank computes batch i+1 while batch i's mosaics drain (two in flight)
        inflight = None
        while not self._stop.is_set():
            jobs = self._collect(0.0 if inflight is not None else 0.1)
            if not jobs:
                if inflight is not None:
                    self._runner_finish(inflight)
                    inflight = None
                    continue
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
                t0 = time.perf_counter()
                self._batch_t0 = t0
                try:
                    for j in group:
                        j.t_launch = t0
                    if self.runner is not None:
                        b = self.runner.launch(layer, [j.image for j in group])
                        if inflight is not None:
                            self._runner_finish(inflight)
                        inflight = (b, group, layer, t0)
                        continue
                    handle = self.launch_batch(layer, [j.image for j in group])
                    self.done_q.put((handle, group, layer, t0))
                except Exception as e:  # noqa: BLE001 - delivered to every waiting request
                    self._batch_t0 = None
                    self._fail(group, e)
        if inflight is not None:
            self._runner_finish(inflight)

    def _runner_finish(self, item) -> None:
        b, group, layer, t0 = item
        try:
            self.done_q.put((("host", self.runner.finish(b)), group, layer, t0))
        except Exception as e:  # noqa: BLE001
            self._batch_t0 = None
            self._fail(group, e)

    def _complete(self):
        """Waits for each batch's copy-back in launch order, then hands the batch to the encode
        pool: several batches encode concurrently (a small batch alone cannot keep the native
        encoder's threads busy, and one serial encoder capped the service at ~2k req/s)."""
        while True:
            item = self.done_q.get()
            if item is None:
                return
            handle, group, layer, t0 = item
            try:
                mos = self.finish_batch(handle)
                if self.device.type == "cuda":
                    ops.conv.check_stream_k()
                tg = time.perf_counter()
                for j in group:
                    j.t_gpu = tg
                self.enc_ex.submit(self._encode_deliver, group, mos, layer, t0)
            except Exception as e:  # noqa: BLE001
                self._fail(group, e)
            finally:
                if self.done_q.empty():
                    self._batch_t0 = None

    def _encode_deliver(self, group, mos, layer, t0):
        try:
            if isinstance(mos, GpuScans):  # encoded on the GPU: header + scan + EOI, base64, quote
                urls = gpu_data_urls(mos.packed, mos.off, mos.H, mos.W, self.cfg.jpeg_quality, self.cfg.encode_threads)
                te = time.perf_counter()
                for j, m in zip(group, urls):
                    j.t_enc = te
                    j.deliver(m, None)
            elif self.native_codec:
                # GIL-free native JPEG + base64 + quote, in chunks of ``encode_chunk`` images over
                # the native threads (a lone request is split into restart segments); each chunk
                # is delivered as soon as it is encoded
                step = max(1, self.cfg.encode_chunk)
                for c0 in range(0, len(group), step):
                    urls = encode_data_urls(mos[c0:c0 + step], self.cfg.jpeg_quality, self.cfg.encode_threads)
                    te = time.perf_counter()
                    for j, m in zip(group[c0:c0 + step], urls):
                        j.t_enc = te
                        j.deliver(m, None)
            else:
                for j, m in zip(group, mos):
                    j.deliver(m, None)
            for j in group:
                if j.t_enc:
                    M.HOST_STAGE.observe(j.t_launch - j.t_enq, stage="queue")
                    M.HOST_STAGE.observe(j.t_gpu - j.t_launch, stage="gpu")
                    M.HOST_STAGE.observe(j.t_enc - j.t_gpu, stage="encode")
            self.batches += 1
            self.images += len(group)
            M.BATCH_SIZE.observe(len(group))
            M.ENGINE_TIME.observe(time.perf_counter() - t0, stage="batch")
            M.IMAGES.inc(len(group), layer=layer)
        except Exception as e:  # noqa: BLE001
            self._fail(group, e)

    def _fail(self, group, e):
        self.last_error = repr(e)
        log.exception("batch failed", exc_info=e)
        for j in group:
            j.deliver(None, e)

    # ------------------------------------------------------------------ batch execution
    def preprocess(self, images: List[np.ndarray]) -> torch.Tensor:
        """Resize + preprocess a batch outside the serving path (tests / tools); the worker stages
        batches through the pinned ring instead (runtime/staging.py)."""
        B, S = len(images), self.cfg.image_size
        if self.device.type == "cuda":
            from ..runtime.staging import resize_batch

            return resize_batch(images, torch.empty(B, S, S, 8, dtype=self.engine.rt.dtype, device=self.device))
        x = torch.empty(B, S, S, 8, dtype=torch.float32)
        for b, img in enumerate(images):
            x[b] = ops.preprocess_ref(ops.resize_u8_ref(img, S, S), 8, torch.float32)
        return x

    def launch_batch(self, layer: str, images: List[np.ndarray]):
        """Enqueue the batch; returns a handle for ``finish_batch`` (GPU work may still run)."""
        if self.runner is not None:
            return ("runner", self.runner.launch(layer, images))
        self.faults.on_batch()
        n = len(images)
        if self.ring is None:  # CPU
            res = self.engine.run(self.preprocess(images), layer, k=self.cfg.filters, mode=self.cfg.mode)
            return ("host", res.mosaic[:n].numpy())
        S = self.cfg.image_size
        if self.graphs is not None:  # resize straight into the graph's static input, then replay
            x = self.graphs.input(layer, n)
            st = self.ring.stage(images, x)
            res = self.graphs.replay(layer, n)
        else:
            x = torch.empty(n, S, S, 8, dtype=self.engine.rt.dtype, device=self.device)
            st = self.ring.stage(images, x)
            res = self.engine.run(x, layer, k=self.cfg.filters, mode=self.cfg.mode)
        if self.cfg.gpu_jpeg and gpu_jpeg_fits(res.mosaic.shape[2]):  # JPEG on the device: only scans cross PCIe
            return ("staged", self.ring.copy_back_jpeg(st, res.mosaic, self.cfg.jpeg_quality))
        return ("staged", self.ring.copy_back(st, res.mosaic))

    def finish_batch(self, handle) -> np.ndarray:
        if handle[0] == "host":
            return handle[1]
        if handle[0] == "runner":
            return self.runner.finish(handle[1])
        return self.ring.finish(handle[1])

    def run_batch(self, layer: str, images: List[np.ndarray]) -> np.ndarray:
        """Synchronous batch (tests / tools)."""
        return self.finish_batch(self.launch_batch(layer, images))


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
