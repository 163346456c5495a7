"""Data-parallel deconvnet serving across ranks, with failover that re-forms the group over the
surviving GPUs (the reference is one blocking worker, app/main.py:46 and
Dockerfile:15).

Planes:
  * control (parallel/elastic.py): the job's TCPStore. Rank 0 posts a numbered command stream;
    each collective is entered only after rank 0 has seen every member acknowledge the command
    and released a "go" key. Followers publish heartbeats; a missing ack plus a stale heartbeat
    marks a peer dead;
  * data (RCCL over xGMI; Gloo on CPU): rank 0 resizes the whole batch on its GPU from one staged
    upload (runtime/staging.py) into uint8 224x224x3 (150 KB/image) and ``scatter``s each rank
    only its shard; every rank preprocesses its shard and runs the engine from a captured hipGraph
    per (layer, shard bucket); the uint8 mosaics are ``gather``ed to rank 0 only (1/N of the bytes
    of an all-gather; rank 0 is the only rank that answers HTTP).

Two batches in flight. A batch is two commands, ``run`` (scatter + engine) and ``gather``; rank 0
issues batch i+1's ``run`` before batch i's ``gather`` whenever i+1 is queued (the service's worker
does that, serve/service.py), so on every rank the engine work of i+1 is on the compute stream
while i's mosaics drain:
  rank 0:   run(i):    cmd -> wait ready(all) -> go1 -> scatter -> engine(i) -> copy to slot i%2
            gather(i): cmd -> wait done(all) -> go2 -> gather on a side stream that waits only for
                       batch i's event -> D2H into the staging ring's pinned block
  follower: run(i):    wait cmd -> ready -> wait go1 -> scatter -> engine(i) -> event(i)
            gather(i): wait cmd -> event(i).synchronize() (not the whole stream) -> done -> wait go2
                       -> gather on a side stream behind event(i)

Collectives with a dead peer: every collective is issued ``async_op=True`` and polled under a
deadline together with the heartbeats (rank 0) or the reform announcement (followers), so a rank
that dies between its ack and the collective (the window the ack protocol alone cannot close) is
detected instead of blocking rank 0 in RCCL until the process-group timeout. Re-forming then
ABORTS the communicator (``_abort_process_group``) before building the new group: destroying an
RCCL group with an operation pending on a dead peer can block (parallel/elastic.py).

Failure: rank 0 publishes ``reform`` on every key a survivor can be waiting on, the survivors and
rank 0 rebuild the group over the survivors (renumbered, new store prefix), and every batch whose
commands ran on the old group is recomputed on the new world. A local error on rank 0 (bad input,
kernel check) fails only that batch; it never degrades the group.

``/deepdream`` across ranks runs as one ``dream`` command (broadcast of the images, every rank
builds its octave generator) followed by one ``dream_oct`` command per octave. Each octave's work
(its per-step pack all-gathers included, eager or captured in the octave graph) is polled to
completion under the same deadlines as a collective: rank 0 checks the followers' heartbeats, a
follower checks for a re-form announcement; eager collectives inside the tiled step are polled
one by one (``TiledDeepDream.coll_wait``). A peer lost mid-dream re-forms the group and the dream
restarts on the survivors (same seed: same rolls, same result up to rounding). The command lock is
a FIFO lock released between octaves, so deconv batches (``POST /``) interleave with a long dream
instead of waiting for all of it.

What stays uncovered: a follower that hangs inside a kernel while still heartbeating (its thread
keeps beating) is only caught by the collective deadline (``ack_timeout``), not by staleness.
"""
from __future__ import annotations

import contextlib
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..codec.image import gpu_jpeg_fits
from ..utils.faults import FaultInjector
from ..utils.logging import get_logger
from .dist import DistInfo, shard_sizes
from .elastic import Control, PeerLost

log = get_logger("deconv_api_amd.sharded")


class FairLock:
    """Reentrant lock granted in arrival order (tickets). ``threading.RLock`` lets a thread that
    releases and re-acquires in a loop (the dream, once per octave) starve a waiting one (the deconv
    worker); here the waiter that arrived first gets the lock next."""

    def __init__(self):
        self._cv = threading.Condition(threading.Lock())
        self._owner: Optional[int] = None
        self._count = 0
        self._next = 0
        self._serving = 0

    def acquire(self) -> bool:
        me = threading.get_ident()
        with self._cv:
            if self._owner == me:
                self._count += 1
                return True
            ticket = self._next
            self._next += 1
            while self._serving != ticket or self._owner is not None:
                self._cv.wait()
            self._owner, self._count = me, 1
            return True

    def release(self) -> None:
        with self._cv:
            if self._owner != threading.get_ident():
                raise RuntimeError("FairLock released by a thread that does not hold it")
            self._count -= 1
            if self._count == 0:
                self._owner = None
                self._serving += 1
                self._cv.notify_all()

    def __enter__(self):
        return self.acquire()

    def __exit__(self, *exc):
        self.release()


class _EventWork:
    """A recorded GPU event polled like an async collective's work object (``_await``)."""

    def __init__(self, ev: torch.cuda.Event):
        self.ev = ev

    def is_completed(self) -> bool:
        return self.ev.query()

    def wait(self) -> None:
        self.ev.synchronize()


class _DreamRestart(Exception):
    """The group was re-formed while a dream was between octaves: restart it on the new group."""


@dataclass
class Batch:
    """A batch whose ``run`` command was issued; ``finish`` gathers it."""
    layer: str
    images: List[np.ndarray]
    epoch: int
    bid: int = 0
    mos: Optional[torch.Tensor] = None  # this rank's mosaics (its slot buffer)
    ev: Optional[torch.cuda.Event] = None  # engine done on the compute stream
    host: Optional[tuple] = None  # world 1: the copy-back handle
    staged: Optional[object] = None  # rank 0's staging-ring record (GPU)
    n: int = 0
    t: Dict[str, float] = field(default_factory=dict)


class ShardedRunner:
    def __init__(self, engine, info: DistInfo, image_size: int = 224, k: int = 4, mode: str = "all",
                 use_graphs: bool = True, hb_timeout: float = 3.0, ack_timeout: float = 600.0,
                 poll_s: float = 0.0001, cfg=None):
        """``cfg`` (serve/config.Config): what the /deepdream engines are built from on every rank
        (seed, weight files, tile size); the default config when None."""
        self.engine = engine
        self.cfg = cfg
        # one command (its store keys and collectives) at a time: the deconv worker and the
        # /deepdream worker both drive the group (FIFO: a dream releases it between octaves)
        self._cmd_lock = FairLock()
        self._did = 0  # dream ids
        self._dreams: Dict[int, tuple] = {}  # follower: dream id -> (octave generator, octaves)
        self.dream_restarts = 0
        self._oct_count = 0  # dream octaves run by this process (fault injection)
        self._dream_tiled: Dict[tuple, object] = {}
        self._dream_nets: Dict[str, object] = {}
        self.info = info
        self.S = image_size
        self.k = k
        self.mode = mode
        self.batches = 0
        self.reforms = 0
        self.poll_s = poll_s
        self.ack_timeout = ack_timeout
        self.last_error: Optional[str] = None
        self.faults = FaultInjector.from_env(info.rank)
        self.ctl = Control(info, hb_timeout=hb_timeout, ack_timeout=ack_timeout) if info.world > 1 else None
        self.graphs = None
        cuda = info.device.type == "cuda"
        if use_graphs and cuda:
            from ..engine.graphs import GraphedDeconv

            self.graphs = GraphedDeconv(engine, image_size, k, mode)
        self.ring = None
        if cuda and info.rank == 0:
            from ..runtime.staging import StagingRing

            self.ring = StagingRing(info.device)
        # mosaics of the (at most two) batches in flight: the graph-owned output is overwritten by
        # the next replay, so each batch's mosaics are copied into its own slot on the compute
        # stream; the gather runs on ``comm_stream`` behind that batch's event only
        self.slots: List[Optional[torch.Tensor]] = [None, None]
        # a batch's input path (upload + resize + scatter) runs on its own stream, never behind the
        # previous batch's engine work on the compute stream nor behind a gather on comm_stream; both
        # side streams are probed onto hardware queues of their own (runtime/streams.py)
        self.comm_stream = self.in_stream = None
        if cuda:
            from ..runtime.streams import independent_stream

            cur = torch.cuda.current_stream(info.device)
            self.comm_stream = independent_stream(info.device, [cur])
            self.in_stream = independent_stream(info.device, [cur, self.comm_stream])
        self._bid = 0

    @property
    def world(self) -> int:
        return self.info.world

    @property
    def degraded(self) -> bool:
        """True once the group lost a member (it keeps serving on the survivors)."""
        return self.reforms > 0

    # ----------------------------------------------------------------- shared compute
    def _resize_u8(self, images: List[np.ndarray], npad: int):
        """rank 0: all images -> uint8 [npad, S, S, 3] (zero rows pad to npad) on this rank's
        device; returns (tensor, staging record or None)."""
        S = self.S
        if self.ring is not None:
            out = torch.zeros(npad, S, S, 3, dtype=torch.uint8, device=self.info.device)
            return out, self.ring.stage(images, out)
        out = torch.zeros(npad, S, S, 3, dtype=torch.uint8)
        for b, img in enumerate(images):
            out[b] = torch.from_numpy(ops.resize_u8_ref(img, S, S))
        return out, None

    def _preprocess(self, u8: torch.Tensor) -> torch.Tensor:
        if u8.is_cuda:
            rt = getattr(self.engine, "rt", None)  # (test doubles have no runtime: bf16)
            x = torch.empty(*u8.shape[:3], 8, dtype=rt.dtype if rt is not None else torch.bfloat16, device=u8.device)
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
        u8, _ = self._resize_u8(images, len(images))
        return self._engine(self._preprocess(u8), layer)

    def _keep(self, bid: int, mos: torch.Tensor) -> tuple:
        """Copy this batch's mosaics into its slot (stream order) and record its done event."""
        if not mos.is_cuda:
            return mos.clone(), None
        s = bid % 2
        if self.slots[s] is None or self.slots[s].shape != mos.shape:
            self.slots[s] = torch.empty_like(mos)
        self.slots[s].copy_(mos)
        ev = torch.cuda.Event()
        ev.record()
        return self.slots[s], ev

    def _await(self, work, what: str, follower: bool = False) -> None:
        """Poll an async collective under the ack deadline. Rank 0 checks the followers'
        heartbeats; a follower checks for a reform announcement (rank 0 saw a peer die)."""
        t0 = last = time.time()
        sleep = self.poll_s
        while True:
            try:
                if work.is_completed():
                    work.wait()  # re-raises a transport error (e.g. Gloo: peer closed its socket)
                    return
            except RuntimeError as e:
                if isinstance(work, _EventWork):
                    # a local GPU fault (this rank's own kernels, e.g. an illegal access surfacing in
                    # hipEventQuery) is NOT a peer loss: degrading the group and restarting the dream
                    # on a faulted context would hide it; it propagates as the local error it is
                    raise
                if follower:
                    raise PeerLost([]) from e
                raise PeerLost(self._which_dead()) from e
            now = time.time()
            if now - last > 0.02:  # store round trips only every 20 ms; the work poll is local
                last = now
                if follower:
                    if self.ctl.reform_announced():
                        raise PeerLost([])
                else:
                    dead = self.ctl.stale()
                    if dead:
                        raise PeerLost(dead)
                if now - t0 > self.ack_timeout:
                    raise PeerLost([] if follower else list(self.ctl.members[1:]))
            time.sleep(sleep)
            sleep = min(sleep * 2, 0.002)

    def _which_dead(self) -> List[int]:
        """rank 0 after a transport error: the error arrives before the dead peer's heartbeat has
        gone stale, so wait up to two heartbeat timeouts for it to (every follower if none does)."""
        t_end = time.time() + 2 * self.ctl.hb_timeout
        while time.time() < t_end:
            dead = self.ctl.stale()
            if dead:
                return dead
            time.sleep(0.05)
        return list(self.ctl.members[1:])

    # ----------------------------------------------------------------- rank 0
    def run(self, layer: str, images: List[np.ndarray]) -> np.ndarray:
        return self.finish(self.launch(layer, images))

    def launch(self, layer: str, images: List[np.ndarray]) -> Batch:
        """rank 0: scatter the batch and enqueue its engine work on every rank; ``finish`` gathers
        it. Another batch may be launched before this one is finished (two in flight)."""
        assert self.info.rank == 0
        with self._cmd_lock:
            return self._launch(layer, images)

    def _launch(self, layer: str, images: List[np.ndarray]) -> Batch:
        self.batches += 1
        while True:
            b = Batch(layer, images, self.ctl.epoch if self.ctl else 0, self._bid, n=len(images))
            self._bid += 1
            if self.world == 1:
                self.faults.on_batch()
                u8, st = self._resize_u8(images, len(images))
                mos = self._engine(self._preprocess(u8), layer)
                b.host = self._copy_back(st, mos, len(images))
                return b
            try:
                self._run_cmd(b)
                return b
            except PeerLost as e:
                self._reform(e)

    def finish(self, b: Batch) -> np.ndarray:
        """rank 0: gather batch ``b``'s mosaics (recomputed on the survivors if the group was
        re-formed since its launch) -> uint8 [n, 2S, 2S, 3] on the host."""
        with self._cmd_lock:
            return self._finish(b)

    def _finish(self, b: Batch) -> np.ndarray:
        while True:
            if b.host is not None:
                return self._host(b.host)
            if b.epoch != self.ctl.epoch:  # launched on a group that no longer exists
                b = self._launch(b.layer, b.images)
                continue
            try:
                self._gather_cmd(b)
            except PeerLost as e:
                self._reform(e)

    def _reform(self, e: PeerLost) -> None:
        self.last_error = repr(e)
        log.error("peer lost, re-forming over the survivors", extra={"fields": {"dead": e.dead}})
        self.ctl.reform(e.dead)
        self.reforms += 1
        self._after_reform()

    def _after_reform(self) -> None:
        self.slots = [None, None]
        self._reset_dream_state()

    def _reset_dream_state(self) -> None:
        self._dreams.clear()
        for dd in self._dream_tiled.values():  # unit plans / packs / graphs were for the old world
            dd._tgraphs.clear()
            dd._plans.clear()

    # ----------------------------------------------------------------- /deepdream across ranks
    def _dream_engine(self, model: str, octaves: int, steps: int):
        from ..config import Config
        from ..serve.dream_service import tiled_engine

        return tiled_engine(self._dream_tiled, self._dream_nets, self.cfg or Config(), model, octaves, steps,
                            self.info.device, info=self.info)

    def _dream_local(self, dd, x_u8: torch.Tensor, seed: int) -> torch.Tensor:
        dd.gen.manual_seed(seed)  # identical rolls on every rank
        dd.coll_wait = None
        return dd.dream_u8(x_u8)

    def _dream_octaves(self, dd, x_u8: torch.Tensor, seed: int, follower: bool):
        """This rank's dream, one octave per ``next``: every eager collective of the tiled step is
        polled under the failure deadlines; yields each octave's (enqueued) image."""
        from ..engine.deepdream import inception_preprocess

        dd.gen.manual_seed(seed)  # identical rolls on every rank
        dd.coll_wait = lambda w: self._await(w, "dream collective", follower)
        yield from dd.octave_steps(inception_preprocess(x_u8))

    def _octave(self, run, follower: bool) -> torch.Tensor:
        """Advance a dream by one octave and poll its completion (GPU: an event recorded behind the
        octave's work, which holds its captured all-gathers) under the deadlines."""
        self._oct_count += 1
        img = next(run)
        if img.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
            self._await(_EventWork(ev), "dream octave", follower)
        return img

    def dream(self, imgs: torch.Tensor, model: str, octaves: int, steps: int) -> np.ndarray:
        """rank 0: DeepDream of u8 [n, H, W, 3] tiled across every rank -> u8 [n, H, W, 3]. The
        images are broadcast (RCCL); each rank runs its share of the (tile, image) units and the
        per-step pack all-gathers inside the tiled engine assemble every step on every rank. One
        command per octave; the command lock is released between octaves. A peer lost at any point
        re-forms the group and restarts the dream on the survivors."""
        assert self.info.rank == 0
        seed = (self.cfg.seed if self.cfg is not None else 0)
        while True:
            if self.world == 1:
                with self._cmd_lock:
                    if self.world == 1:
                        dd = self._dream_engine(model, octaves, steps)
                        return self._dream_local(dd, imgs.to(self.info.device), seed).cpu().numpy()
                continue
            try:
                return self._dream_cmds(imgs, model, octaves, steps, seed)
            except _DreamRestart:
                self.dream_restarts += 1

    def _dream_cmds(self, imgs: torch.Tensor, model: str, octaves: int, steps: int, seed: int) -> np.ndarray:
        from ..engine.deepdream import inception_deprocess

        ctl = self.ctl
        n, H, W, _ = imgs.shape
        with self._cmd_lock:
            if self.world == 1:
                raise _DreamRestart()
            epoch = ctl.epoch
            did = self._did
            self._did += 1
            try:
                seq = ctl.post_cmd({"op": "dream", "did": did, "model": model, "octaves": octaves, "steps": steps,
                                    "n": n, "H": H, "W": W, "seed": seed})
                dd = self._dream_engine(model, octaves, steps)  # overlaps the followers' acks
                x = imgs.to(self.info.device).contiguous()
                ctl.wait_acks("ready", seq)
                ctl.go("go1", seq)
                self._await(dist.broadcast(x, src=0, async_op=True), "broadcast")
                run = self._dream_octaves(dd, x, seed, follower=False)
            except PeerLost as e:
                self._reform(e)
                raise _DreamRestart() from e
        img = None
        for o in range(octaves):
            with self._cmd_lock:  # released between octaves: deconv batches interleave
                if ctl.epoch != epoch:  # another command re-formed the group meanwhile
                    self._reset_dream_state()  # (done by its _reform already; idempotent)
                    raise _DreamRestart()
                try:
                    seq = ctl.post_cmd({"op": "dream_oct", "did": did, "o": o})
                    ctl.wait_acks("ready", seq)
                    ctl.go("go1", seq)
                    img = self._octave(run, follower=False)
                    ctl.wait_acks("done", seq)
                except PeerLost as e:
                    self._reform(e)
                    raise _DreamRestart() from e
        return inception_deprocess(img).cpu().numpy()

    def _run_cmd(self, b: Batch) -> None:
        n = len(b.images)
        per = shard_sizes(n, self.world)[0]
        ctl = self.ctl
        seq = ctl.post_cmd({"op": "run", "layer": b.layer, "n": n, "per": per, "b": b.bid})
        # upload + resize + scatter on the side stream: on the compute stream they would queue behind
        # the previous batch's engine work, and the host (polling the scatter below) could enqueue
        # this batch's engine only after that finished - an idle GPU gap per batch with two in flight
        with self._side():
            u8, b.staged = self._resize_u8(b.images, per * self.world)  # overlaps the followers' acks
            ctl.wait_acks("ready", seq)
            ctl.go("go1", seq)
            shard = torch.empty(per, self.S, self.S, 3, dtype=torch.uint8, device=u8.device)
            work = dist.scatter(shard, scatter_list=list(u8.chunk(self.world)), src=0, async_op=True)
        self._await(work, "scatter")
        shard = self._to_compute(shard)
        self.faults.on_batch()
        b.mos, b.ev = self._keep(b.bid, self._engine(self._preprocess(shard), b.layer).contiguous())

    def _side(self):
        """Stream context for a batch's input path (resize + scatter): the side stream on a GPU."""
        return torch.cuda.stream(self.in_stream) if self.in_stream is not None else contextlib.nullcontext()

    def _to_compute(self, t: torch.Tensor) -> torch.Tensor:
        """Hand a tensor produced on the side stream (its collective polled complete) to the compute
        stream: stream order for the kernels, allocator lifetime for its block."""
        if self.in_stream is not None and t.is_cuda:
            cur = torch.cuda.current_stream(t.device)
            cur.wait_stream(self.in_stream)
            t.record_stream(cur)
        return t

    def _gather_cmd(self, b: Batch) -> None:
        ctl = self.ctl
        seq = ctl.post_cmd({"op": "gather", "b": b.bid})
        ctl.wait_acks("done", seq)
        ctl.go("go2", seq)
        if self.comm_stream is not None:
            self.comm_stream.wait_event(b.ev)
            with torch.cuda.stream(self.comm_stream):
                # the receive buffers come from comm_stream's pool: a compute-stream block may still
                # be in use by the NEXT batch's queued engine work (two in flight), which the gather
                # (ordered only behind THIS batch's event) would overwrite
                parts = [torch.empty_like(b.mos) for _ in range(self.world)]
                work = dist.gather(b.mos, gather_list=parts, dst=0, async_op=True)
                self._await(work, "gather")
                full = torch.cat(parts)
                ev = torch.cuda.Event()
                ev.record()
            torch.cuda.current_stream().wait_event(ev)
            full.record_stream(torch.cuda.current_stream())
        else:
            parts = [torch.empty_like(b.mos) for _ in range(self.world)]
            self._await(dist.gather(b.mos, gather_list=parts, dst=0, async_op=True), "gather")
            full = torch.cat(parts)
        b.host = self._copy_back(b.staged, full, b.n)

    def _copy_back(self, st, mos: torch.Tensor, n: int) -> tuple:
        if not mos.is_cuda:
            return ("host", mos[:n].numpy())
        if st is not None and self.ring is not None:  # reuse the staging ring's slot + stream
            st.n = n
            if (self.cfg is None or self.cfg.gpu_jpeg) and gpu_jpeg_fits(mos.shape[2]):  # only scans cross PCIe
                q = self.cfg.jpeg_quality if self.cfg is not None else 95
                return ("staged", self.ring.copy_back_jpeg(st, mos, q))
            return ("staged", self.ring.copy_back(st, mos))
        host = torch.empty((n, *mos.shape[1:]), dtype=mos.dtype, pin_memory=True)
        host.copy_(mos[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return ("event", ev, host)

    def _host(self, h: tuple) -> np.ndarray:
        if h[0] == "host":
            return h[1]
        if h[0] == "staged":
            return self.ring.finish(h[1])
        h[1].synchronize()
        return h[2].numpy()

    def ping(self) -> bool:
        """Idle liveness check: re-forms the group if a follower stopped heartbeating. Under the
        command lock (a dream between octaves may hold the group: its own _await and this must not
        re-form concurrently) and through ``_reform``, so ``_after_reform`` drops every per-world
        state (dream unit plans, packs, octave graphs with captured collectives)."""
        if self.world == 1 or self.ctl is None:
            return True
        with self._cmd_lock:
            if self.world == 1:
                return True
            dead = self.ctl.stale()
            if dead:
                self._reform(PeerLost(dead))
                return False
        return True

    def stop(self):
        if self.ctl is not None and self.info.rank == 0:
            if self.world > 1:
                self.ctl.post_cmd({"op": "stop"})
            self.ctl.close()

    # ----------------------------------------------------------------- followers
    def follow(self) -> int:
        """Serve rank 0's command stream until 'stop' (or until dropped from the group). Returns
        the number of batches gathered."""
        assert self.info.rank != 0
        ctl = self.ctl
        done = 0
        runs = 0
        pending: Dict[int, tuple] = {}  # batch id -> (mosaics slot, event)
        dev = self.info.device
        while True:
            seq, msg = ctl.wait_cmd()
            op = msg["op"]
            if op == "stop":
                ctl.close()
                return done
            try:
                if op == "reform":
                    raise PeerLost([])
                if op == "run":
                    runs += 1
                    ctl.ack("ready", seq)
                    self.faults.at("ready", runs)  # fault window: acked, then gone before the scatter
                    self._go(ctl, "go1", seq)
                    with self._side():  # not queued behind the previous batch's engine work (_run_cmd)
                        shard = torch.empty(msg["per"], self.S, self.S, 3, dtype=torch.uint8, device=dev)
                        work = dist.scatter(shard, scatter_list=None, src=0, async_op=True)
                    self._await(work, "scatter", True)
                    shard = self._to_compute(shard)
                    self.faults.on_batch()
                    mos = self._engine(self._preprocess(shard), msg["layer"]).contiguous()
                    pending[msg["b"]] = self._keep(msg["b"], mos)
                    continue
                if op == "dream":
                    ctl.ack("ready", seq)
                    self._go(ctl, "go1", seq)
                    x = torch.empty(msg["n"], msg["H"], msg["W"], 3, dtype=torch.uint8, device=dev)
                    self._await(dist.broadcast(x, src=0, async_op=True), "broadcast", True)
                    dd = self._dream_engine(msg["model"], msg["octaves"], msg["steps"])
                    self._dreams.clear()  # one dream at a time (a restarted one replaces it)
                    self._dreams[msg["did"]] = (self._dream_octaves(dd, x, msg["seed"], True), msg["octaves"])
                    continue
                if op == "dream_oct":
                    run, octaves = self._dreams[msg["did"]]
                    ctl.ack("ready", seq)
                    self._go(ctl, "go1", seq)
                    self.faults.at("octave", self._oct_count + 1)  # fault window: inside a dream
                    self._octave(run, follower=True)
                    ctl.ack("done", seq)
                    if msg["o"] + 1 == octaves:
                        del self._dreams[msg["did"]]
                    continue
                if op == "gather":
                    mos, ev = pending.pop(msg["b"])
                    if ev is not None:
                        ev.synchronize()  # this batch's engine work only, not the whole stream
                    ctl.ack("done", seq)
                    self.faults.at("done", runs)  # fault window: acked, then gone before the gather
                    self._go(ctl, "go2", seq)
                    if self.comm_stream is not None:
                        self.comm_stream.wait_event(ev)
                        with torch.cuda.stream(self.comm_stream):
                            self._await(dist.gather(mos, gather_list=None, dst=0, async_op=True), "gather", True)
                    else:
                        self._await(dist.gather(mos, gather_list=None, dst=0, async_op=True), "gather", True)
                    done += 1
                    continue
                raise RuntimeError(f"unknown command {msg!r}")
            except PeerLost:
                r = msg if op == "reform" else ctl.wait_reform()
                pending.clear()
                self._after_reform()
                if not ctl.follow_reform(r):
                    return done

    @staticmethod
    def _go(ctl: Control, kind: str, seq: int) -> None:
        r = ctl.wait_go(kind, seq)
        if r is not None:  # reform announced instead of go
            raise PeerLost([])
