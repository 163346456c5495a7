"""Control plane of the data-parallel service: per-batch commands, acks and go-signals through the
job's TCPStore, follower heartbeats, and re-forming the process group over the survivors
(the reference has a static health check only, app/main.py:41-43).

Why a store and not collectives: a rank blocked in a collective cannot notice that a third rank
died, and an RCCL collective with a dead peer never returns (the watchdog aborts the process).
Store waits are polled with deadlines and heartbeat checks, so every survivor learns about a
failure at its next wait, and collectives are only entered after rank 0 released them.

Identity: every process keeps its launch rank (``orig``); ``members`` lists the launch ranks of
the current group in rank order (rank 0 always survives: it serves HTTP, and the store lives
with the job). Keys: ``dv/<epoch>/<kind>/<seq>[/<orig>]``, heartbeats ``dv/hb/<orig>``.
"""
from __future__ import annotations

import datetime
import json
import os
import threading
import time
from typing import List, Optional, Tuple

import torch.distributed as dist

from ..utils.logging import get_logger

log = get_logger("deconv_api_amd.elastic")


class PeerLost(RuntimeError):
    def __init__(self, dead: List[int]):
        super().__init__(f"peer(s) lost: {dead}")
        self.dead = dead


def _client() -> "dist.TCPStore":
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ["MASTER_PORT"])
    return dist.TCPStore(host, port, is_master=False, timeout=datetime.timedelta(seconds=60))


class Control:
    def __init__(self, info, hb_timeout: float = 3.0, ack_timeout: float = 600.0, hb_interval: float = 0.25):
        self.info = info
        self.orig = info.rank
        self.members = list(range(info.world))
        self.epoch = 0
        self.seq = 0
        self.backend = info.backend
        self.hb_timeout = hb_timeout
        # rebuild a process group even for a world of 1 (tools/rccl_selftest.py --reform: the
        # abort + re-init path on a real RCCL group with the one GPU a test box has)
        self.single_pg = False
        self.ack_timeout = ack_timeout
        # keep the default store (hosted by rank 0 in env:// init) alive past destroy_process_group
        self._keep = dist.distributed_c10d._get_default_store()
        self.store = _client()
        self._stop = threading.Event()
        self._hb: Optional[threading.Thread] = None
        if self.orig != 0:
            self.store.set(f"dv/hb/{self.orig}", repr(time.time()))
            self._hb = threading.Thread(target=self._beat, args=(hb_interval,), name="dv-heartbeat", daemon=True)
            self._hb.start()
        else:  # start-up barrier: every follower is heartbeating before rank 0 judges staleness
            self.store.wait([f"dv/hb/{m}" for m in self.members[1:]], datetime.timedelta(seconds=600))

    # ------------------------------------------------------------------ keys / heartbeats
    def _k(self, kind: str, seq: int, who: Optional[int] = None) -> str:
        key = f"dv/{self.epoch}/{kind}/{seq}"
        return key if who is None else f"{key}/{who}"

    def _beat(self, interval: float) -> None:
        st = _client()  # own connection: the main thread may be blocked in a store wait
        while not self._stop.is_set():
            try:
                st.set(f"dv/hb/{self.orig}", repr(time.time()))
            except Exception:  # noqa: BLE001 - store gone: rank 0 exited
                return
            self._stop.wait(interval)

    def stale(self, among: Optional[List[int]] = None) -> List[int]:
        """Members (launch ranks, not rank 0) whose heartbeat is older than ``hb_timeout``."""
        now = time.time()
        dead = []
        for m in (among if among is not None else self.members[1:]):
            key = f"dv/hb/{m}"
            if not self.store.check([key]) or now - float(self.store.get(key)) > self.hb_timeout:
                dead.append(m)
        return dead

    # ------------------------------------------------------------------ rank 0
    def post_cmd(self, msg: dict) -> int:
        self.seq += 1
        self.store.set(self._k("cmd", self.seq), json.dumps(msg))
        if self.seq > 3:  # keys of finished batches
            for kind in ("cmd", "go1", "go2"):
                self.store.delete_key(self._k(kind, self.seq - 3))
            for m in self.members[1:]:
                for kind in ("ready", "done"):
                    self.store.delete_key(self._k(kind, self.seq - 3, m))
        return self.seq

    def wait_acks(self, kind: str, seq: int) -> None:
        """Wait until every follower posted ``kind`` for ``seq``; PeerLost if one whose ack is
        missing stopped heartbeating (or the ack deadline passed)."""
        pending = list(self.members[1:])
        t0 = time.time()
        sleep = 0.0002
        while pending:
            pending = [m for m in pending if not self.store.check([self._k(kind, seq, m)])]
            if not pending:
                return
            dead = self.stale(pending)
            if dead or time.time() - t0 > self.ack_timeout:
                raise PeerLost(dead or pending)
            time.sleep(sleep)
            sleep = min(sleep * 2, 0.001)

    def go(self, kind: str, seq: int) -> None:
        self.store.set(self._k(kind, seq), json.dumps({"op": "go"}))

    def reform(self, dead: List[int]) -> None:
        """rank 0: drop ``dead``, announce the new membership on every key a survivor can be
        waiting on, and rebuild the process group over the survivors."""
        members = [m for m in self.members if m not in dead]
        msg = {"op": "reform", "epoch": self.epoch + 1, "members": members}
        for key in (self._k("cmd", self.seq + 1), self._k("go1", self.seq), self._k("go2", self.seq)):
            self.store.set(key, json.dumps(msg))
        log.warning("re-forming the group", extra={"fields": {"members": members, "epoch": msg["epoch"]}})
        self._rebuild(msg["epoch"], members)

    # ------------------------------------------------------------------ followers
    def _wait_key(self, key: str) -> dict:
        while True:
            try:
                self.store.wait([key], datetime.timedelta(seconds=1))
                return json.loads(self.store.get(key))
            except RuntimeError as e:  # timeout: keep waiting (a dead rank 0 kills the store)
                if "timeout" not in str(e).lower() and "wait" not in str(e).lower():
                    raise

    def wait_cmd(self) -> Tuple[int, dict]:
        self.seq += 1
        return self.seq, self._wait_key(self._k("cmd", self.seq))

    def ack(self, kind: str, seq: int) -> None:
        self.store.set(self._k(kind, seq, self.orig), "1")

    def wait_go(self, kind: str, seq: int) -> Optional[dict]:
        """None once rank 0 released the step; the reform message if it announced one instead."""
        msg = self._wait_key(self._k(kind, seq))
        return None if msg.get("op") == "go" else msg

    def reform_announced(self) -> bool:
        """True once rank 0 announced a re-form after this rank's current command (polled by a
        follower waiting in a collective: a third rank may have died)."""
        key = self._k("cmd", self.seq + 1)
        return bool(self.store.check([key])) and json.loads(self.store.get(key)).get("op") == "reform"

    def wait_reform(self) -> dict:
        """A follower that saw its collective fail: rank 0's re-form announcement (it follows the
        current command). Anything else means this rank lost sync with the group."""
        msg = self._wait_key(self._k("cmd", self.seq + 1))
        if msg.get("op") != "reform":
            raise RuntimeError(f"collective failed but rank 0 moved on: {msg!r}")
        return msg

    def follow_reform(self, msg: dict) -> bool:
        """Join the re-formed group; False if this rank is no longer a member."""
        if self.orig not in msg["members"]:
            self.close()
            return False
        self._rebuild(msg["epoch"], msg["members"])
        return True

    # ------------------------------------------------------------------ group rebuild
    def _rebuild(self, epoch: int, members: List[int]) -> None:
        if dist.is_initialized():
            if self.backend == "nccl":
                # abort first: destroying an RCCL communicator with an operation still pending on
                # a dead peer can block; abort tears the communicator down without waiting for it
                dist.distributed_c10d._abort_process_group()
                try:
                    dist.destroy_process_group()
                except Exception:  # noqa: BLE001 - already torn down by the abort
                    pass
            else:
                dist.destroy_process_group()
        self.epoch = epoch
        self.members = list(members)
        self.seq = 0
        rank, world = members.index(self.orig), len(members)
        if world > 1 or self.single_pg:
            kw = dict(backend=self.backend, store=dist.PrefixStore(f"dvpg{epoch}", self.store), rank=rank,
                      world_size=world, timeout=datetime.timedelta(seconds=600))
            if self.backend == "nccl":
                kw["device_id"] = self.info.device
            dist.init_process_group(**kw)
        self.info.rank = rank
        self.info.world = world
        self.info.ctrl_group = None

    def close(self) -> None:
        self._stop.set()
