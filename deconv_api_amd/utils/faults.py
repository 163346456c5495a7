"""Fault injection for failure-detection tests (the reference has none).

``DV_FAULT`` is a comma-separated list of ``<action>@<batch>[:<arg>][/rank=<r>]``:
  raise@3        the 3rd engine batch on this process raises RuntimeError
  hang@2:5       the 2nd batch sleeps 5 s before running (watchdog / timeout tests)
  exit@2/rank=1  rank 1 terminates (os._exit(17)) when its 2nd batch arrives (failover tests)
  exit_ready@2   terminates right after acknowledging its 2nd batch, before entering the scatter
  exit_done@2    terminates right after acknowledging that its 2nd batch is computed, before the
                 gather (the two windows the ack protocol alone cannot close, parallel/sharded.py)
  exit_octave@2  terminates when released into its 2nd DeepDream octave (the other ranks are
                 then inside that octave's collectives)
Batches are counted per process from 1.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import List, Optional


class InjectedFault(RuntimeError):
    pass


@dataclass
class Fault:
    action: str
    batch: int
    arg: float = 0.0
    rank: Optional[int] = None


def parse(spec: str) -> List[Fault]:
    out = []
    for item in filter(None, (s.strip() for s in spec.split(","))):
        rank = None
        if "/rank=" in item:
            item, r = item.split("/rank=")
            rank = int(r)
        action, rest = item.split("@")
        arg = 0.0
        if ":" in rest:
            rest, a = rest.split(":")
            arg = float(a)
        if action not in ("raise", "hang", "exit", "exit_ready", "exit_done", "exit_octave"):
            raise ValueError(f"unknown fault action {action!r}")
        out.append(Fault(action, int(rest), arg, rank))
    return out


class FaultInjector:
    def __init__(self, faults: List[Fault], rank: int = 0):
        self.faults = faults
        self.rank = rank
        self.count = 0

    @classmethod
    def from_env(cls, rank: int = 0) -> "FaultInjector":
        return cls(parse(os.environ.get("DV_FAULT", "")), rank)

    def on_batch(self) -> None:
        self.count += 1
        for f in self.faults:
            if f.batch != self.count or (f.rank is not None and f.rank != self.rank):
                continue
            if f.action == "raise":
                raise InjectedFault(f"injected fault at batch {self.count}")
            if f.action == "hang":
                time.sleep(f.arg)
            if f.action == "exit":
                os._exit(17)

    def at(self, point: str, batch: int) -> None:
        """Named fault point of batch ``batch`` (``exit_<point>@<batch>``)."""
        for f in self.faults:
            if f.action == f"exit_{point}" and f.batch == batch and (f.rank is None or f.rank == self.rank):
                os._exit(17)
