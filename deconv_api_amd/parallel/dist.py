"""One process per GPU over torch.distributed (backend "nccl" == RCCL on ROCm, xGMI links).

Data-parallel deconvnet serving/benchmarking (BASELINE config 4):
  * weights are created (or loaded) on rank 0 and broadcast once over RCCL, bucketed into a
    few large flat messages (xGMI is point-to-point: fewer, larger collectives);
  * each rank processes its own shard of the request batch (shards are bucket-padded to one
    fixed per-rank size so every collective and graph has a static shape);
  * the uint8 output mosaics are all-gathered with ``all_gather_into_tensor`` (one collective,
    602 KB per image) so any rank can encode/serve the whole batch;
  * the serving control plane (commands, acks, heartbeats, re-forming the group over survivors)
    runs over the job's TCPStore (parallel/elastic.py), off the RCCL rings.
The reference is single-process (Dockerfile:15, app/main.py:46); this layer is new.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    ctrl_group: Optional[object] = None

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init(backend: Optional[str] = None, device_type: Optional[str] = None, timeout_s: int = 600) -> DistInfo:
    """Initialise from torchrun env vars (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*). Single process
    without those vars returns a world of 1 and creates no process group."""
    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    # torchrun env (even with one rank) or DV_FORCE_PG=1: a real process group, so a 1-rank run
    # exercises the RCCL collectives; a plain `python x.py` creates none
    force = os.environ.get("DV_FORCE_PG") == "1" or "TORCHELASTIC_RUN_ID" in os.environ
    if world == 1 and not (force and "MASTER_PORT" in os.environ):
        return DistInfo(0, 1, 0, device, "none")
    backend = backend or ("nccl" if device_type == "cuda" else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
    if backend == "nccl":
        kw["device_id"] = device
    dist.init_process_group(**kw)
    return DistInfo(rank, world, local, device, backend, None)


def shutdown() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def barrier(info: DistInfo) -> None:
    if info.backend != "none":
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def broadcast_state(sd: Dict[str, torch.Tensor], info: DistInfo, src: int = 0,
                    bucket_bytes: int = 256 << 20) -> Dict[str, torch.Tensor]:
    """Broadcast a state dict from ``src`` as flat fp32 buckets (shapes are known on every rank
    because every rank builds the same architecture). Returns tensors on CPU."""
    if info.backend == "none":
        return sd
    names = sorted(sd.keys())
    out: Dict[str, torch.Tensor] = {}
    dev = info.device
    i = 0
    while i < len(names):
        group: List[str] = []
        size = 0
        while i < len(names) and (not group or size + sd[names[i]].numel() * 4 <= bucket_bytes):
            group.append(names[i])
            size += sd[names[i]].numel() * 4
            i += 1
        if info.rank == src:
            flat = torch.cat([sd[n].reshape(-1).float() for n in group]).to(dev)
        else:
            flat = torch.empty(size // 4, dtype=torch.float32, device=dev)
        dist.broadcast(flat, src)
        off = 0
        flat = flat.cpu()
        for n in group:
            k = sd[n].numel()
            out[n] = flat[off:off + k].view_as(sd[n]).clone()
            off += k
    return out


def all_gather_rows(x: torch.Tensor, info: DistInfo, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[b, ...] per rank -> [world*b, ...] on every rank (rank-major order)."""
    if info.backend == "none":
        return x
    if out is None:
        out = torch.empty((info.world * x.shape[0], *x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x.contiguous())
    return out


def all_reduce_max(v: float, info: DistInfo) -> float:
    if info.backend == "none":
        return v
    t = torch.tensor([v], dtype=torch.float64, device=info.device if info.backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_sizes(total: int, world: int, bucket: int = 1) -> List[int]:
    """Per-rank shard sizes of a ragged batch, each padded up to the same bucket-multiple size
    (static shapes for collectives/graphs). Returns [per_rank_padded] * world and the real
    counts via ``shard_counts``."""
    per = -(-total // world)
    per = -(-per // bucket) * bucket
    return [per] * world


def shard_counts(total: int, world: int) -> List[int]:
    per = -(-total // world)
    return [max(0, min(per, total - r * per)) for r in range(world)]



def _spin_vs_gather(info: DistInfo, spinner: Optional[torch.cuda.Stream], x, y, idle, spin_cycles: int,
                    timeout_s: float) -> bool:
    """One probe round (collective): ``spinner`` (this rank only, None elsewhere) runs a ~2 ms spin,
    every rank issues an async all-gather from an idle stream. True when, on the spinning rank, the
    gather completed while the spin still ran (the two are on different hardware queues)."""
    dev = info.device
    torch.cuda.synchronize(dev)
    end = None
    if spinner is not None:
        with torch.cuda.stream(spinner):
            torch.cuda._sleep(spin_cycles)
            end = torch.cuda.Event()
            end.record(spinner)
    with torch.cuda.stream(idle):
        work = dist.all_gather_into_tensor(y, x, async_op=True)
    ok = True
    if end is not None:
        import time

        ok, t0 = False, time.perf_counter()
        while time.perf_counter() - t0 < timeout_s:
            w, e = work.is_completed(), end.query()
            if w and not e:
                ok = True
                break
            if e:
                break
    torch.cuda.synchronize(dev)
    return ok


def pick_compute_stream(info: DistInfo, tries: int = 6, spin_cycles: int = 4_000_000,
                        timeout_s: float = 10.0):
    """This rank's compute stream for steps whose collectives run async beside the next step's compute
    (bench.py's all-gather). HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues round-robin, and
    RCCL's internal stream can share one with the compute stream: the gather then waits for, and
    delays, the compute queued before it. Measured on MI355X (tools/queue_alias_probe.py, 1-rank RCCL
    group): the NULL stream and 2 of 6 pool streams were serialized with the all-gather; every
    high-priority stream overlapped it, but a high-priority compute stream cost 3-4 % at N=1
    (profiles/bench_c2_r6_stream_prio_ab.txt), so a normal-priority stream is probed instead.

    Probed rank by rank (collective; every rank calls it): only the probing rank spins, so the
    all-gather's completion answers for that rank alone. Returns ``(stream, independent)``; the
    current stream and None without an RCCL group."""
    dev = info.device
    if info.backend != "nccl":
        return torch.cuda.current_stream(dev) if dev.type == "cuda" else None, None
    x = torch.ones(1 << 14, device=dev)
    y = torch.empty(info.world << 14, device=dev)
    idle = torch.cuda.Stream(dev)
    _spin_vs_gather(info, None, x, y, idle, spin_cycles, timeout_s)  # communicator / kernels warm
    chosen, independent = torch.cuda.current_stream(dev), False
    for r in range(info.world):
        cand = chosen
        for _ in range(max(1, tries)):
            me = r == info.rank
            ok = _spin_vs_gather(info, cand if me else None, x, y, idle, spin_cycles, timeout_s)
            flag = torch.tensor([0.0 if (ok or not me) else 1.0], device=dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            if float(flag.item()) == 0.0:
                if me:
                    chosen, independent = cand, True
                break
            if me:
                cand = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    return chosen, independent
