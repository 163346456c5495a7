"""Does the RCCL collective stream share a hardware queue with the compute stream? (torchrun, any world)

HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default) round-robin; two streams on one
queue execute in order, so an async all-gather would wait behind (and delay) the next step's compute.
For each candidate compute stream: a ~2 ms spin on it, then an async all-gather issued from an idle
stream; the collective is independent when it completes while the spin still runs. Prints one JSON line.

    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 tools/queue_alias_probe.py
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def probe(comp, idle, x, y, spin=4_000_000):
    torch.cuda.synchronize()
    with torch.cuda.stream(comp):
        torch.cuda._sleep(spin)
        end = torch.cuda.Event()
        end.record(comp)
    with torch.cuda.stream(idle):
        work = dist.all_gather_into_tensor(y, x, async_op=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 5:
        w = work.is_completed()
        e = end.query()
        if w and not e:
            torch.cuda.synchronize()
            return "independent"
        if e:
            torch.cuda.synchronize()
            return "serialized"
    return "timeout"


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.ones(1 << 16, device=dev)
    y = torch.empty(dist.get_world_size() << 16, device=dev)
    dist.all_gather_into_tensor(y, x)
    torch.cuda.synchronize()
    idle = torch.cuda.Stream(dev)
    res = {"null": probe(torch.cuda.current_stream(dev), idle, x, y)}
    for i in range(6):
        res[f"pool{i}"] = probe(torch.cuda.Stream(dev), idle, x, y)
    for i in range(3):
        res[f"high{i}"] = probe(torch.cuda.Stream(dev, priority=-1), idle, x, y)
    res["rank"] = dist.get_rank()
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
