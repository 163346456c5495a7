"""RCCL self-test of the data-parallel code paths, for a 1..N-rank torchrun launch on GPUs:

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \\
        --master-port 29531 tools/rccl_selftest.py

Runs parallel/dist.broadcast_state (bucketed weight broadcast), all_gather_rows, all_reduce_max,
and the serving data plane's scatter (uint8 shards) + gather (uint8 mosaics) through the process
group the launcher created (backend "nccl" == RCCL), checks the results, prints one JSON line."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deconv_api_amd.models.vgg16 import VGG16  # noqa: E402
from deconv_api_amd.parallel import dist as pdist  # noqa: E402


def main():
    info = pdist.init()
    assert info.backend == "nccl", info.backend
    ref = VGG16.random(0, include_top=False).state_dict()
    mine = ref if info.rank == 0 else VGG16.random(99, include_top=False).state_dict()
    sd = pdist.broadcast_state(mine, info, bucket_bytes=16 << 20)
    bcast_ok = all(torch.equal(sd[k], ref[k]) for k in ref)
    x = torch.full((2, 5), float(info.rank), device=info.device)
    g = pdist.all_gather_rows(x, info)
    gather_ok = g[:, 0].tolist() == [float(r) for r in range(info.world) for _ in range(2)]
    mx = pdist.all_reduce_max(float(info.rank) + 0.5, info)
    per = 3
    src = torch.arange(info.world * per * 12, dtype=torch.int64).to(torch.uint8).view(info.world * per, 2, 2, 3)
    src = src.to(info.device)
    shard = torch.empty(per, 2, 2, 3, dtype=torch.uint8, device=info.device)
    dist.scatter(shard, scatter_list=list(src.chunk(info.world)) if info.rank == 0 else None, src=0)
    scatter_ok = torch.equal(shard, src[info.rank * per:(info.rank + 1) * per])
    parts = [torch.empty_like(shard) for _ in range(info.world)] if info.rank == 0 else None
    dist.gather(shard, gather_list=parts, dst=0)
    gath_ok = torch.equal(torch.cat(parts), src) if info.rank == 0 else True
    torch.cuda.synchronize()
    out = {"backend": info.backend, "world": info.world, "broadcast_state": bcast_ok,
           "all_gather_rows": gather_ok, "all_reduce_max": mx == info.world - 0.5,
           "scatter": scatter_ok, "gather": gath_ok}
    if "--reform" in sys.argv:
        out.update(reform(info))
    if info.rank == 0:
        print(json.dumps(out), flush=True)
    pdist.shutdown()


def reform(info):
    """The serving failover's group rebuild on RCCL: an async collective is in flight, the
    communicator is ABORTED (parallel/elastic.py:_rebuild) and a new group is built over the same
    membership under a new store prefix; collectives then run on the new group."""
    from deconv_api_amd.parallel.elastic import Control

    ctl = Control(info, hb_timeout=5.0)
    ctl.single_pg = True
    t = torch.ones(1 << 20, device=info.device)
    work = dist.all_reduce(t, async_op=True)
    ctl._rebuild(ctl.epoch + 1, list(ctl.members))
    del work
    y = torch.full((4,), 2.0, device=info.device)
    dist.all_reduce(y)
    torch.cuda.synchronize()
    ok = bool(torch.all(y == 2.0 * info.world)) and dist.is_initialized() and dist.get_backend() == "nccl"
    ctl.close()
    return {"reform_epoch": ctl.epoch, "reform_all_reduce": ok}


if __name__ == "__main__":
    main()
