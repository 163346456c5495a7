#!/usr/bin/env python
"""DeepDream benchmarks (BASELINE configs 3 and 5; extensions beyond the reference).

  config 3: python bench_dream.py --model inception_v3 --batch 64 --size 299 --octaves 4 --steps 20
  config 5: python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16   (1 GPU)
            python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
                bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 32 --dtype fp16   (8 GPUs:
            batch 32 gives each rank 4-16 (tile, image) units per step; at batch 8 a rank holds 1-4 and runs
            latency-bound, profiles/dream_c5_r4_virtual_ranks.txt; a rank's units run as 2 chunks on two
            forked streams, each chunk's pack all-gather issued behind it: profiles/dream_c5_r5_local_chunks.txt)

One timed run = the whole octave loop (octaves x steps gradient-ascent iterations + octave
resizes/detail re-injection) over the batch. Prints ONE JSON line (rank 0). Synthetic uint8
images, seeded random-init weights, bf16 (default) or fp16 compute.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

import torch

from deconv_api_amd import ops
import deconv_api_amd.engine.deepdream as D
from deconv_api_amd.engine.deepdream import (RESNET_LAYERS, DeepDream, DreamSettings, TiledDeepDream,
                                             inception_preprocess)
from deconv_api_amd.parallel import dist as pdist


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="inception_v3", choices=["inception_v3", "resnet50"])
    ap.add_argument("--batch", type=int, default=64, help="images (per GPU for untiled; total for tiled)")
    ap.add_argument("--size", type=int, default=299)
    ap.add_argument("--octaves", type=int, default=4)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--tile", type=int, default=0, help="tile size (0 = untiled, hipGraph per octave)")
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"],
                    help="16-bit storage / MFMA dtype (BASELINE config 5 is quoted in fp16)")
    ap.add_argument("--virtual-world", type=int, default=0,
                    help="tiled only: time ONE rank's share of a W-rank dream on this GPU (no collective; "
                         "readiness sizing for config 5, not a dream result)")
    ap.add_argument("--virtual-rank", type=int, default=0)
    ap.add_argument("--xgmi-gbs", type=float, default=300.0,
                    help="--virtual-world: assumed all-gather receive bandwidth per GPU (GB/s) for the exposed-"
                         "communication estimate (8 x MI355X RCCL all-gather over xGMI; not measured here)")
    a = ap.parse_args(argv)
    if a.virtual_world:
        return virtual_rank(a)

    info = pdist.init()
    dev = info.device
    ops.native.load()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    if a.model == "inception_v3":
        from deconv_api_amd.models.inception_v3 import InceptionV3

        net = InceptionV3(0).build(dev, dt)
        s = DreamSettings(octaves=a.octaves, iterations=a.steps)
    else:
        from deconv_api_amd.models.resnet50 import ResNet50

        net = ResNet50(0).build(dev, dt)
        s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=a.octaves, iterations=a.steps)
    if a.tile:
        dd = TiledDeepDream(net, s, tile=a.tile, info=info, use_graphs=not a.no_graphs)
    else:
        dd = DeepDream(net, s, use_graphs=not a.no_graphs)
    g = torch.Generator(device=dev).manual_seed(7 + info.rank * (0 if a.tile else 1))
    img = torch.randint(0, 256, (a.batch, a.size, a.size, 3), dtype=torch.uint8, device=dev, generator=g)
    x = inception_preprocess(img)
    t0 = time.perf_counter()
    for _ in range(a.warmup):
        dd.run(x)
    torch.cuda.synchronize()
    print(f"[rank {info.rank}] warmup (incl. graph capture) {time.perf_counter() - t0:.1f}s", file=sys.stderr)
    pdist.barrier(info)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.runs):
        out = dd.run(x)
    host_s = (time.perf_counter() - t0) / a.runs  # host enqueue time per run (graph launches)
    torch.cuda.synchronize()
    pdist.barrier(info)
    el = pdist.all_reduce_max(time.perf_counter() - t0, info)
    per_run = el / a.runs
    imgs = a.batch * (1 if a.tile else info.world)
    if info.is_main:
        print(json.dumps({
            "metric": f"DeepDream images/sec ({a.model}, {a.octaves} octaves x {a.steps} steps)",
            "value": round(imgs / per_run, 3), "unit": "images/s", "n_gpus": info.world,
            "s_per_dream_batch": round(per_run, 3), "host_enqueue_s": round(host_s, 3), "runs": a.runs, "warmup": a.warmup,
            "higher_is_better": True, "scaling": "strong" if a.tile else "weak", "dtype": a.dtype,
            "data": "synthetic uint8 images, seeded random-init weights", "hip_graphs": not a.no_graphs,
            "finite": bool(torch.isfinite(out).all()),
            "sub_batch_streams": dd.split if dd.fused else 1,
            **(_tile_info(dd) if a.tile else {}),
            "config": {"model": a.model, "batch": a.batch, "image_size": a.size, "tile": a.tile,
                       "parallelism": f"{'tiles' if a.tile else 'dp'}{info.world}"},
        }), flush=True)
    pdist.shutdown()


def virtual_rank(a) -> dict:
    """Per-rank step time of a W-rank tiled dream, measured on one GPU: rank r's plan (its
    (tile, image) units dealt round-robin, its pack slot, tile_update over W packs) runs every
    octave without the all-gather. Prints per octave: units on this rank, ms per gradient step,
    and the bytes one step's pack all-gather moves into every rank (W x pack)."""
    from types import SimpleNamespace

    dev = torch.device("cuda", 0)
    ops.native.load()
    dt = torch.float16 if a.dtype == "fp16" else torch.bfloat16
    assert a.tile, "--virtual-world needs --tile"
    if a.model == "inception_v3":
        from deconv_api_amd.models.inception_v3 import InceptionV3

        net = InceptionV3(0).build(dev, dt)
        s = DreamSettings(octaves=a.octaves, iterations=a.steps)
    else:
        from deconv_api_amd.models.resnet50 import ResNet50

        net = ResNet50(0).build(dev, dt)
        s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=a.octaves, iterations=a.steps)
    info = SimpleNamespace(world=a.virtual_world, rank=a.virtual_rank, backend="none", device=dev)
    dd = TiledDeepDream(net, s, tile=a.tile, info=info, use_graphs=not a.no_graphs)
    dd.virtual = True
    g = torch.Generator(device=dev).manual_seed(7)
    img = torch.randint(0, 256, (a.batch, a.size, a.size, 3), dtype=torch.uint8, device=dev, generator=g)
    x = inception_preprocess(img)
    for _ in range(a.warmup):
        for _o in dd.octave_steps(x):
            pass
    torch.cuda.synchronize()
    per_oct = {}
    for _ in range(a.runs):
        evs = [torch.cuda.Event(enable_timing=True)]
        evs[0].record()
        for _o in dd.octave_steps(x):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            evs.append(e)
        torch.cuda.synchronize()
        for i in range(len(evs) - 1):
            per_oct.setdefault(i, []).append(evs[i].elapsed_time(evs[i + 1]))
    shapes = dd.octave_shapes(a.size, a.size)
    rows = []
    for i, hw in enumerate(shapes):
        st = dd._tgraphs[(a.batch, hw[0], hw[1])]
        ms = sorted(per_oct[i])[len(per_oct[i]) // 2]
        step_ms = ms / a.steps
        gather_bytes = int(st.packs.numel() * st.packs.element_size())
        # exposed communication estimate at --xgmi-gbs of all-gather receive bandwidth per GPU: one
        # all-gather after the step (chunks 1) exposes all of it; with C chunks the last chunk's gather
        # is exposed and the others hide behind the next chunk's network (ms per step)
        comm = gather_bytes * (a.virtual_world - 1) / a.virtual_world / (a.xgmi_gbs * 1e9) * 1e3
        C = st.C
        # chunks in waves of S concurrent streams: the last wave's gathers are exposed, earlier waves'
        # hide behind the following waves' networks
        S = max(1, min(D.TILE_CHUNK_STREAMS, C))
        waves = -(-C // S)
        exposed_c = comm / waves + (waves - 1) / waves * max(0.0, comm - step_ms)
        rows.append({"octave": list(hw), "tiles": st.ntiles, "units_this_rank": st.mine, "units_all": st.plan.shape[0],
                     "ms_per_step": round(step_ms, 3), "ms_octave": round(ms, 2),
                     "allgather_bytes_per_step": gather_bytes, "comm_ms_per_step_est": round(comm, 3),
                     "exposed_ms_per_step_est": {"chunks_1": round(comm, 3), f"chunks_{C}_streams_{S}": round(exposed_c, 3)}})
    out = {"virtual_world": a.virtual_world, "virtual_rank": a.virtual_rank, "model": a.model, "batch": a.batch,
           "size": a.size, "tile": a.tile, "dtype": a.dtype, "octaves": rows,
           "ms_per_dream_batch_compute": round(sum(r["ms_octave"] for r in rows), 1),
           "xgmi_gbs_assumed": a.xgmi_gbs,
           "note": "one rank's share, no collective: compute-only lower bound of a W-rank dream batch; comm / "
                   "exposed figures are estimates at the assumed all-gather bandwidth, not measurements"}
    print(json.dumps(out), flush=True)
    return out


def _tile_info(dd) -> dict:
    """how the tiled octaves ran: whole-octave graphs (collectives captured inside when the
    collective path is on) vs per-step graphs with eager collectives"""
    sts = [st for st in dd._tgraphs.values() if hasattr(st, "graph")]
    return {"tile_octave_graphs": sum(st.graph is not None for st in sts),
            "tile_step_graph_octaves": sum(st.step_graph is not None for st in sts),
            "tile_collective": any(dd._collective(st) for st in sts)}


if __name__ == "__main__":
    main()
