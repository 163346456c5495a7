#!/usr/bin/env python
"""Flagship benchmark: VGG16 block5_conv3 deconvnet, 256 synthetic 224x224 images per GPU, bf16.

One timed step = what the reference's ``POST /`` computes for a batch of images (app/main.py:
45-78), minus only the host JPEG encode: preprocess (uint8 -> caffe bf16 NHWC), VGG16 forward to
the target with fused pool+switch, per-image top-4 filter selection, 4 deconv chains per image
to the input (unpool fused or split), 2x2 mosaic + deprocess to uint8, and with N > 1 an RCCL
all-gather of every rank's uint8 mosaics over xGMI (weak scaling: 256 img/GPU). The all-gather
of step i runs asynchronously on RCCL's stream and overlaps step i+1's compute (double-buffered
output); the clock stops only after the last gather completed on every rank.

Request latency: every step's mosaics are copied back to pinned host memory on a copy stream
(overlapping the next step's compute, as the service does); ``p50_req_latency_ms`` is the median
over steps of (step start on the compute stream -> its mosaics on the host), hipEvent-timed.

Run: ``python bench.py [--gpus N --steps K --warmup W]``; for N > 1 under
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N``
(also with N = 1: torchrun env -> a real 1-rank RCCL group, the collective path runs).
``--profile`` re-runs the same command under ``rocprofv3 --kernel-trace`` (before any GPU call)
and prints a per-kernel table (tools/kstats.py); ``--profile pmc`` adds one counter pass.
Rank 0 prints ONE JSON line. Weights: seeded random-init VGG16 (no network for ImageNet
weights); data: synthetic uint8 images. ``--device cpu --tiny`` is a functional rehearsal of the
same code path (gloo, scaled model) used by the CPU test-suite.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

from deconv_api_amd import ops
from deconv_api_amd.codec.image import encode_gpu
from deconv_api_amd.engine.deconvnet import DeconvNet
from deconv_api_amd.models.vgg16 import VGG16, vgg16_specs
from deconv_api_amd.parallel import dist as pdist
from deconv_api_amd.runtime.streams import copy_stream as copy_stream_for

# DV_BENCH_JPEG=1: each step also JPEG-encodes its mosaics on the GPU (csrc/jpeg_gpu.hip, what the
# service does) and copies back only the scans (~10x fewer PCIe bytes). Sizing that copy needs the
# step's scan total on the host, so it is issued from inside the NEXT step's forward, right before
# block3_conv1 (the engine's layer hook): by then the GPU has finished the step and still has the
# next step's first layers queued. Raw mosaics are copied right after their step is enqueued (the
# copy costs ~0.2 % of the step: --no-copyback 7016 vs 6999 img/s, profiles/bench_c2_r3_copy_ab.txt).
JPEG = os.environ.get("DV_BENCH_JPEG", "0") == "1"
COPY_AT = os.environ.get("DV_BENCH_COPY_AT", "block3_conv1" if JPEG else "")

# the reference's implied end-to-end rate for layer=block5_conv3 is ~0.03-0.04 img/s
# (CPU, one request at a time; a lower bound on its cost). We divide by the favourable 0.04.
REF_IMG_PER_S = 0.04
METRIC = "images/sec, VGG16 deconv 224px (block5_conv3 deconvnet, top-4 mosaic)"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU")
    ap.add_argument("--layer", default="block5_conv3")
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--tiny", action="store_true", help="scaled VGG16 at 32px (CPU rehearsal only)")
    ap.add_argument("--breakdown", action="store_true", help="per-phase timing to stderr (extra syncs)")
    ap.add_argument("--no-copyback", action="store_true",
                    help="DIAGNOSTIC ONLY (not a benchmark number): skip the mosaics' copy to the host, to price it")
    ap.add_argument("--emulate-gather-world", type=int, default=0,
                    help="DIAGNOSTIC ONLY (not a benchmark number): every step also copies (N-1) x the step's "
                         "mosaics device-to-device on a side stream, overlapping the next step, i.e. the HBM "
                         "writes and CU time an N-rank all-gather of the mosaics costs each rank")
    ap.add_argument("--emulate-rccl-world", type=int, default=0,
                    help="DIAGNOSTIC ONLY (not a benchmark number): model an N-rank all-gather of the mosaics on a "
                         "side stream behind every step as RCCL runs it: --rccl-channels workgroups (CUs) busy "
                         "for (N-1) x mosaic bytes / --rccl-gbs, writing those bytes to HBM (csrc/misc.hip:"
                         "paced_copy_kernel), overlapping the next step's compute")
    ap.add_argument("--rccl-channels", type=int, default=32, help="--emulate-rccl-world: CUs the collective holds")
    ap.add_argument("--rccl-gbs", type=float, default=300.0,
                    help="--emulate-rccl-world: all-gather receive bandwidth per GPU (GB/s, xGMI ring)")
    ap.add_argument("--profile", nargs="?", const="trace", default=None, choices=["trace", "pmc"],
                    help="re-run under rocprofv3 and print a per-kernel table (trace) [+ PMC pass]")
    return ap.parse_args(argv)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class _Sync:
    def __init__(self, dev):
        self.cuda = dev.type == "cuda"

    def __call__(self):
        if self.cuda:
            torch.cuda.synchronize()


PMC_PASS = "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS"


def profile(argv, mode: str) -> int:
    """Re-launch this benchmark under rocprofv3 as a CHILD process (nothing in this process has
    touched the GPU), then summarize the kernel trace (and a PMC pass for ``pmc``)."""
    import os
    import subprocess
    import tempfile

    here = os.path.dirname(os.path.abspath(__file__))
    args_in = list(argv if argv is not None else sys.argv[1:])
    child, skip = [], False
    for a in args_in:  # drop --profile [mode] / --profile=mode so the child never re-profiles itself
        if skip:
            skip = False
            if a in ("trace", "pmc"):
                continue
        if a == "--profile":
            skip = True
            continue
        if a.startswith("--profile="):
            continue
        child.append(a)
    out = tempfile.mkdtemp(prefix="dv_prof_", dir=os.environ.get("TMPDIR", "/tmp"))
    cmd = ["rocprofv3", "--kernel-trace", "-d", out, "-o", "bench", "--", sys.executable,
           os.path.join(here, "bench.py"), *child]
    rc = subprocess.call(cmd)
    if rc != 0:
        return rc
    db = next((os.path.join(d, f) for d, _, fs in os.walk(out) for f in fs if f.endswith(".db")), None)
    if db is not None:
        subprocess.call([sys.executable, os.path.join(here, "tools", "kstats.py"), db, "--top", "30",
                         "--last-frac", "0.6"])
    if mode == "pmc":
        pdir = out + "_pmc"
        rc = subprocess.call(["rocprofv3", "--pmc", *PMC_PASS.split(), "-d", pdir, "-o", "bench", "--",
                              sys.executable, os.path.join(here, "bench.py"), *child, "--steps", "2", "--warmup", "1"])
        if rc == 0:
            subprocess.call([sys.executable, os.path.join(here, "tools", "pmc_summary.py"), pdir])
    return rc


def main(argv=None):
    args = parse(argv)
    if args.profile and os.environ.get("DV_PROFILE_CHILD") != "1":
        os.environ["DV_PROFILE_CHILD"] = "1"  # inherited by the rocprofv3 child: never recurse
        raise SystemExit(profile(argv, args.profile))
    info = pdist.init(device_type=args.device)
    if info.world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={info.world}; using WORLD_SIZE")
    dev = info.device
    sync = _Sync(dev)
    if dev.type == "cuda":
        ops.native.load()
    elif not args.tiny:
        raise SystemExit("bench.py on CPU is a rehearsal: pass --tiny")
    specs = vgg16_specs(width_div=8, image_size=32, fc=64, classes=10) if args.tiny else None
    S = 32 if args.tiny else 224
    dtype = torch.bfloat16 if dev.type == "cuda" else torch.float32

    # ---- weights: built on rank 0, broadcast once over RCCL ----
    t0 = time.time()
    model = VGG16.random(args.seed if info.is_main else args.seed + 12345, specs=specs)
    if info.backend != "none":  # any real process group (incl. a 1-rank RCCL group under torchrun)
        sd = pdist.broadcast_state(model.state_dict(), info)
        model = VGG16.from_state_dict(sd, specs=specs)
    eng = DeconvNet(model.build(dev, dtype))
    log(f"[rank {info.rank}] weights ready in {time.time() - t0:.1f}s ({model.num_params() / 1e6:.1f}M params)")

    # with RCCL: every step's work on a stream whose hardware queue is not the all-gather's, so step i's
    # async gather overlaps step i+1's compute instead of queueing with it (parallel/dist.py)
    comp, overlap = pdist.pick_compute_stream(info) if dev.type == "cuda" else (None, None)
    if comp is not None:
        torch.cuda.set_stream(comp)
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(1000 + info.rank)
    images = torch.randint(0, 256, (B, S, S, 3), dtype=torch.uint8, device=dev, generator=g)
    xbuf = torch.empty(B, S, S, 8, dtype=dtype, device=dev)
    gathered = [torch.empty(info.world * B, 2 * S, 2 * S, 3, dtype=torch.uint8, device=dev) for _ in range(2)]
    pending = [None, None]
    cuda = dev.type == "cuda"
    # copy-back of every step's mosaics on its own stream into a pinned double buffer (an
    # ordinary stream by default; runtime/streams.py:copy_stream)
    copy_stream = copy_stream_for(dev) if cuda else None
    host = [torch.empty(B, 2 * S, 2 * S, 3, dtype=torch.uint8, pin_memory=cuda) for _ in range(2)]
    back_done = [None, None]
    lat = []  # (start event, copy-back end event) per timed step

    # the copy-back of step i's mosaics is issued from step i+1's forward (COPY_AT hook) or, if the
    # target comes before that layer, right after step i+1 is enqueued; every copy still lands
    # inside the timed region (drain)
    deferred = [None]

    off_host = [torch.empty(B + 1, dtype=torch.int64, pin_memory=cuda) for _ in range(2)]
    scans_host = [None, None]
    # JPEG mode with N > 1: step i's scans are all-gathered from step i+1's hook, padded to the
    # largest scan total over the ranks (an all-reduce issued at step i, read on the host at the
    # hook), i.e. ~10x fewer xGMI bytes than gathering the raw mosaics
    mx_host = [torch.empty(1, dtype=torch.int64, pin_memory=cuda) for _ in range(2)]
    jpeg_bytes = []  # scan bytes per image, per step
    gpend = [None, None]
    gscans = [None, None]
    goff = [torch.empty(info.world * (B + 1), dtype=torch.int64, device=dev) for _ in range(2)]

    def issue_gather(slot):
        if gpend[slot] is None:
            return
        packed, off, mx_ev = gpend[slot]
        gpend[slot] = None
        if pending[slot] is not None:
            pending[slot].wait()  # the gather that last used this slot's buffers (step i-2)
        mx_ev.synchronize()
        cap = -(-int(mx_host[slot][0]) // (1 << 16)) * (1 << 16)  # 64 KiB granules: stable sizes
        if gscans[slot] is None or gscans[slot].numel() < info.world * cap:
            gscans[slot] = torch.empty(info.world * cap, dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(goff[slot], off, async_op=False)
        pending[slot] = dist.all_gather_into_tensor(gscans[slot][: info.world * cap], packed[:cap], async_op=True)

    def issue_copy():
        if deferred[0] is None:
            return
        if args.no_copyback:
            deferred[0] = None
            return
        slot, mosaic, ev0 = deferred[0]
        deferred[0] = None
        if back_done[slot] is not None:
            back_done[slot].synchronize()  # host slot free again (its step i-2 copy landed)
        if JPEG:  # mosaic = (device scans, event of the offsets' copy into off_host[slot])
            issue_gather(slot)
            packed, off_ev = mosaic
            off_ev.synchronize()  # step i's scan sizes (long done: the GPU is in step i+1)
            total = int(off_host[slot][-1])
            jpeg_bytes.append(total / B)
            if scans_host[slot] is None or scans_host[slot].numel() < total:
                scans_host[slot] = torch.empty(max(total, 1) * 5 // 4, dtype=torch.uint8, pin_memory=True)
            with torch.cuda.stream(copy_stream):
                scans_host[slot][:total].copy_(packed[:total], non_blocking=True)
                back_done[slot] = torch.cuda.Event(enable_timing=True)
                back_done[slot].record()
            if ev0 is not None:
                lat.append((ev0, back_done[slot]))
            return
        ready = torch.cuda.Event()
        ready.record()
        copy_stream.wait_event(ready)
        mosaic.record_stream(copy_stream)
        with torch.cuda.stream(copy_stream):
            host[slot].copy_(mosaic, non_blocking=True)
            back_done[slot] = torch.cuda.Event(enable_timing=True)
            back_done[slot].record()
        if ev0 is not None:
            lat.append((ev0, back_done[slot]))

    emu_n = max(0, args.emulate_gather_world - 1)
    emu_stream = torch.cuda.Stream(dev) if (cuda and emu_n) else None
    emu_dst = torch.empty(emu_n * B, 2 * S, 2 * S, 3, dtype=torch.uint8, device=dev) if emu_stream else None

    def emulate_gather(mosaic):
        """(N-1) mosaic-sized D2D copies on a side stream behind this step (what an N-rank all-gather
        writes into each rank's HBM, and the copy kernels' CUs), overlapping the next step."""
        ready = torch.cuda.Event()
        ready.record()
        emu_stream.wait_event(ready)
        mosaic.record_stream(emu_stream)
        with torch.cuda.stream(emu_stream):
            for r in range(emu_n):
                emu_dst[r * B:(r + 1) * B].copy_(mosaic)

    rccl_n = max(0, args.emulate_rccl_world - 1)
    rccl_stream = torch.cuda.Stream(dev) if (cuda and rccl_n) else None
    rccl_dst = torch.empty(rccl_n * B, 2 * S, 2 * S, 3, dtype=torch.uint8, device=dev) if rccl_stream else None

    def emulate_rccl(mosaic):
        """The all-gather's receive side as RCCL runs it: --rccl-channels CUs busy for the link time of
        (N-1) mosaic-sized blocks, those bytes written to HBM (a paced copy), behind this step."""
        ready = torch.cuda.Event()
        ready.record()
        rccl_stream.wait_event(ready)
        mosaic.record_stream(rccl_stream)
        with torch.cuda.stream(rccl_stream):
            ops.native.lib().paced_copy(mosaic.contiguous(), rccl_dst, args.rccl_channels, args.rccl_gbs)

    def step(i, ev0=None):
        ops.resize_preprocess(images, xbuf)
        hook = (COPY_AT, issue_copy) if cuda and COPY_AT else None
        res = eng.run(xbuf, args.layer, k=args.k, hook=hook)
        if cuda:
            issue_copy()  # no-op when the hook already issued step i-1's copy
        if emu_stream is not None:
            emulate_gather(res.mosaic)
        if rccl_stream is not None:
            emulate_rccl(res.mosaic)
        slot = i % 2
        if info.backend != "none" and not (JPEG and cuda):
            if pending[slot] is not None:
                pending[slot].wait()  # the gather that last used this buffer (step i-2)
            pending[slot] = dist.all_gather_into_tensor(gathered[slot], res.mosaic.contiguous(), async_op=True)
        if cuda:
            out = res.mosaic
            if JPEG:
                packed, off = encode_gpu(res.mosaic)
                done = torch.cuda.Event()
                done.record()
                copy_stream.wait_event(done)
                packed.record_stream(copy_stream)
                with torch.cuda.stream(copy_stream):
                    off_host[slot].copy_(off, non_blocking=True)
                    off_ev = torch.cuda.Event()
                    off_ev.record()
                out = (packed, off_ev)
                if info.backend != "none":  # the largest scan total over the ranks (for the gather)
                    mx = off[-1:].clone()
                    work = dist.all_reduce(mx, op=dist.ReduceOp.MAX, async_op=True)
                    with torch.cuda.stream(copy_stream):
                        work.wait()  # the copy stream (not the compute stream) waits for the collective
                        mx_host[slot].copy_(mx, non_blocking=True)
                        mx_ev = torch.cuda.Event()
                        mx_ev.record()
                    gpend[slot] = (packed, off, mx_ev)
            deferred[0] = (slot, out, ev0)
            if not COPY_AT:
                issue_copy()
        else:
            host[slot].copy_(res.mosaic)
        return res

    def drain():
        if cuda:
            issue_copy()  # the last step's copy-back
        for s in (0, 1):
            if pending[s] is not None:
                pending[s].wait()
                pending[s] = None

    for i in range(args.warmup):
        step(i)
    drain()
    sync()

    if args.breakdown and info.is_main:
        _breakdown(eng, images, xbuf, args, sync)

    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if cuda else None
    pdist.barrier(info)
    sync()
    t_start = time.perf_counter()
    if cuda:
        evs[0].record()
    host_steps = []
    for i in range(args.steps):
        ts = time.perf_counter()
        res = step(i, evs[i] if cuda else None)
        if cuda:
            evs[i + 1].record()
        host_steps.append(time.perf_counter() - ts)
    drain()
    if cuda:
        copy_stream.synchronize()
    if emu_stream is not None:
        emu_stream.synchronize()
    sync()
    pdist.barrier(info)
    sync()
    elapsed = time.perf_counter() - t_start
    if cuda:  # outside the clock: no stream-K tile of the timed steps was finished without its partner
        ops.conv.check_stream_k()
    elapsed = pdist.all_reduce_max(elapsed, info)
    if cuda:
        per_step = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps))
    else:
        per_step = sorted(1e3 * t for t in host_steps)
    p50 = pdist.all_reduce_max(per_step[len(per_step) // 2], info)
    req = sorted(a.elapsed_time(b) for a, b in lat) if cuda else []
    if not req:  # CPU, or --no-copyback (nothing delivered): the batch latency stands in
        req = per_step
    p50_req = pdist.all_reduce_max(req[len(req) // 2], info)

    ms = elapsed / args.steps * 1e3
    value = B * info.world * args.steps / elapsed
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": info.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "p50_req_latency_ms": round(p50_req, 3),
        "p50_batch_latency_ms": round(p50, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / REF_IMG_PER_S, 1),
        "baseline_img_per_s": REF_IMG_PER_S,
        "dtype": "bf16" if cuda else "fp32",
        "gpu_jpeg": bool(JPEG and cuda),
        **({"jpeg_scan_bytes_per_image": round(sum(jpeg_bytes) / len(jpeg_bytes))} if jpeg_bytes else {}),
        "process_group": info.backend,
        **({"collective_overlaps_compute": overlap} if overlap is not None else {}),
        "data": "synthetic uint8 224x224 images, seeded random-init VGG16 weights",
        "config": {"model": f"vgg16_deconvnet_{args.layer}", "global_batch": B * info.world, "seq_len": S,
                   "image_size": S, "filters_per_image": args.k, "parallelism": f"dp{info.world}"},
    }
    if args.tiny:
        line["data"] = "REHEARSAL: scaled VGG16 (width/8, 32px) on CPU - not a benchmark"
    if args.no_copyback:
        line["data"] = "DIAGNOSTIC: mosaics not copied back to the host - not a benchmark"
    if emu_n:
        line["data"] = f"DIAGNOSTIC: + {emu_n} mosaic-sized D2D copies per step (emulated {emu_n + 1}-rank all-gather)"
        line["emulated_gather_bytes_per_step"] = int(emu_dst.numel())
    if rccl_n:
        line["data"] = (f"DIAGNOSTIC: + a paced {rccl_n + 1}-rank all-gather model per step ({args.rccl_channels} CUs, "
                        f"{args.rccl_gbs} GB/s)")
        line["emulated_gather_bytes_per_step"] = int(rccl_dst.numel())
        line["emulated_gather_ms_per_step"] = round(rccl_dst.numel() / (args.rccl_gbs * 1e6), 3)
    if info.is_main:
        print(json.dumps(line), flush=True)
    pdist.shutdown()
    return line


def _breakdown(eng, images, xbuf, args, sync):
    """Per-phase wall time with syncs (diagnostic only, not the reported number)."""
    def t(fn):
        sync()
        a = time.perf_counter()
        r = fn()
        sync()
        return r, (time.perf_counter() - a) * 1e3

    _, tp = t(lambda: ops.resize_preprocess(images, xbuf))
    st, tf = t(lambda: eng.forward(xbuf, args.layer))
    (idx, _), ts = t(lambda: eng.select_filters(st.out, args.k))
    rec, tb = t(lambda: eng.backward(st, idx))
    B = rec.shape[0]
    _, td = t(lambda: ops.deprocess_mosaic(rec.reshape(B * args.k, *rec.shape[2:]).contiguous()))
    log(f"breakdown ms: preprocess {tp:.2f} forward {tf:.2f} select {ts:.2f} backward {tb:.2f} deprocess {td:.2f}")


if __name__ == "__main__":
    main()
