"""Latency / serving throughput on one GPU.

1. engine: p50 latency of one deconvnet batch (block5_conv3) for several batch sizes, eager vs
   hipGraph replay;
2. service: the full request path (base64 decode, PIL decode, GPU resize+preprocess, batched
   engine, D2H, JPEG encode, quoted data URL) driven by C concurrent in-process clients:
   requests/s and p50/p99 request latency.
Prints one JSON object.
"""
import argparse
import asyncio
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.codec import make_data_url  # noqa: E402
from deconv_api_amd.config import Config  # noqa: E402
from deconv_api_amd.engine.deconvnet import DeconvNet  # noqa: E402
from deconv_api_amd.engine.graphs import GraphedDeconv  # noqa: E402
from deconv_api_amd.models.vgg16 import VGG16  # noqa: E402
from deconv_api_amd.serve.service import DeconvService  # noqa: E402


def p(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))]


def engine_latency(eng, layer, sizes, reps):
    dev = eng.rt.device
    gd = GraphedDeconv(eng)
    out = {}
    for B in sizes:
        x = torch.randn(B, 224, 224, 8, device=dev).mul(50).to(torch.bfloat16)
        row = {}
        for mode in ("eager", "graph"):
            fn = (lambda: eng.run(x, layer)) if mode == "eager" else (lambda: gd.run(x, layer))
            fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t) * 1e3)
            row[mode] = {"p50_ms": round(p(ts, 0.5), 3), "img_per_s": round(B / (p(ts, 0.5) / 1e3), 1)}
        out[str(B)] = row
    return out


async def serve_load(svc, layer, clients, total, size):
    rng = np.random.default_rng(0)
    urls = [make_data_url(rng.integers(0, 256, (size, size, 3), dtype=np.uint8), "JPEG") for _ in range(16)]
    lat = []
    sem = asyncio.Semaphore(clients)

    async def one(i):
        async with sem:
            t = time.perf_counter()
            s = await svc.deconv(urls[i % len(urls)], layer)
            assert s.startswith("data:image/webp;base64,")
            lat.append((time.perf_counter() - t) * 1e3)

    await one(0)  # warm (graph capture for bucket 1)
    lat.clear()
    t0 = time.perf_counter()
    await asyncio.gather(*(one(i) for i in range(total)))
    dt = time.perf_counter() - t0
    return {"clients": clients, "requests": total, "req_per_s": round(total / dt, 1),
            "p50_ms": round(p(lat, 0.5), 2), "p99_ms": round(p(lat, 0.99), 2)}


class Sampler:
    """Poor man's sampling profiler: every ``period`` s, the innermost Python frame of every
    thread (function, file:line) is counted; shows where the host time of the service goes."""

    def __init__(self, period=0.0005):
        import collections
        import threading

        self.period = period
        self.counts = collections.Counter()
        self.stop = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        import threading

        me = threading.get_ident()
        names = {}
        while not self.stop.wait(self.period):
            for tid, fr in sys._current_frames().items():
                if tid == me:
                    continue
                if tid not in names:
                    names = {t.ident: t.name for t in threading.enumerate()}
                key = (names.get(tid, "?").split("_")[0], f"{fr.f_code.co_name} {os.path.basename(fr.f_code.co_filename)}:{fr.f_lineno}")
                self.counts[key] += 1

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *a):
        self.stop.set()
        self.t.join()

    def top(self, n=40):
        tot = sum(self.counts.values())
        return [[th, fn, round(c / tot, 4)] for (th, fn), c in self.counts.most_common(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="block5_conv3")
    ap.add_argument("--sizes", default="1,4,16,64")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--clients", default="1,16,64")
    ap.add_argument("--requests", type=int, default=256)
    ap.add_argument("--img", type=int, default=320, help="client image side (resized to 224 on GPU)")
    ap.add_argument("--sample", action="store_true", help="sample Python stacks during the last load run")
    ap.add_argument("--timeout-ms", type=float, default=Config.batch_timeout_ms,
                    help="batcher straggler wait while the GPU is busy")
    ap.add_argument("--chunk", type=int, default=16, help="images per encode+deliver chunk")
    ap.add_argument("--codec-workers", type=int, default=16)
    ap.add_argument("--max-batch", type=int, default=Config.max_batch)
    ap.add_argument("--switch-us", type=int, default=500)
    ap.add_argument("--enc-workers", type=int, default=2)
    ap.add_argument("--enc-threads", type=int, default=8)
    ap.add_argument("--gpu-jpeg", type=int, default=1, help="1: responses JPEG-encoded on the GPU (csrc/jpeg_gpu.hip)")
    a = ap.parse_args()
    ops.native.load()
    dev = torch.device("cuda", 0)
    eng = DeconvNet(VGG16.random(0).build(dev, torch.bfloat16))
    res = {"engine": engine_latency(eng, a.layer, [int(s) for s in a.sizes.split(",")], a.reps)}
    cfg = Config.from_env(device="cuda", max_batch=a.max_batch, batch_timeout_ms=a.timeout_ms, codec_workers=a.codec_workers,
                          encode_chunk=a.chunk, gil_switch_us=a.switch_us,
                          encode_workers=a.enc_workers, encode_threads=a.enc_threads, gpu_jpeg=bool(a.gpu_jpeg))
    svc = DeconvService(cfg, engine=eng)
    res["service"] = []
    clients = [int(x) for x in a.clients.split(",")]
    svc.trace = []
    for i, c in enumerate(clients):
        if a.sample and i == len(clients) - 1:
            with Sampler() as smp:
                res["service"].append(asyncio.run(serve_load(svc, a.layer, c, max(a.requests, c), a.img)))
            res["samples"] = smp.top()
        else:
            res["service"].append(asyncio.run(serve_load(svc, a.layer, c, max(a.requests, c), a.img)))
    from deconv_api_amd.utils import metrics as M

    tr = svc.trace[-min(len(svc.trace), 2000):]
    if tr:
        names = ["decode", "queue", "gpu+d2h", "encode", "deliver"]
        res["breakdown_ms"] = {n: round(1e3 * sum(t[i + 1] - t[i] for t in tr) / len(tr), 2) for i, n in enumerate(names)}

    res["stage_metrics"] = [l for l in M.REGISTRY.render().splitlines() if l.startswith("dv_stage_seconds_sum")
                            or l.startswith("dv_stage_seconds_count")]
    res["graphs"] = svc.status()["graphs"]
    res["settings"] = {"enc": [a.enc_workers, a.enc_threads], "switch_us": a.switch_us, "max_batch": a.max_batch, "timeout_ms": a.timeout_ms, "chunk": a.chunk, "codec_workers": a.codec_workers, "gpu_jpeg": bool(a.gpu_jpeg)}
    svc.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
