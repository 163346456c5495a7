#!/usr/bin/env python
"""Host codec throughput vs threads (GIL behaviour): PIL JPEG encode, PIL decode, and the native
encoder (csrc/jpeg_enc.cpp) on realistic 448x448 mosaics. Prints one JSON line per case."""
import concurrent.futures as cf
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from deconv_api_amd.codec import encode_data_url, make_data_url, read_data_url  # noqa: E402
from deconv_api_amd.ops import native  # noqa: E402


def smooth(seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:448, 0:448].astype(np.float32)
    img = 128 + 60 * np.sin(xx / (7 + seed)) * np.cos(yy / 11) + rng.normal(0, 12, (448, 448))
    return np.clip(np.stack([img, img[::-1], img.T], -1), 0, 255).astype(np.uint8)


def rate(fn, n, workers):
    with cf.ThreadPoolExecutor(workers) as ex:
        list(ex.map(fn, range(min(n, 16))))
        t = time.perf_counter()
        list(ex.map(fn, range(n)))
        return n / (time.perf_counter() - t)


def main():
    mos = [smooth(i) for i in range(8)]
    urls = [make_data_url(np.ascontiguousarray(m[::2, ::2][:320, :320]), "JPEG") for m in mos]
    lib = native.load()
    batch = torch.from_numpy(np.stack(mos * 8))
    print(json.dumps({"cpus": os.cpu_count(), "sched": len(os.sched_getaffinity(0))}))
    for w in (1, 4, 8, 16):
        r = {"threads": w,
             "pil_encode_per_s": round(rate(lambda i: encode_data_url(mos[i % 8]), 256, w), 1),
             "pil_decode_per_s": round(rate(lambda i: read_data_url(urls[i % 8]), 256, w), 1)}
        t = time.perf_counter()
        lib.jpeg_data_urls(batch, 95, "data:image/webp;base64,", w)
        r["native_encode_per_s"] = round(64 / (time.perf_counter() - t), 1)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
