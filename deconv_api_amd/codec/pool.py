"""Host codec thread pool: PIL/libjpeg-turbo release the GIL while decoding/encoding, so a
thread pool overlaps JPEG work for one batch with GPU compute of the next (at GPU
speed the host codec, ~1.6 ms/img/core, is the end-to-end limit)."""
from __future__ import annotations

import concurrent.futures as cf
import os
from typing import List, Sequence

import numpy as np

from .image import encode_data_url, read_data_url


class CodecPool:
    def __init__(self, workers: int | None = None):
        workers = workers or max(2, min(16, (os.cpu_count() or 4)))
        self.ex = cf.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="codec")
        self.workers = workers

    def decode_many(self, uris: Sequence[str]) -> List:
        """Returns per-item ndarray or the exception raised while decoding it."""
        futs = [self.ex.submit(read_data_url, u) for u in uris]
        out = []
        for f in futs:
            try:
                out.append(f.result())
            except Exception as e:  # noqa: BLE001 - propagated per item
                out.append(e)
        return out

    def encode_many(self, mosaics: np.ndarray, quality: int = 95) -> List[str]:
        return list(self.ex.map(lambda m: encode_data_url(m, quality), list(mosaics)))

    def submit(self, fn, *a, **k):
        return self.ex.submit(fn, *a, **k)

    def shutdown(self):
        self.ex.shutdown(wait=False, cancel_futures=True)
