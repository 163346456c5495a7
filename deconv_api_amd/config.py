"""Single frozen configuration with ``DV_*`` environment overrides.

The reference hard-codes every setting (app/main.py:16-17,53,64,67-69,73; Dockerfile:10,15);
the defaults below reproduce those values."""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass
from typing import Tuple


def _env(name: str, default, cast):
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    if cast is bool:
        return v.lower() in ("1", "true", "yes", "on")
    if cast is tuple:
        return tuple(x.strip() for x in v.split(",") if x.strip())
    return cast(v)


DTYPES = ("bf16", "fp16", "fp32")


@dataclass(frozen=True)
class Config:
    weights: str = ""                     # VGG16 (app/main.py:17) .safetensors/.pt/.h5; empty = seeded random init
    seed: int = 0
    dtype: str = "bf16"                   # GPU engine storage dtype: bf16 | fp16 (MFMA, fp32 accumulate);
                                          #   fp32 is the CPU engine's (the oracle); fp32 on a GPU is refused
    device: str = "auto"                  # auto | cuda | cpu
    image_size: int = 224                 # app/main.py:53
    filters: int = 4                      # tiles in the mosaic (app/main.py:67-69)
    mode: str = "all"                     # visualize_mode (app/main.py:64)
    frontends: int = 4                    # serve/launch.py: HTTP front-end processes per rank (serve/ingest.py);
                                          #   0 = uvicorn inside the GPU process (multi-rank: rank 0 shards batches)
    jpeg_quality: int = 95                # OpenCV imencode default (app/main.py:73)
    # request batcher. Through real HTTP with 8 front-end processes (profiles/http_load_r6.txt run d):
    # 16 -> 4957, 32 -> 5566, 64 -> 5357 req/s (JPEG-only, 256 clients): at 16 the GPU was ~85 % busy
    # with B = 16 batches. (Round 3, in-process clients and one GIL, preferred 16: latency_r3_batch_sweep.txt)
    max_batch: int = 32
    batch_timeout_ms: float = 2.0
    max_queue: int = 4096                 # backpressure: 503 beyond this many pending requests
    request_timeout_s: float = 120.0
    codec_workers: int = 8                # decode threads (PIL releases the GIL while decoding)
    encode_threads: int = 8               # native JPEG encoder threads per encode call (GIL released)
    encode_workers: int = 2               # batches encoded concurrently (tools/latency.py A/B: 2 x 8 best)
    encode_chunk: int = 16                # images per encode call; each chunk is delivered at once
    gil_switch_us: int = 500              # sys.setswitchinterval for the serving process (0 = leave)
    native_codec: bool = True             # native encoder for responses (PIL fallback when False/unbuilt)
    gpu_jpeg: bool = True                 # GPU: responses JPEG-encoded on the device (csrc/jpeg_gpu.hip);
                                          #   the host only base64s the scans
    cors_origins: Tuple[str, ...] = ("*",)  # app/main.py:22-32
    host: str = "0.0.0.0"
    port: int = 80                        # Dockerfile:10,15
    hip_graphs: bool = True
    inception_weights: str = ""          # /deepdream InceptionV3: folded .safetensors or Keras .h5 (empty = random)
    resnet_weights: str = ""             # /deepdream ResNet-50: same
    dream_max_batch: int = 8              # /deepdream: same-shape requests run as one DeepDream batch
    dream_window_ms: float = 20.0         # /deepdream: how long the worker waits to fill a batch
    dream_tile: int = 512                 # /deepdream: images with a side above this (or any image when
                                          #   world > 1) run tiled (TiledDeepDream), across every rank
    log_json: bool = True
    asyncio_debug: bool = False           # DV_ASYNCIO_DEBUG=1: event-loop debug mode, slow-callback log
    slow_callback_ms: float = 50.0        # ... threshold for logging a blocking callback (debug mode)

    @classmethod
    def from_env(cls, **overrides) -> "Config":
        kw = {}
        for f in dataclasses.fields(cls):
            cast = {int: int, float: float, bool: bool, str: str}.get(type(f.default), tuple)
            if isinstance(f.default, tuple):
                cast = tuple
            kw[f.name] = _env("DV_" + f.name.upper(), f.default, cast)
        kw.update(overrides)
        return cls(**kw)

    def __post_init__(self):
        if self.dtype not in DTYPES:
            raise ValueError(f"DV_DTYPE must be one of {DTYPES}, got {self.dtype!r}")
        if self.mode not in ("all", "max"):
            raise ValueError(f"DV_MODE must be 'all' or 'max', got {self.mode!r}")
        if not 1 <= self.filters <= 4:
            raise ValueError("DV_FILTERS must be 1..4 (tiles of the 2x2 mosaic)")
        if self.frontends < 0:
            raise ValueError("DV_FRONTENDS must be >= 0")

    def torch_dtype(self, device):
        """Engine dtype on ``device``: the MFMA kernels run bf16 or fp16 storage; the CPU engine is
        the fp32 PyTorch oracle whatever ``dtype`` says."""
        import torch

        if torch.device(device).type != "cuda":
            return torch.float32
        if self.dtype == "fp32":
            raise ValueError("DV_DTYPE=fp32 is not served on the GPU: the deconvnet kernels are bf16 / fp16 "
                             "MFMA with fp32 accumulation (the fp32 path is the CPU engine, DV_DEVICE=cpu)")
        return torch.float16 if self.dtype == "fp16" else torch.bfloat16

    def resolve_device(self) -> str:
        if self.device != "auto":
            return self.device
        import torch

        return "cuda" if torch.cuda.is_available() else "cpu"
