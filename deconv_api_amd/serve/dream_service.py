"""Service behind the ``POST /deepdream`` extension route (not in the reference): decode ->
DeepDream (InceptionV3 or ResNet-50) on the GPU worker -> JPEG data URL (same conventions as
``POST /``)."""
from __future__ import annotations

import asyncio
import concurrent.futures as cf
import threading
from typing import Dict, Optional

import numpy as np
import torch

from ..codec import encode_data_url, read_data_url
from ..config import Config
from ..engine.deepdream import RESNET_LAYERS, DeepDream, DreamSettings

MAX_SIDE = 1024


class DreamService:
    def __init__(self, cfg: Optional[Config] = None):
        self.cfg = cfg or Config.from_env()
        self.device = torch.device(self.cfg.resolve_device())
        self._engines: Dict[str, DeepDream] = {}
        self._lock = threading.Lock()
        self._gpu = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="dv-dream")

    def engine(self, model: str, octaves: int, steps: int) -> DeepDream:
        if model not in ("inception_v3", "resnet50"):
            raise ValueError("model must be inception_v3 or resnet50")
        if not (1 <= octaves <= 6 and 1 <= steps <= 100):
            raise ValueError("octaves must be 1..6 and steps 1..100")
        with self._lock:
            if model not in self._engines:
                if model == "inception_v3":
                    from ..models.inception_v3 import InceptionV3

                    net = InceptionV3(self.cfg.seed).build(self.device)
                    self._engines[model] = DeepDream(net, DreamSettings(), use_graphs=self.cfg.hip_graphs)
                else:
                    from ..models.resnet50 import ResNet50

                    net = ResNet50(self.cfg.seed).build(self.device)
                    self._engines[model] = DeepDream(net, DreamSettings(layers=dict(RESNET_LAYERS)),
                                                     use_graphs=self.cfg.hip_graphs)
            e = self._engines[model]
        e.s.octaves, e.s.iterations = octaves, steps
        return e

    def _run(self, img: np.ndarray, model: str, octaves: int, steps: int) -> np.ndarray:
        e = self.engine(model, octaves, steps)
        h, w = img.shape[:2]
        scale = min(1.0, MAX_SIDE / max(h, w))
        t = torch.from_numpy(img).unsqueeze(0)
        if scale < 1.0:
            from ..engine.deepdream import resize

            t = resize(t.float(), (int(h * scale), int(w * scale))).round().clamp(0, 255).to(torch.uint8)
        small = min(t.shape[1:3]) / (e.s.octave_scale ** (octaves - 1))
        if small < 75:
            raise ValueError(f"image too small for {octaves} octaves (smallest octave side {small:.0f} < 75)")
        return e.dream_u8(t)[0].cpu().numpy()

    async def dream(self, uri: str, model: str = "inception_v3", octaves: int = 4, steps: int = 20) -> str:
        loop = asyncio.get_running_loop()
        img = await loop.run_in_executor(None, read_data_url, uri)
        out = await loop.run_in_executor(self._gpu, self._run, img, model, octaves, steps)
        return await loop.run_in_executor(None, encode_data_url, out, self.cfg.jpeg_quality)
