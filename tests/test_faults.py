"""CPU: injected faults are contained (failed batch -> error response, service keeps serving) and
the watchdog reports a stalled batch on /ready."""
import asyncio
import time

import numpy as np
import pytest
import torch

from deconv_api_amd.codec import make_data_url
from deconv_api_amd.config import Config
from deconv_api_amd.engine.deconvnet import DeconvNet
from deconv_api_amd.models.vgg16 import VGG16
from deconv_api_amd.serve.service import DeconvService

pytestmark = pytest.mark.filterwarnings("ignore::DeprecationWarning")


def _svc(small_specs, monkeypatch, fault, **cfg):
    monkeypatch.setenv("DV_FAULT", fault)
    c = Config.from_env(device="cpu", image_size=32, max_batch=4, batch_timeout_ms=1.0, codec_workers=2, **cfg)
    eng = DeconvNet(VGG16.random(0, specs=small_specs).build("cpu", torch.float32))
    return DeconvService(c, engine=eng)


def _url(seed=0):
    return make_data_url(np.random.default_rng(seed).integers(0, 256, (32, 32, 3), dtype=np.uint8), "PNG")


def test_injected_raise_is_contained(small_specs, monkeypatch):
    svc = _svc(small_specs, monkeypatch, "raise@1")
    try:
        with pytest.raises(RuntimeError):
            asyncio.run(svc.deconv(_url(), "block2_conv1"))
        out = asyncio.run(svc.deconv(_url(1), "block2_conv1"))
        assert out.startswith("data:image/webp;base64,")
        assert "InjectedFault" in (svc.last_error or "")
        assert svc.status()["worker_alive"]
    finally:
        svc.close()


def test_watchdog_marks_stall(small_specs, monkeypatch):
    svc = _svc(small_specs, monkeypatch, "hang@1:2.0", request_timeout_s=0.5)
    try:
        async def go():
            t = asyncio.ensure_future(svc.deconv(_url(), "block1_conv1"))
            await asyncio.sleep(1.3)
            st = svc.status()
            try:
                await t
            except asyncio.TimeoutError:
                pass
            return st

        st = asyncio.run(go())
        assert st["stalled"] is True and st["worker_alive"] is False
        time.sleep(1.5)
        assert svc.status()["stalled"] is False
    finally:
        svc.close()
