"""Config: every field is read by the code it configures, the precision switch maps to
the engine dtype, and bad values fail at construction (app/main.py:16-17 hard-codes the reference's)."""
import dataclasses
import pathlib
import re

import pytest
import torch

from deconv_api_amd.config import Config

PKG = pathlib.Path(__file__).resolve().parents[1] / "deconv_api_amd"


def _sources():
    return "\n".join(p.read_text() for p in PKG.rglob("*.py") if p.name != "config.py")


def test_every_config_field_is_consumed():
    src = _sources()
    unused = []
    for f in dataclasses.fields(Config):
        pat = {"dtype": r"torch_dtype\(", "device": r"resolve_device\("}.get(
            f.name, rf"(cfg|config|self\.cfg)\.{f.name}\b")  # (methods of Config that read the field)
        if not re.search(pat, src):
            unused.append(f.name)
    assert not unused, f"Config fields nothing reads: {unused}"


def test_dtype_switch():
    assert Config().torch_dtype("cuda") == torch.bfloat16
    assert Config(dtype="fp16").torch_dtype("cuda") == torch.float16
    for d in ("bf16", "fp16", "fp32"):
        assert Config(dtype=d).torch_dtype("cpu") == torch.float32  # the CPU engine is the fp32 oracle
    with pytest.raises(ValueError, match="fp32"):
        Config(dtype="fp32").torch_dtype("cuda")
    with pytest.raises(ValueError):
        Config(dtype="int8")


def test_env_overrides(monkeypatch):
    monkeypatch.setenv("DV_DTYPE", "fp16")
    monkeypatch.setenv("DV_FRONTENDS", "3")
    monkeypatch.setenv("DV_CORS_ORIGINS", "http://a, http://b")
    c = Config.from_env()
    assert c.dtype == "fp16" and c.frontends == 3 and c.cors_origins == ("http://a", "http://b")
    monkeypatch.setenv("DV_MODE", "sideways")
    with pytest.raises(ValueError):
        Config.from_env()
