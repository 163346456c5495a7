"""utils/tracing.py: roctx ranges (rocprofv3 --marker-trace) are safe to call with or without libroctx64, and
range_() accumulates host wall time per name."""
from __future__ import annotations

import time

from deconv_api_amd.utils import tracing


def test_range_accumulates_and_nests():
    t = {}
    with tracing.range_("outer", t):
        with tracing.range_("inner", t):
            time.sleep(0.01)
        with tracing.range_("inner", t):
            time.sleep(0.01)
    tracing.mark("done")
    assert t["inner"] >= 0.018 and t["outer"] >= t["inner"]


def test_disabled_is_a_noop(monkeypatch):
    monkeypatch.setattr(tracing, "ENABLED", False)
    called = []

    class Lib:
        def roctxRangePushA(self, *_):
            called.append("push")

    monkeypatch.setattr(tracing, "_lib", Lib())
    tracing.push("x")
    tracing.mark("x")
    assert called == []
    assert isinstance(tracing.available(), bool)
