"""Batcher (serve/service.py _collect): under load a batch is trimmed to a full graph bucket and the rest
is carried, in order, into the next batch (a 46-image batch would replay the 64-image graph)."""
import queue
import time

from deconv_api_amd.config import Config
from deconv_api_amd.serve import service as S


def _svc(n_queued, max_batch=64):
    svc = S.DeconvService.__new__(S.DeconvService)
    svc.cfg = Config(max_batch=max_batch, batch_timeout_ms=1.0)
    svc.q = queue.Queue()
    svc.done_q = queue.Queue()
    svc._carry = []
    svc._batch_t0 = time.perf_counter()  # a batch in flight: the collector waits for stragglers
    svc.graphs = object()
    for i in range(n_queued):
        svc.q.put(i)
    return svc


def test_trim_to_bucket_and_carry_in_order():
    svc = _svc(46)
    b1 = svc._collect(0.0)
    assert b1 == list(range(32)) and svc._carry == list(range(32, 46))
    b2 = svc._collect(0.0)
    assert b2 == list(range(32, 46))  # 14 <= TRIM_MIN: not trimmed
    assert svc._collect(0.0) == []


def test_full_buckets_and_small_batches_untouched():
    svc = _svc(64)
    assert svc._collect(0.0) == list(range(64))
    svc = _svc(13)
    assert svc._collect(0.0) == list(range(13))
    svc = _svc(80)
    assert svc._collect(0.0) == list(range(64))  # max_batch
    assert svc._collect(0.0) == list(range(64, 80))  # 16: a bucket


def test_no_trim_without_graphs():
    svc = _svc(46)
    svc.graphs = None
    assert svc._collect(0.0) == list(range(46))
