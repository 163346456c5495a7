"""Multi-GPU serving input path on a real GPU (ADVICE-low / VERDICT r4 weak #6): a batch's upload,
resize and scatter run on ``ShardedRunner.in_stream``, so rank 0 enqueues batch i+1's engine work
while batch i's engine work is still running (two batches in flight, no idle GPU gap per batch).

One GPU cannot hold a multi-rank RCCL group, so the runner is driven at world 2 with the collectives
replaced by stream-ordered stand-ins with RCCL's async semantics: the scatter is a copy enqueued on
the CURRENT stream and its work object completes when the stream reaches it (``is_completed`` =
event query), which is exactly what made the old compute-stream scatter wait behind the previous
batch's engine. The engine is a stand-in too: a fixed GPU spin (``torch.cuda._sleep``) long enough
that the host certainly returns from ``launch`` before it ends, plus a mosaic derived from the
shard so the data path can be checked end to end (``finish``: gather, raw copy-back). This test found
a real race of the overlapped path: the gather's receive buffers came from the compute stream's pool,
where they could alias the NEXT batch's still-queued engine buffers (``_gather_cmd`` now allocates them
on ``comm_stream``).
"""
import time
import types

import numpy as np
import pytest
import torch

SPIN = 400_000_000  # GPU cycles per engine call (~170 ms at 2.4 GHz)


class _Work:
    def __init__(self):
        self.ev = torch.cuda.Event()
        self.ev.record()

    def is_completed(self):
        return self.ev.query()

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


class _Ctl:
    epoch = 0
    members = [0, 1]
    hb_timeout = 3.0

    def __init__(self):
        self.seq = 0

    def post_cmd(self, msg):
        self.seq += 1
        return self.seq

    def wait_acks(self, kind, seq):
        pass

    def go(self, kind, seq):
        pass

    def stale(self):
        return []


class _Engine:
    def run(self, x, layer, k=4, mode="all"):
        torch.cuda._sleep(SPIN)
        n, S = x.shape[0], x.shape[1]
        v = x[:, :, :, :3].float().mean(dim=(1, 2))  # [n, 3] from the shard the engine received
        mos = (v.abs() * 40).clamp(0, 255).to(torch.uint8)[:, None, None, :].expand(n, 2 * S, 2 * S, 3)

        class R:
            mosaic = mos.contiguous()
        return R()


def _runner(monkeypatch, side: bool):
    from deconv_api_amd.parallel import sharded
    from deconv_api_amd.parallel.dist import DistInfo

    dev = torch.device("cuda", 0)
    cfg = types.SimpleNamespace(gpu_jpeg=False, jpeg_quality=95, seed=0)  # raw mosaics back
    r = sharded.ShardedRunner(_Engine(), DistInfo(0, 1, 0, dev, "nccl"), image_size=64, use_graphs=False, cfg=cfg)
    r.info = DistInfo(0, 2, 0, dev, "nccl")
    r.ctl = _Ctl()
    if not side:
        r.in_stream = None  # the round-4 behaviour: input path on the compute stream

    def scatter(out, scatter_list=None, src=0, async_op=True):
        out.copy_(scatter_list[0], non_blocking=True)
        return _Work()

    def gather(t, gather_list=None, dst=0, async_op=True):
        for p in gather_list:
            p.copy_(t, non_blocking=True)
        return _Work()

    monkeypatch.setattr(sharded.dist, "scatter", scatter)
    monkeypatch.setattr(sharded.dist, "gather", gather)
    return r


def _images(seed):
    g = np.random.default_rng(seed)
    return [g.integers(0, 256, (80 + 8 * i, 96, 3), dtype=np.uint8) for i in range(4)]


@pytest.mark.gpu
@pytest.mark.parametrize("side", [True, False])
def test_next_batch_enqueued_while_previous_runs(monkeypatch, side):
    r = _runner(monkeypatch, side)
    # warm-up in the measured pattern (two in flight), every staging slot twice: stream pools, pinned
    # host blocks (a fresh pinned block is a device-synchronizing hipHostMalloc), native library
    for _ in range(3):
        w = [r.launch("block5_conv3", _images(0)) for _ in range(2)]
        for b in w:
            r.finish(b)
    torch.cuda.synchronize()
    # no cyclic-GC pass inside the timed launches: collecting an earlier test's hipGraphs destroys
    # them, and hipGraphExecDestroy waits for the device (it did, behind batch 1's engine spin)
    import gc

    gc.collect()
    gc.disable()
    import sys
    import threading
    import traceback

    main, where = threading.get_ident(), []
    # if the launches block, record where (the host stack 60 ms in, while the spin still runs)
    timer = threading.Timer(0.06, lambda: where.append("".join(traceback.format_stack(sys._current_frames()[main]))))
    t0 = time.perf_counter()
    timer.start()
    b1 = r.launch("block5_conv3", _images(1))
    t1 = time.perf_counter()
    b2 = r.launch("block5_conv3", _images(2))
    timer.cancel()
    host_ms = (time.perf_counter() - t0) * 1e3
    host_ms = f"{host_ms:.1f} (batch 1 {1e3 * (t1 - t0):.1f}) {where[-1][-1500:] if where else ''}"
    b1_running = not b1.ev.query()  # batch 2's engine is enqueued: was batch 1's still running?
    gc.enable()
    out1, out2 = r.finish(b1), r.finish(b2)
    if side:
        assert b1_running, f"batch 2's scatter waited for batch 1's engine work ({host_ms} ms to launch both)"
    else:
        assert not b1_running  # the gap this change removes (guards the stand-ins' semantics)
    # rank 0's half of each batch went through scatter -> engine -> gather -> copy-back intact
    # (the stand-in gather fills the peer's half with rank 0's, so only the first two are compared)
    for out, seed in ((out1, 1), (out2, 2)):
        assert isinstance(out, np.ndarray) and out.shape == (4, 128, 128, 3)
        ref = r._local("block5_conv3", _images(seed)).cpu().numpy()
        np.testing.assert_array_equal(out[:2], ref[:2])
