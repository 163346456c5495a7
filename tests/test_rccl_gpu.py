"""RCCL on the GPU box: a real 1-rank process group (torchrun) runs the collective code paths of
bench.py and of parallel/dist.py + the serving data plane (the driver's 8-GPU scaling run uses the
same calls with more ranks)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(script_args, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), *script_args]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert lines, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(lines[-1])


@pytest.mark.gpu
def test_rccl_collectives_selftest():
    out = _torchrun(["tools/rccl_selftest.py"])
    assert out == {"backend": "nccl", "world": 1, "broadcast_state": True, "all_gather_rows": True,
                   "all_reduce_max": True, "scatter": True, "gather": True}, out


@pytest.mark.gpu
def test_rccl_reform_aborts_and_rebuilds():
    """The failover's re-form path on a real RCCL group (world 1, same membership): abort the
    communicator with a collective in flight, build the new group, run a collective on it."""
    out = _torchrun(["tools/rccl_selftest.py", "--reform"])
    assert out["backend"] == "nccl" and out["reform_epoch"] == 1 and out["reform_all_reduce"] is True, out


@pytest.mark.gpu
def test_bench_under_torchrun_uses_rccl():
    out = _torchrun(["bench.py", "--gpus", "1", "--steps", "2", "--warmup", "1", "--batch", "8"])
    assert out["process_group"] == "nccl" and out["n_gpus"] == 1 and out["config"]["parallelism"] == "dp1"
    assert out["value"] > 0 and out["p50_req_latency_ms"] >= out["p50_batch_latency_ms"] * 0.5
    # the step's compute stream was probed onto a hardware queue apart from RCCL's (parallel/dist.py:
    # pick_compute_stream): the async all-gather of step i overlaps step i+1 instead of queueing behind it
    assert out["collective_overlaps_compute"] is True, out


@pytest.mark.gpu
def test_bench_gpu_jpeg_gather_under_torchrun(monkeypatch):
    """bench.py's GPU-JPEG mode on a real RCCL group: per-step scans, the max-size all-reduce and the
    deferred exact-size all-gather of the scans (the N > 1 data path, at world 1)."""
    monkeypatch.setenv("DV_BENCH_JPEG", "1")
    out = _torchrun(["bench.py", "--gpus", "1", "--steps", "3", "--warmup", "1", "--batch", "8"])
    assert out["process_group"] == "nccl" and out["gpu_jpeg"] is True and out["value"] > 0, out
    assert 1000 < out["jpeg_scan_bytes_per_image"] < 600000, out
