#!/usr/bin/env python
"""Scaling sweep of the flagship benchmark: runs ``bench.py`` at N = 1, 2, 4, 8
ranks on one node (one process per GPU under torch.distributed.run, RCCL over xGMI; rendezvous on
127.0.0.1), parses each run's JSON line and reports per-N throughput and weak-scaling efficiency
value_N / (N * value_1).

  python tools/scale_sweep.py                      # every power of two up to the visible GPUs
  python tools/scale_sweep.py --max-gpus 2 --device cpu --tiny   # CPU/Gloo rehearsal
  python tools/scale_sweep.py --out scale.json --steps 20 --warmup 5

The driver measures the official scaling curve itself (SCALE_rNN.json); this is the same
measurement for development boxes.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus() -> int:
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if env:
        return len([d for d in env.split(",") if d.strip()])
    try:  # counting devices does not initialise the GPU on this image
        import torch

        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def bench_cmd(n: int, a) -> list:
    extra = ["--gpus", str(n), "--steps", str(a.steps), "--warmup", str(a.warmup)]
    if a.device == "cpu":
        extra += ["--device", "cpu"]
    if a.tiny:
        extra += ["--tiny"]
    if a.batch:
        extra += ["--batch", str(a.batch)]
    bench = os.path.join(HERE, "bench.py")
    if n == 1:
        return [sys.executable, bench, *extra]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), bench, *extra]


def parse_json_line(text: str):
    for line in reversed(text.splitlines()):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    return None


def efficiency(rows):
    """Weak scaling: value_N / (N * value_1) for every N with a result (needs the N = 1 row)."""
    base = next((r["value"] for r in rows if r["n"] == 1 and r.get("value")), None)
    for r in rows:
        r["efficiency"] = None if (base is None or not r.get("value")) else round(r["value"] / (r["n"] * base), 4)
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--max-gpus", type=int, default=0, help="0: all visible GPUs")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="images per rank (0: bench default)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--timeout", type=int, default=900, help="seconds per run")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    top = a.max_gpus or (visible_gpus() if a.device == "cuda" else 2)
    ns = [n for n in (1, 2, 4, 8) if n <= max(1, top)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
               MASTER_ADDR="127.0.0.1")
    rows = []
    for n in ns:
        t0 = time.time()
        try:
            p = subprocess.run(bench_cmd(n, a), cwd=HERE, env=env, capture_output=True, text=True, timeout=a.timeout)
            res = parse_json_line(p.stdout)
            row = {"n": n, "rc": p.returncode, "wall_s": round(time.time() - t0, 1)}
            if res:
                row.update(value=res["value"], unit=res.get("unit"), ms_per_step=res.get("ms_per_step"),
                           parallelism=res.get("config", {}).get("parallelism"))
            else:
                row["error"] = (p.stderr or p.stdout)[-400:]
        except subprocess.TimeoutExpired:
            row = {"n": n, "rc": None, "error": f"timeout after {a.timeout}s"}
        rows.append(row)
        print(json.dumps(row), flush=True)
    out = {"metric": rows[0].get("unit") if rows else None, "scaling": "weak", "rows": efficiency(rows)}
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0 if all(r.get("rc") == 0 for r in rows) else 1


if __name__ == "__main__":
    raise SystemExit(main())
