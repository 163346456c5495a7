"""Front-end supervisor of one rank (``DV_FRONTENDS`` > 0; design: serve/ingest.py).

    python -m deconv_api_amd.serve.supervisor --sock /tmp/dv-ingest-80-r0-123.sock --n 4 --owner-pid 123

serve/launch.py starts this process BEFORE the rank's GPU owner touches the GPU, and it starts and
watches the rank's HTTP front ends (serve/frontend.py). A front end that exits while its owner is alive
(a crash, an OOM kill, a killed process) is started again, so its share of the SO_REUSEPORT group comes
back; one that keeps dying (port taken, bad configuration) is left down after ``RESTARTS_PER_MIN``
restarts in a minute. The process - never the GPU owner - forks the front ends: no process with a GPU
context starts another program. It exits when the owner is gone, on SIGTERM / SIGINT (terminating the
front ends), or with status 3 when every front end is down for good (the owner then stops).
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import threading
import time

from ..config import Config
from ..utils.logging import get_logger, setup

log = get_logger("deconv_api_amd.supervisor")

RESTARTS_PER_MIN = 5


def spawn_frontend(cfg: Config, path: str, i: int) -> subprocess.Popen:
    env = dict(os.environ, DV_HOST=cfg.host, DV_PORT=str(cfg.port))
    return subprocess.Popen([sys.executable, "-m", "deconv_api_amd.serve.frontend", "--sock", path,
                             "--index", str(i)], env=env)


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


def supervise(cfg: Config, path: str, fes: list, history: dict, now: float, can_restart: bool) -> bool:
    """One pass: restart front ends that exited (bounded per minute). False when all are down for good."""
    alive = False
    for i, p in enumerate(fes):
        if p.poll() is None:
            alive = True
            continue
        if not can_restart:
            continue
        recent = [t for t in history.get(i, []) if now - t < 60.0]
        history[i] = recent
        if len(recent) >= RESTARTS_PER_MIN:
            continue
        log.warning("front end exited, restarting", extra={"fields": {"index": i, "code": p.returncode,
                                                                    "restarts_last_min": len(recent)}})
        fes[i] = spawn_frontend(cfg, path, i)
        recent.append(now)
        alive = True
    return alive


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sock", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--owner-pid", type=int, required=True)
    ap.add_argument("--poll", type=float, default=0.5)
    a = ap.parse_args(argv)
    cfg = Config.from_env()
    setup(cfg.log_json)
    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    fes = [spawn_frontend(cfg, a.sock, i) for i in range(a.n)]
    history: dict = {}
    code = 0
    try:
        while not stop.wait(a.poll):
            owner = _alive(a.owner_pid)
            if not owner:
                log.info("GPU owner gone, stopping front ends", extra={"fields": {"owner_pid": a.owner_pid}})
                break
            # restart only while the owner is serving (its socket exists: it unlinks it when it closes)
            if not supervise(cfg, a.sock, fes, history, time.monotonic(), os.path.exists(a.sock)):
                log.error("every front end is down", extra={"fields": {"codes": [p.returncode for p in fes]}})
                code = 3
                break
    finally:
        for p in fes:
            if p.poll() is None:
                p.terminate()
        for p in fes:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return code


if __name__ == "__main__":
    sys.exit(main())
