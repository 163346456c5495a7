"""Minimal Prometheus text-format metrics (no client library dependency; the reference pins
prometheus-client but never imports it, app/requirements.txt:79)."""
from __future__ import annotations

import threading
import time
from collections import defaultdict
from typing import Dict, Iterable, Tuple

DEFAULT_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1.0, 2.5, 5.0, 10.0, 30.0)


def _labels(d: Tuple[Tuple[str, str], ...]) -> str:
    if not d:
        return ""
    return "{" + ",".join(f'{k}="{v}"' for k, v in d) + "}"


class Counter:
    def __init__(self, name: str, help_: str):
        self.name, self.help = name, help_
        self.values: Dict[tuple, float] = defaultdict(float)
        self.lock = threading.Lock()

    def inc(self, v: float = 1.0, **labels):
        with self.lock:
            self.values[tuple(sorted(labels.items()))] += v

    def render(self) -> Iterable[str]:
        yield f"# HELP {self.name} {self.help}"
        yield f"# TYPE {self.name} counter"
        for k, v in sorted(self.values.items()):
            yield f"{self.name}{_labels(k)} {v}"


class Gauge(Counter):
    def set(self, v: float, **labels):
        with self.lock:
            self.values[tuple(sorted(labels.items()))] = v

    def render(self):
        yield f"# HELP {self.name} {self.help}"
        yield f"# TYPE {self.name} gauge"
        for k, v in sorted(self.values.items()):
            yield f"{self.name}{_labels(k)} {v}"


class Histogram:
    def __init__(self, name: str, help_: str, buckets=DEFAULT_BUCKETS):
        self.name, self.help, self.buckets = name, help_, tuple(buckets)
        self.counts: Dict[tuple, list] = {}
        self.sums: Dict[tuple, float] = defaultdict(float)
        self.lock = threading.Lock()

    def observe(self, v: float, **labels):
        k = tuple(sorted(labels.items()))
        with self.lock:
            c = self.counts.setdefault(k, [0] * (len(self.buckets) + 1))
            for i, b in enumerate(self.buckets):
                if v <= b:
                    c[i] += 1
            c[-1] += 1
            self.sums[k] += v

    def quantile(self, q: float, **labels) -> float:
        """Bucket-resolution quantile estimate (upper bound of the bucket)."""
        k = tuple(sorted(labels.items()))
        c = self.counts.get(k)
        if not c or c[-1] == 0:
            return 0.0
        target = q * c[-1]
        for i, b in enumerate(self.buckets):
            if c[i] >= target:
                return b
        return float("inf")

    def render(self):
        yield f"# HELP {self.name} {self.help}"
        yield f"# TYPE {self.name} histogram"
        for k, c in sorted(self.counts.items()):
            for i, b in enumerate(self.buckets):
                yield f"{self.name}_bucket{_labels(k + (('le', str(b)),))} {c[i]}"
            yield f"{self.name}_bucket{_labels(k + (('le', '+Inf'),))} {c[-1]}"
            yield f"{self.name}_sum{_labels(k)} {self.sums[k]}"
            yield f"{self.name}_count{_labels(k)} {c[-1]}"


class Registry:
    def __init__(self):
        self.metrics = []
        self.start = time.time()

    def counter(self, name, help_):
        m = Counter(name, help_)
        self.metrics.append(m)
        return m

    def gauge(self, name, help_):
        m = Gauge(name, help_)
        self.metrics.append(m)
        return m

    def histogram(self, name, help_, buckets=DEFAULT_BUCKETS):
        m = Histogram(name, help_, buckets)
        self.metrics.append(m)
        return m

    def render(self) -> str:
        lines = [f"# HELP dv_uptime_seconds process uptime", "# TYPE dv_uptime_seconds gauge",
                 f"dv_uptime_seconds {time.time() - self.start:.3f}"]
        for m in self.metrics:
            lines.extend(m.render())
        return "\n".join(lines) + "\n"


def merge_text(local: str, remote: str) -> str:
    """Union of two Prometheus text renders (a front-end process and its GPU owner, serve/ingest.py):
    one HELP/TYPE header per metric, the local sample when both processes have the same series.
    Each process only populates its own metrics (HTTP counters in the front end, batch / GPU
    stage histograms in the owner), so the union is the whole picture of one front end."""
    def blocks(txt):
        out, cur = {}, None
        for line in txt.splitlines():
            if line.startswith("# HELP "):
                cur = line.split()[2]
                out.setdefault(cur, ([], {}))[0].append(line)
            elif line.startswith("# TYPE ") and cur is not None:
                out[cur][0].append(line)
            elif line and cur is not None:
                out[cur][1].setdefault(line.rsplit(" ", 1)[0], line)
        return out

    a, b = blocks(local), blocks(remote)
    lines = []
    for name in list(a) + [n for n in b if n not in a]:
        head, samples = a.get(name) or b[name]
        merged = dict(samples)
        for k, v in (b.get(name, ([], {}))[1]).items():
            merged.setdefault(k, v)
        lines.extend(head)
        lines.extend(merged.values())
    return "\n".join(lines) + "\n"


REGISTRY = Registry()
REQUESTS = REGISTRY.counter("dv_requests_total", "HTTP requests by route and status")
LATENCY = REGISTRY.histogram("dv_request_latency_seconds", "request latency by route and layer")
BATCH_SIZE = REGISTRY.histogram("dv_batch_size", "images per engine batch",
                                buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512))
ENGINE_TIME = REGISTRY.histogram("dv_engine_seconds", "engine time per batch by stage")
QUEUE_DEPTH = REGISTRY.gauge("dv_queue_depth", "pending requests in the batcher")
IMAGES = REGISTRY.counter("dv_images_total", "images processed by the engine")
STAGE_TIME = REGISTRY.histogram("dv_stage_seconds", "per-batch GPU stage time from hipEvents (h2d, compute, d2h)",
                                (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 1.0))
HOST_STAGE = REGISTRY.histogram("dv_host_stage_seconds",
                                "per-request host stage time: parse, decode (front end / codec pool), ipc, "
                                "queue (batcher wait), gpu (launch -> results on the host), encode (-> data URL)",
                                (0.0005, 0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 1.0))
