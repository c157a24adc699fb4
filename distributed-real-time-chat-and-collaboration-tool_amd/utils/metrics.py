"""Process-wide metrics registry: counters and latency histograms.

The reference has only ad-hoc log lines (SURVEY §5 "Metrics"); every server
here records RPC latencies, Raft proposals, engine tokens/s, TTFT/TPOT and
KV occupancy into this registry, which the bench harness and the
``status`` RPCs dump.  Histograms keep a bounded reservoir so percentiles
(p50/p99) are exact up to ``reservoir`` samples and sampled beyond.
"""
from __future__ import annotations

import random
import threading
import time
from collections import defaultdict
from contextlib import contextmanager


class Histogram:
    def __init__(self, reservoir: int = 8192):
        self.n = 0
        self.total = 0.0
        self.min = float("inf")
        self.max = float("-inf")
        self.samples: list[float] = []
        self.reservoir = reservoir
        self._rng = random.Random(0)

    def observe(self, v: float) -> None:
        self.n += 1
        self.total += v
        self.min = min(self.min, v)
        self.max = max(self.max, v)
        if len(self.samples) < self.reservoir:
            self.samples.append(v)
        else:
            j = self._rng.randrange(self.n)
            if j < self.reservoir:
                self.samples[j] = v

    def percentile(self, q: float) -> float:
        if not self.samples:
            return 0.0
        s = sorted(self.samples)
        k = min(len(s) - 1, max(0, int(round(q / 100.0 * (len(s) - 1)))))
        return s[k]

    def summary(self) -> dict:
        return {"count": self.n, "mean": self.total / self.n if self.n else 0.0,
                "p50": self.percentile(50), "p99": self.percentile(99),
                "min": self.min if self.n else 0.0, "max": self.max if self.n else 0.0}


class Registry:
    def __init__(self):
        self._lock = threading.Lock()
        self.counters: dict[str, float] = defaultdict(float)
        self.gauges: dict[str, float] = {}
        self.hists: dict[str, Histogram] = {}

    def inc(self, name: str, v: float = 1.0) -> None:
        with self._lock:
            self.counters[name] += v

    def set_gauge(self, name: str, v: float) -> None:
        with self._lock:
            self.gauges[name] = v

    def observe(self, name: str, v: float) -> None:
        with self._lock:
            h = self.hists.get(name)
            if h is None:
                h = self.hists[name] = Histogram()
            h.observe(v)

    def observe_many(self, name: str, values) -> None:
        """Record a batch of observations under one lock acquisition."""
        with self._lock:
            h = self.hists.get(name)
            if h is None:
                h = self.hists[name] = Histogram()
            for v in values:
                h.observe(v)

    @contextmanager
    def timer(self, name: str):
        t = time.perf_counter()
        try:
            yield
        finally:
            self.observe(name, time.perf_counter() - t)

    def snapshot(self) -> dict:
        with self._lock:
            return {"counters": dict(self.counters), "gauges": dict(self.gauges),
                    "histograms": {k: h.summary() for k, h in self.hists.items()}}

    def reset(self) -> None:
        with self._lock:
            self.counters.clear()
            self.gauges.clear()
            self.hists.clear()


METRICS = Registry()
