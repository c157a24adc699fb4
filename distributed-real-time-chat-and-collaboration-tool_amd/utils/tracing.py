"""Tracing: roctx ranges + an in-process span recorder (SURVEY §5 "Tracing").

The reference has no tracing (an unused ``PerformanceLogger``,
utils/logger_config.py:102-123).  Here:

* ``span(name)`` marks a region.  With ``DRTC_TRACE=1`` it pushes a roctx
  range (``torch.cuda.nvtx`` is roctx on ROCm), so ``rocprofv3
  --marker-trace`` shows engine steps, graph replays and RPC handlers on the
  same timeline as the HIP kernels; and it records the span (name, thread,
  start, duration) into a bounded ring buffer that ``dump_chrome_trace``
  writes as Chrome/Perfetto ``traceEvents`` JSON - tracing with no profiler
  attached.
* With tracing off a span costs one global flag check.
"""
from __future__ import annotations

import collections
import functools
import json
import os
import threading
import time
from contextlib import contextmanager

_enabled = os.environ.get("DRTC_TRACE", "0") not in ("", "0")
_lock = threading.Lock()
_events: collections.deque = collections.deque(maxlen=int(os.environ.get("DRTC_TRACE_EVENTS",
                                                                          "200000")))
_t0 = time.perf_counter()
_nvtx = None


def _roctx():
    global _nvtx
    if _nvtx is None:
        try:
            import torch

            _nvtx = torch.cuda.nvtx
        except Exception:  # pragma: no cover - torch always present here
            _nvtx = False
    return _nvtx


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = on


def enabled() -> bool:
    return _enabled


@contextmanager
def span(name: str, **args):
    if not _enabled:
        yield
        return
    nv = _roctx()
    if nv:
        nv.range_push(name)
    t = time.perf_counter()
    try:
        yield
    finally:
        dur = time.perf_counter() - t
        if nv:
            nv.range_pop()
        ev = {"name": name, "ph": "X", "ts": (t - _t0) * 1e6, "dur": dur * 1e6,
              "pid": os.getpid(), "tid": threading.get_ident()}
        if args:
            ev["args"] = args
        with _lock:
            _events.append(ev)


def traced(name: str | None = None):
    """Decorator form of :func:`span`."""
    def deco(fn):
        label = name or fn.__qualname__

        @functools.wraps(fn)
        def wrapper(*a, **kw):
            if not _enabled:
                return fn(*a, **kw)
            with span(label):
                return fn(*a, **kw)
        return wrapper
    return deco


def events() -> list[dict]:
    with _lock:
        return list(_events)


def clear() -> None:
    with _lock:
        _events.clear()


def dump_chrome_trace(path: str) -> int:
    """Write the recorded spans as Chrome trace JSON; returns the span count."""
    ev = events()
    with open(path, "w") as f:
        json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
    return len(ev)
