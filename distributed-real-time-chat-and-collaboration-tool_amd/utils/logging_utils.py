"""Logging setup (the reference's utils/logger_config.py capabilities, used).

* ``setup_logging``: console (optionally coloured, component-tagged) and an
  optional file handler;
* ``ColoredFormatter``: ANSI level colours + a per-component tag;
* ``PerformanceLogger``: context manager that logs an operation's duration
  and warns above a threshold (default 1 s), also feeding the metrics
  registry.
"""
from __future__ import annotations

import logging
import sys
import time

from .metrics import METRICS

_COLORS = {"DEBUG": "\033[36m", "INFO": "\033[32m", "WARNING": "\033[33m",
           "ERROR": "\033[31m", "CRITICAL": "\033[35m"}
_RESET = "\033[0m"
_TAGS = {"raft": "[RAFT]", "server": "[SRV ]", "llm": "[LLM ]", "engine": "[GPU ]",
         "client": "[CLI ]", "parallel": "[RCCL]"}


class ColoredFormatter(logging.Formatter):
    def __init__(self, fmt: str | None = None, use_color: bool = True):
        super().__init__(fmt or "%(asctime)s %(tag)s %(levelname)s %(name)s: %(message)s",
                         datefmt="%H:%M:%S")
        self.use_color = use_color

    def format(self, record: logging.LogRecord) -> str:
        tag = ""
        for key, t in _TAGS.items():
            if f".{key}" in record.name or record.name.startswith(key):
                tag = t
                break
        record.tag = tag
        s = super().format(record)
        if self.use_color and record.levelname in _COLORS:
            return f"{_COLORS[record.levelname]}{s}{_RESET}"
        return s


def setup_logging(level: str | int = "INFO", log_file: str | None = None,
                  color: bool | None = None) -> logging.Logger:
    root = logging.getLogger()
    root.setLevel(level if isinstance(level, int) else getattr(logging, str(level).upper()))
    for h in list(root.handlers):
        root.removeHandler(h)
    sh = logging.StreamHandler(sys.stderr)
    sh.setFormatter(ColoredFormatter(use_color=sys.stderr.isatty() if color is None else color))
    root.addHandler(sh)
    if log_file:
        fh = logging.FileHandler(log_file)
        fh.setFormatter(ColoredFormatter(use_color=False))
        root.addHandler(fh)
    return root


class PerformanceLogger:
    def __init__(self, name: str, logger: logging.Logger | None = None, warn_s: float = 1.0):
        self.name = name
        self.log = logger or logging.getLogger("perf")
        self.warn_s = warn_s

    def __enter__(self):
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        dt = time.perf_counter() - self.t0
        METRICS.observe(f"perf.{self.name}", dt)
        if dt > self.warn_s:
            self.log.warning("%s took %.3fs", self.name, dt)
        else:
            self.log.debug("%s took %.3fs", self.name, dt)
        return False
