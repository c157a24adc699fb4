"""Loader for the in-tree HIP kernel module (``_hipk``).

Policy: a GPU tensor always goes through the HIP kernel.  If the extension is
missing or fails to load on a machine with a GPU, the op raises - there is no
silent eager fallback on the device path.  CPU tensors use the PyTorch
reference implementations (the numerics oracle the GPU tests compare to).
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def hipk():
    """Return the loaded ``_hipk`` module (building it in-tree if absent)."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        try:
            pkg = __name__.rsplit(".", 2)[0]
            try:
                m = importlib.import_module(pkg + "._hipk")
            except ImportError:
                if os.environ.get("DRTC_NO_AUTOBUILD"):
                    raise
                from .. import _build

                _build.build_hip()
                m = importlib.import_module(pkg + "._hipk")
            rc = m.configure()
            if rc != 0 and torch.cuda.is_available():
                raise RuntimeError(f"_hipk.configure() failed with code {rc}")
            _mod = m
        except Exception as e:  # pragma: no cover - exercised on broken installs
            _err = e
            raise RuntimeError(
                "drtc_amd HIP kernels are unavailable; build them with "
                "`python -m drtc_amd._build` (hipcc --offload-arch=gfx950)"
            ) from e
    return _mod


def stream_ptr(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"HIP kernel {name} failed (code {rc})")


def ptr(t: torch.Tensor | None) -> int:
    return 0 if t is None else t.data_ptr()


_force_ref = threading.local()


def on_gpu(t: torch.Tensor) -> bool:
    """True when ``t`` must take the HIP-kernel path."""
    return t.is_cuda and not getattr(_force_ref, "on", False)


class reference_mode:
    """Context manager: run the PyTorch reference implementations even for
    GPU tensors (numerics oracle for end-to-end GPU tests)."""

    def __enter__(self):
        self._prev = getattr(_force_ref, "on", False)
        _force_ref.on = True
        return self

    def __exit__(self, *exc):
        _force_ref.on = self._prev
        return False
