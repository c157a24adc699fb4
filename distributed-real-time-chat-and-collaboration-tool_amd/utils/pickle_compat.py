"""Byte-compatible pickle I/O for the reference's on-disk formats.

Writers pin protocol 4 (the default of the CPython 3.8-3.13 interpreters the
reference ran on).  Readers NEVER execute code from a file: ``safe_load``
uses an Unpickler whose ``find_class`` only admits the plain data types the
formats contain (datetime/timezone/timedelta, set/frozenset, and the
``_codecs.encode`` shim older protocols use for bytes).  A file naming any
other global is rejected with ``pickle.UnpicklingError``.
"""
from __future__ import annotations

import io
import os
import pickle
import tempfile

PROTOCOL = 4

_ALLOWED = {
    ("datetime", "datetime"), ("datetime", "date"), ("datetime", "time"),
    ("datetime", "timedelta"), ("datetime", "timezone"),
    ("builtins", "set"), ("builtins", "frozenset"), ("builtins", "bytearray"),
    ("_codecs", "encode"), ("collections", "OrderedDict"),
}


class SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name}")


def safe_loads(data: bytes):
    return SafeUnpickler(io.BytesIO(data)).load()


def safe_load(path: str):
    with open(path, "rb") as f:
        return SafeUnpickler(f).load()


def _fsync_dir(d: str) -> None:
    fd = os.open(d, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


def dump(obj, path: str, fsync: bool = False) -> None:
    """Atomic write (temp file + rename) of ``pickle.dumps(obj, protocol=4)``."""
    write_bytes(pickle.dumps(obj, protocol=PROTOCOL), path, fsync)


def write_bytes(data: bytes, path: str, fsync: bool = False) -> None:
    """Atomic write (temp file + rename) of already-pickled bytes: lets a caller
    pickle under its lock (a consistent image) and do the file I/O outside it."""
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix=".tmp_", suffix=".pkl")
    try:
        with os.fdopen(fd, "wb") as f:
            f.write(data)
            if fsync:
                f.flush()
                os.fsync(f.fileno())
        os.replace(tmp, path)
        if fsync:
            _fsync_dir(d)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise
