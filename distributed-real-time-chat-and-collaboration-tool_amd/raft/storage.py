"""Durable Raft storage, on-disk compatible with the reference.

Layout: ``<base>/raft_node_{id}_data/`` (server/raft_node.py:100-105)
  raft_state_port_{port}.pkl   {'current_term','voted_for','commit_index','last_applied'}
  raft_log_port_{port}.pkl     [{'term','command','data'(bytes)}, ...]   (reference log)
  raft_log_port_{port}.seg     native append-only CRC log (NativeStorage only)
  users.pkl / channels.pkl / messages.pkl / direct_messages.pkl   app state

``NativeStorage`` (default) appends each entry to the C++ LogStore
(csrc/runtime/log_store.cpp) and rewrites the reference-format log pickle
only on ``export()`` (snapshots, clean shutdown), instead of on every write
(survey quirk Q5).  ``PickleStorage`` reproduces the reference exactly
(whole-log pickle per append).  Either imports a reference data dir.
"""
from __future__ import annotations

import importlib
import os

from ..utils import pickle_compat
from .core import Entry


def data_dir(base: str, node_id: int) -> str:
    return os.path.join(base, f"raft_node_{node_id}_data")


class _StateFile:
    def __init__(self, path: str, fsync: bool):
        self.path = path
        self.fsync = fsync

    def load(self) -> dict:
        st = {"current_term": 0, "voted_for": None, "commit_index": -1, "last_applied": -1}
        if os.path.exists(self.path):
            st.update(pickle_compat.safe_load(self.path))
        return st

    def save(self, state: dict) -> None:
        pickle_compat.dump({"current_term": state["current_term"], "voted_for": state["voted_for"],
                            "commit_index": state["commit_index"],
                            "last_applied": state["last_applied"]}, self.path, self.fsync)


def _load_ref_log(path: str) -> list[Entry]:
    if not os.path.exists(path):
        return []
    return [Entry(int(d["term"]), str(d["command"]), bytes(d["data"]))
            for d in pickle_compat.safe_load(path)]


def _dump_ref_log(entries, path: str, fsync: bool) -> None:
    pickle_compat.dump([{"term": e.term, "command": e.command, "data": e.data} for e in entries],
                       path, fsync)


class PickleStorage:
    """The reference's storage behaviour, byte for byte."""

    def __init__(self, directory: str, port: int, fsync: bool = False):
        os.makedirs(directory, exist_ok=True)
        self.dir = directory
        self.log_path = os.path.join(directory, f"raft_log_port_{port}.pkl")
        self.state = _StateFile(os.path.join(directory, f"raft_state_port_{port}.pkl"), fsync)
        self.fsync = fsync
        self.entries: list[Entry] = []

    def load(self):
        self.entries = _load_ref_log(self.log_path)
        return self.state.load(), list(self.entries)

    def append(self, entries) -> None:
        self.entries.extend(entries)
        _dump_ref_log(self.entries, self.log_path, self.fsync)

    def truncate_from(self, index: int) -> None:
        del self.entries[index:]
        _dump_ref_log(self.entries, self.log_path, self.fsync)

    def save_state(self, state: dict) -> None:
        self.state.save(state)

    def export(self) -> None:
        pass

    def flush(self) -> None:
        pass

    def close(self) -> None:
        pass


class NativeStorage:
    def __init__(self, directory: str, port: int, fsync: bool = False):
        os.makedirs(directory, exist_ok=True)
        self.dir = directory
        self.seg_path = os.path.join(directory, f"raft_log_port_{port}.seg")
        self.log_path = os.path.join(directory, f"raft_log_port_{port}.pkl")
        self.state = _StateFile(os.path.join(directory, f"raft_state_port_{port}.pkl"), fsync)
        pkg = __name__.rsplit(".", 2)[0]
        native = importlib.import_module(pkg + "._native")
        fresh = not os.path.exists(self.seg_path)
        self.store = native.LogStore(self.seg_path, fsync)
        self.entries: list[Entry] = []
        if fresh and os.path.exists(self.log_path):  # migrate a reference data dir
            for e in _load_ref_log(self.log_path):
                self.store.append(e.term, e.command, e.data)

    def load(self):
        self.entries = []
        for i in range(self.store.size()):
            t, c, d = self.store.get(i)
            self.entries.append(Entry(int(t), c, bytes(d)))
        return self.state.load(), list(self.entries)

    def append(self, entries) -> None:
        for e in entries:
            self.store.append(e.term, e.command, e.data)
        self.entries.extend(entries)

    def truncate_from(self, index: int) -> None:
        self.store.truncate_from(index)
        del self.entries[index:]

    def save_state(self, state: dict) -> None:
        self.state.save(state)

    def export(self) -> None:
        """Write the reference-format log pickle (for tools / the reference)."""
        _dump_ref_log(self.entries, self.log_path, False)

    def flush(self) -> None:
        self.store.sync()

    def close(self) -> None:
        self.store.close()


def open_storage(kind: str, directory: str, port: int, fsync: bool = False):
    if kind == "pickle":
        return PickleStorage(directory, port, fsync)
    if kind == "native":
        return NativeStorage(directory, port, fsync)
    raise ValueError(f"unknown storage kind {kind!r}")
