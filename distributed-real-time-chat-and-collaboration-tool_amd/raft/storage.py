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

Log compaction (opt-in; the reference has none): ``raft_snapshot_port_{port}.pkl``
holds ``{'index', 'term', 'data'}`` (the state-machine image at ``index``) and
is written first; the native log then moves to a new segment file
``raft_log_port_{port}.b{index+1}.seg`` holding only the entries after it, and
older segments are deleted.  A crash between the steps leaves an older segment
whose covered prefix is skipped on load, so every ordering recovers.  With
compaction the exported reference-format log pickle holds the suffix only;
``PickleStorage`` (the reference's exact format) does not compact.
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


class _SnapshotFile:
    def __init__(self, path: str, fsync: bool):
        self.path, self.fsync = path, fsync

    def load(self):
        if not os.path.exists(self.path):
            return None
        d = pickle_compat.safe_load(self.path)
        return int(d["index"]), int(d["term"]), bytes(d["data"])

    def save(self, index: int, term: int, data: bytes) -> None:
        pickle_compat.dump({"index": index, "term": term, "data": data}, self.path, self.fsync)


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

    # The reference format is one whole-log list with implicit 0-based
    # indices; it cannot express a compacted prefix crash-safely, so log
    # compaction / InstallSnapshot need NativeStorage (--storage native).
    def latest_snapshot(self):
        return None

    def compact(self, index, term, data) -> None:
        raise NotImplementedError("log compaction requires native storage")

    def install_snapshot(self, index, term, data, keep) -> None:
        raise NotImplementedError("InstallSnapshot requires native storage")

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
        self.port = port
        self.fsync = fsync
        self.log_path = os.path.join(directory, f"raft_log_port_{port}.pkl")
        self.state = _StateFile(os.path.join(directory, f"raft_state_port_{port}.pkl"), fsync)
        self.snap = _SnapshotFile(os.path.join(directory, f"raft_snapshot_port_{port}.pkl"), fsync)
        pkg = __name__.rsplit(".", 2)[0]
        self._native = importlib.import_module(pkg + "._native")
        segs = self._segments()
        fresh = not segs
        self.base = segs[-1][0] if segs else 0
        self.seg_path = segs[-1][1] if segs else self._seg_name(0)
        self.store = self._native.LogStore(self.seg_path, fsync)
        for _, old in segs[:-1]:  # leftovers of an interrupted compaction
            os.unlink(old)
        self.entries: list[Entry] = []
        if fresh and os.path.exists(self.log_path):  # migrate a reference data dir
            for e in _load_ref_log(self.log_path):
                self.store.append(e.term, e.command, e.data)

    def _seg_name(self, base: int) -> str:
        tail = ".seg" if base == 0 else f".b{base}.seg"
        return os.path.join(self.dir, f"raft_log_port_{self.port}{tail}")

    def _segments(self) -> list[tuple[int, str]]:
        pre = f"raft_log_port_{self.port}"
        out = []
        for f in os.listdir(self.dir):
            if not (f.startswith(pre) and f.endswith(".seg")):
                continue
            mid = f[len(pre):-len(".seg")]
            if mid == "":
                out.append((0, os.path.join(self.dir, f)))
            elif mid.startswith(".b") and mid[2:].isdigit():
                out.append((int(mid[2:]), os.path.join(self.dir, f)))
        return sorted(out)

    def load(self):
        st = self.state.load()
        snap = self.snap.load()
        st["snap_index"], st["snap_term"] = (snap[0], snap[1]) if snap else (-1, 0)
        skip = st["snap_index"] + 1 - self.base  # entries the snapshot already covers
        self.entries = []
        for i in range(max(0, skip), self.store.size()):
            t, c, d = self.store.get(i)
            self.entries.append(Entry(int(t), c, bytes(d)))
        if skip > 0:  # finish an interrupted compaction
            self._rewrite(st["snap_index"] + 1, self.entries)
        return st, list(self.entries)

    def append(self, entries) -> None:
        for e in entries:
            self.store.append(e.term, e.command, e.data)
        self.entries.extend(entries)

    def truncate_from(self, index: int) -> None:
        self.store.truncate_from(index - self.base)
        del self.entries[index - self.base:]

    def _rewrite(self, base: int, entries) -> None:
        """Move the log to a fresh segment starting at absolute index ``base``."""
        path = self._seg_name(base)
        tmp = path + ".tmp"
        if os.path.exists(tmp):
            os.unlink(tmp)
        st = self._native.LogStore(tmp, self.fsync)
        for e in entries:
            st.append(e.term, e.command, e.data)
        st.sync()
        st.close()
        os.replace(tmp, path)
        old = self.seg_path
        self.store.close()
        self.store = self._native.LogStore(path, self.fsync)
        self.seg_path, self.base = path, base
        self.entries = list(entries)
        if old != path and os.path.exists(old):
            os.unlink(old)

    def latest_snapshot(self):
        return self.snap.load()

    def compact(self, index: int, term: int, data: bytes | None) -> None:
        self.snap.save(index, term, data)  # durable image first
        self._rewrite(index + 1, self.entries[index + 1 - self.base:])

    def install_snapshot(self, index: int, term: int, data: bytes, keep) -> None:
        self.snap.save(index, term, data)
        self._rewrite(index + 1, list(keep))

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
