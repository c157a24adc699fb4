"""Durable Raft storage, on-disk compatible with the reference.

Layout: ``<base>/raft_node_{id}_data/`` (server/raft_node.py:100-105)
  raft_state_port_{port}.pkl   {'current_term','voted_for','commit_index','last_applied'}
  raft_log_port_{port}.pkl     [{'term','command','data'(bytes)}, ...]   (reference log)
  raft_log_port_{port}.seg     native append-only CRC log (NativeStorage only)
  users.pkl / channels.pkl / messages.pkl / direct_messages.pkl   app state

``NativeStorage`` (default) appends each entry to the C++ LogStore
(csrc/runtime/log_store.cpp) and rewrites the reference-format log pickle
only on ``export()`` (periodically from the runtime's persister, on
snapshots and at clean shutdown), instead of on every write (survey quirk
Q5).  ``PickleStorage`` reproduces the reference exactly (whole-log pickle
per append).  Either imports a reference data dir.

Durability (``fsync=True``, the server default): a batch of appended entries
is made durable with ONE fdatasync before the append returns (group commit:
an AppendEntries batch or a leader proposal is acknowledged only after it),
and a change of ``current_term`` / ``voted_for`` is fsynced (file + directory)
before a vote is answered.  ``commit_index`` / ``last_applied`` are
recomputable and written without a sync.  NativeStorage keeps the hard state
(term, vote) in a file of its own, ``raft_hardstate_port_{port}.pkl``, rewritten
(and fsynced) only when it changes: the reference-format state pickle, which is
also rewritten on every commit_index change without a sync, can then come back
empty or stale after a power loss without undoing a vote (the term and vote are
taken from the hard-state file when it is at least as new).

Crash consistency of the reference-format PAIR: the state pickle is written
on every state change but its ``commit_index`` / ``last_applied`` are
clamped to the last index present in the exported log pickle (recorded in
``raft_log_port_{port}.exported``), so after a crash at any point the pair
on disk never claims a commit beyond the log it holds - a reference node
booting from it replays a consistent committed prefix (the app-state
pickles, which it loads afterwards, carry the rest).

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
            try:
                st.update(pickle_compat.safe_load(self.path))
            except Exception:  # torn / empty after a crash: the hard state lives elsewhere
                pass
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

    def export_begin(self):
        return None  # the log pickle is rewritten on every append already

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
        self.export_path = os.path.join(directory, f"raft_log_port_{port}.exported")
        self.state = _StateFile(os.path.join(directory, f"raft_state_port_{port}.pkl"), fsync)
        self.hard_path = os.path.join(directory, f"raft_hardstate_port_{port}.pkl")
        self.snap = _SnapshotFile(os.path.join(directory, f"raft_snapshot_port_{port}.pkl"), fsync)
        pkg = __name__.rsplit(".", 2)[0]
        self._native = importlib.import_module(pkg + "._native")
        segs = self._segments()
        fresh = not segs
        self.base = segs[-1][0] if segs else 0
        self.seg_path = segs[-1][1] if segs else self._seg_name(0)
        # per-entry syncs off: append() syncs once per batch (group commit)
        self.store = self._native.LogStore(self.seg_path, False)
        for _, old in segs[:-1]:  # leftovers of an interrupted compaction
            os.unlink(old)
        self.entries: list[Entry] = []
        self._state: dict = {}
        self._durable = (None, None)  # (term, voted_for) last fsynced
        self._trunc_floor = 1 << 62
        self.exported_last = self._read_exported()
        if fresh and os.path.exists(self.log_path):  # migrate a reference data dir
            ref = _load_ref_log(self.log_path)
            for e in ref:
                self.store.append(e.term, e.command, e.data)
            self.store.sync()
            self.exported_last = len(ref) - 1
            self._write_exported()

    # -- the exported reference-format log: last absolute index it holds
    def _read_exported(self) -> int:
        try:
            with open(self.export_path) as f:
                return int(f.read().strip() or -1)
        except (OSError, ValueError):
            return -1

    def _write_exported(self) -> None:
        tmp = self.export_path + ".tmp"
        with open(tmp, "w") as f:
            f.write(str(self.exported_last))
            if self.fsync:
                f.flush()
                os.fsync(f.fileno())
        os.replace(tmp, self.export_path)

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

    def _load_hard(self):
        if not os.path.exists(self.hard_path):
            return None
        try:
            d = pickle_compat.safe_load(self.hard_path)
            return int(d["current_term"]), d["voted_for"]
        except Exception:  # never fsync-acknowledged if torn: the previous vote stands
            return None

    def load(self):
        st = self.state.load()
        hard = self._load_hard()
        if hard is not None and hard[0] >= int(st.get("current_term") or 0):
            st["current_term"], st["voted_for"] = hard
        snap = self.snap.load()
        st["snap_index"], st["snap_term"] = (snap[0], snap[1]) if snap else (-1, 0)
        skip = st["snap_index"] + 1 - self.base  # entries the snapshot already covers
        self.entries = []
        for i in range(max(0, skip), self.store.size()):
            t, c, d = self.store.get(i)
            self.entries.append(Entry(int(t), c, bytes(d)))
        if skip > 0:  # finish an interrupted compaction
            self._rewrite(st["snap_index"] + 1, self.entries)
        self._state = dict(st)
        # durable = what the fsynced hard-state file holds.  A data directory from before that
        # file existed (term / vote only in the state pickle, which save_state now rewrites
        # without fsync) has none: leave _durable unset so the first save_state writes and
        # fsyncs the hard state before the unsynced pickle rewrite could tear the only copy
        if hard is not None and (st.get("current_term"), st.get("voted_for")) == hard:
            self._durable = hard
        else:
            self._durable = (None, None)
        return st, list(self.entries)

    def append(self, entries) -> None:
        for e in entries:
            self.store.append(e.term, e.command, e.data)
        if self.fsync:
            self.store.sync()  # one fdatasync per batch, before the caller acknowledges
        self.entries.extend(entries)

    def truncate_from(self, index: int) -> None:
        self.store.truncate_from(index - self.base)
        if self.fsync:
            self.store.sync()
        del self.entries[index - self.base:]
        self._trunc_floor = min(self._trunc_floor, index)
        if self.exported_last >= index:
            # the exported pickle now holds replaced (uncommitted) entries past
            # index - 1: never let the reference state point into them
            self.exported_last = index - 1
            self._write_exported()

    def _rewrite(self, base: int, entries) -> None:
        """Move the log to a fresh segment starting at absolute index ``base``."""
        path = self._seg_name(base)
        tmp = path + ".tmp"
        if os.path.exists(tmp):
            os.unlink(tmp)
        st = self._native.LogStore(tmp, False)
        for e in entries:
            st.append(e.term, e.command, e.data)
        st.sync()
        st.close()
        os.replace(tmp, path)
        old = self.seg_path
        self.store.close()
        self.store = self._native.LogStore(path, False)
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
        self._state.update(state)
        st = self._state
        clamp = self.exported_last
        ref = {"current_term": st["current_term"], "voted_for": st["voted_for"],
               "commit_index": min(int(st["commit_index"]), clamp),
               "last_applied": min(int(st["last_applied"]), clamp)}
        hard = (st["current_term"], st["voted_for"])
        if hard != self._durable:  # term / vote changed: durable before the vote is answered
            pickle_compat.dump({"current_term": hard[0], "voted_for": hard[1]}, self.hard_path,
                               self.fsync)
            self._durable = hard
        pickle_compat.dump(ref, self.state.path, False)

    # -- export of the reference-format log, in three steps so the runtime can
    # pickle a large log outside its consensus lock
    def export_begin(self):
        """Under the consensus lock: (base, entries) to write, or None."""
        last = self.base + len(self.entries) - 1
        if last == self.exported_last and os.path.exists(self.log_path):
            return None
        self._trunc_floor = last + 1  # lowest index truncated while the export runs
        return self.base, list(self.entries)

    def export_write(self, snapshot) -> int:
        """Any thread: write the log pickle; returns the last index written."""
        base, entries = snapshot
        _dump_ref_log(entries, self.log_path, self.fsync)
        return base + len(entries) - 1

    def export_end(self, last: int) -> None:
        """Under the consensus lock: record the export, re-clamp the state."""
        # a truncation while the pickle was being written invalidates it
        # from the truncation point on (entries there may have been replaced)
        last = min(last, self._trunc_floor - 1, self.base + len(self.entries) - 1)
        self.exported_last = last
        self._write_exported()
        if self._state:
            self.save_state({})

    def export(self) -> None:
        """Write the reference-format log pickle and the matching state."""
        snap = self.export_begin()
        if snap is not None:
            self.export_end(self.export_write(snap))

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
