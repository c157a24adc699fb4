"""Raft node runtime: drives RaftCore over gRPC and applies to ChatState.

Threads and locks (the fix for survey quirks Q2/Q3):
  * ``core_lock`` guards RaftCore; it is held only for in-memory state
    transitions and the (append-only) log write, never across network I/O;
  * outgoing RPCs are asynchronous gRPC futures whose callbacks feed the
    replies back into the core under the lock;
  * ``state_lock`` guards the chat state machine (reads by RPC handlers,
    writes by the apply callback); order is always core_lock -> state_lock;
  * a timer thread ticks the core every ``tick`` seconds (elections,
    heartbeats, retries) and a persister thread snapshots dirty app state
    to the reference-format pickles.
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time

import grpc

from ..protos import RAFT_SERVICE, RAFT_SNAPSHOT_SERVICE, make_stub, raft_pb, raft_snap_pb
from .core import (NOOP, AppendReq, AppendResp, Entry, NotLeaderError, RaftConfig, RaftCore,
                   SnapshotReq, SnapshotResp, VoteReq, VoteResp)
from ..utils import pickle_compat
from .state_machine import ChatState
from .storage import data_dir, open_storage

log = logging.getLogger(__name__)

GRPC_OPTS = [
    ("grpc.max_send_message_length", 50 * 1024 * 1024),
    ("grpc.max_receive_message_length", 50 * 1024 * 1024),
    ("grpc.keepalive_time_ms", 10000),
    ("grpc.keepalive_timeout_ms", 5000),
    ("grpc.keepalive_permit_without_calls", True),
    ("grpc.http2.max_pings_without_data", 0),
]


def to_pb_entry(e: Entry):
    return raft_pb.LogEntry(term=e.term, command=e.command, data=e.data)


def from_pb_entry(p) -> Entry:
    return Entry(p.term, p.command, bytes(p.data))


class _Waiter:
    __slots__ = ("term", "event", "ok")

    def __init__(self, term):
        self.term = term
        self.event = threading.Event()
        self.ok = False


class RaftRuntime:
    def __init__(self, node_id: int, port: int, peers: dict, data_root: str = ".",
                 storage: str = "native", config: RaftConfig | None = None,
                 state: ChatState | None = None, fsync: bool = False, tick: float = 0.01,
                 persist_interval: float = 0.2, seed_defaults=None, snapshot_every: int = 0,
                 snapshot_chunk: int = 4 << 20, export_interval: float = 5.0):
        self.id = node_id
        self.port = port
        self.peers = {int(k): v for k, v in peers.items() if int(k) != node_id}
        self.dir = data_dir(data_root, node_id)
        os.makedirs(self.dir, exist_ok=True)
        self.storage = open_storage(storage, self.dir, port, fsync)
        self.state = state or ChatState()
        self.state_lock = threading.RLock()
        self._persist_lock = threading.Lock()
        self.core_lock = threading.RLock()
        self.tick_interval = tick
        self.persist_interval = persist_interval
        self.export_interval = export_interval  # reference-format log pickle refresh (s)
        self.waiters: dict[int, _Waiter] = {}
        self.apply_listeners = []
        if snapshot_every and storage != "native":
            raise ValueError("log compaction (snapshot_every) requires native storage")
        self.snapshot_every = snapshot_every
        self.snapshot_chunk = snapshot_chunk
        self._snap_rx: dict = {}        # (term, leader, index) -> bytearray being received
        self._snap_tx: set[int] = set()  # peers with a snapshot transfer in flight
        snap = self.storage.latest_snapshot()
        if snap is not None:
            # a Raft snapshot is the authoritative baseline; the log after it
            # is replayed below
            self.state.restore_image(snap[2])
        else:
            # app-state cache first (reference load order), defaults if empty
            self.state.load(self.dir)
            if not self.state.channels and seed_defaults is not None:
                seed_defaults(self.state)
        self.core = RaftCore(node_id, self.peers.keys(), self.storage, self._apply, config,
                             now=time.monotonic(), restore_fn=self._restore)
        # rebuild: replay every committed entry after the snapshot over the
        # cached state (apply is idempotent), so a cache that lags the log
        # loses nothing
        with self.core_lock:
            self.core.last_applied = self.core.snap_index
            self.core._apply()
        self.channels = {p: grpc.insecure_channel(a, options=GRPC_OPTS) for p, a in self.peers.items()}
        self.stubs = {p: make_stub(ch, RAFT_SERVICE) for p, ch in self.channels.items()}
        self.snap_stubs = {p: make_stub(ch, RAFT_SNAPSHOT_SERVICE) for p, ch in self.channels.items()}
        self.running = False
        self._threads = []

    # ------------------------------------------------------------ lifecycle
    def start(self) -> "RaftRuntime":
        self.running = True
        for fn, name in ((self._timer_loop, "raft-timer"), (self._persist_loop, "raft-persist")):
            t = threading.Thread(target=fn, name=f"{name}-{self.id}", daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self) -> None:
        self.running = False
        for t in self._threads:
            t.join(timeout=2)
        self.persist(all_files=True)
        with self.core_lock:
            self.storage.export()
            self.storage.close()
        for ch in self.channels.values():
            ch.close()

    def _timer_loop(self) -> None:
        while self.running:
            time.sleep(self.tick_interval)
            with self.core_lock:
                self.core.tick(time.monotonic())
                out = self.core.drain()
            self._send(out)
            if self.snapshot_every:
                self.maybe_compact()

    # ------------------------------------------------------------ snapshots
    def maybe_compact(self, force: bool = False) -> bool:
        """Snapshot the state machine at the applied index and compact the log
        once ``snapshot_every`` entries accumulated since the last snapshot.
        Runs under core_lock, so the image is exactly the state at
        last_applied (applies happen under the same lock)."""
        with self.core_lock:
            c = self.core
            if c.last_applied <= c.snap_index:
                return False
            if not force and c.last_applied - c.snap_index < self.snapshot_every:
                return False
            with self.state_lock:
                img = self.state.image()
            return c.compact(c.last_applied, img)

    def _restore(self, data: bytes) -> None:
        with self.state_lock:
            self.state.restore_image(data)

    def _send_snapshot(self, peer: int, req: SnapshotReq) -> None:
        """Stream the latest snapshot to ``peer`` in chunks (own thread)."""
        resp = None
        try:
            snap = self.storage.latest_snapshot()
            if snap is not None:
                idx, term, data = snap
                req = SnapshotReq(req.term, req.leader_id, idx, term)
                stub = self.snap_stubs[peer]
                n = len(data)
                off = 0
                while True:
                    chunk = data[off:off + self.snapshot_chunk]
                    done = off + len(chunk) >= n
                    r = stub.InstallSnapshot(raft_snap_pb.InstallSnapshotRequest(
                        term=req.term, leader_id=req.leader_id, last_included_index=idx,
                        last_included_term=term, offset=off, data=chunk, done=done, total_size=n),
                        timeout=max(self.core.cfg.rpc_timeout_append, 10.0))
                    if done or not r.success or r.term > req.term:
                        resp = SnapshotResp(r.term, r.success and done)
                        break
                    off += len(chunk)
        except grpc.RpcError:
            resp = None
        finally:
            with self.core_lock:
                self._snap_tx.discard(peer)
                self.core.now = time.monotonic()
                self.core.on_snapshot_reply(peer, req, resp)
                out = self.core.drain()
            self._send(out)

    def InstallSnapshot(self, request, context):
        """raft.RaftSnapshot/InstallSnapshot: reassemble chunks, then hand the
        whole image to the core."""
        key = (request.term, request.leader_id, request.last_included_index)
        with self.core_lock:
            c = self.core
            if request.term < c.term:
                return raft_snap_pb.InstallSnapshotResponse(term=c.term, success=False)
            c.now = time.monotonic()
            c.election_deadline = c.now + c._timeout()  # the leader is alive
            buf = self._snap_rx.get(key)
            if request.offset == 0:
                self._snap_rx = {key: bytearray()}  # a new transfer supersedes old ones
                buf = self._snap_rx[key]
            if buf is None or len(buf) != request.offset:
                return raft_snap_pb.InstallSnapshotResponse(term=c.term, success=False)
            buf += request.data
            if not request.done:
                return raft_snap_pb.InstallSnapshotResponse(term=c.term, success=True)
            del self._snap_rx[key]
            r = c.on_install_snapshot(SnapshotReq(request.term, request.leader_id,
                                                  request.last_included_index,
                                                  request.last_included_term, bytes(buf)))
            out = c.drain()
        self._send(out)
        return raft_snap_pb.InstallSnapshotResponse(term=r.term, success=r.success)

    def _persist_loop(self) -> None:
        last_export = time.monotonic()
        pause = self.persist_interval
        while self.running:
            time.sleep(pause)
            try:
                # the app-state pickles are a cache (the log is the source of truth):
                # under write load with a large state, pace them so that pickling under
                # the state lock takes at most ~5 % of the time
                held = self.persist()
                pause = max(self.persist_interval, 20.0 * held)
                if self.export_interval and time.monotonic() - last_export >= self.export_interval:
                    self.export_reference_log()
                    last_export = time.monotonic()
            except Exception:  # pragma: no cover - disk errors are logged, not fatal
                log.exception("persist failed")

    def export_reference_log(self) -> None:
        """Refresh the reference-format log pickle (raft_log_port_*.pkl) and the
        clamped state pickle; the O(log) pickling runs outside core_lock."""
        with self.core_lock:
            snap = self.storage.export_begin()
        if snap is None:
            return
        last = self.storage.export_write(snap)
        with self.core_lock:
            self.storage.export_end(last)

    def persist(self, all_files: bool = False) -> float:
        """Write the dirty (or all) app-state pickles.  They are pickled under the
        state lock (a consistent image) and written after it is released, so applies
        and reads wait for the pickling only, never for file I/O.  Returns the
        seconds the lock was held."""
        with self._persist_lock:  # writes land in the order their images were taken
            with self.state_lock:
                t0 = time.perf_counter()
                files = self.state.encode(self.dir, list(self.state.FILES) if all_files else None)
                held = time.perf_counter() - t0
            names = {os.path.join(self.dir, f): w for w, f in self.state.FILES.items()}
            for k, (path, data) in enumerate(files):
                try:
                    pickle_compat.write_bytes(data, path)
                except BaseException:
                    # disk full / I/O error: encode() marked these files clean, so mark
                    # this one and every one not yet written dirty again (the next persist
                    # retries them instead of leaving them stale until an unrelated change)
                    with self.state_lock:
                        for p2, _ in files[k:]:
                            if p2 in names:
                                self.state.dirty.add(names[p2])
                    raise
        return held

    # ------------------------------------------------------------ apply
    def _apply(self, index: int, e: Entry) -> None:
        if e.command != NOOP:
            try:
                data = json.loads(e.data.decode("utf-8"))
            except Exception:
                log.error("undecodable entry %d (%s)", index, e.command)
                data = None
            if data is not None:
                with self.state_lock:
                    try:
                        self.state.apply(e.command, data)
                    except Exception:
                        log.exception("apply of entry %d (%s) failed", index, e.command)
                for cb in self.apply_listeners:
                    cb(index, e.command, data)
        w = self.waiters.pop(index, None)
        if w is not None:
            w.ok = (w.term == e.term)
            w.event.set()

    # ------------------------------------------------------------ network
    def _send(self, out) -> None:
        for peer, kind, req in out:
            stub = self.stubs.get(peer)
            if stub is None:
                continue
            if kind == "snapshot":
                with self.core_lock:
                    if peer in self._snap_tx:
                        continue
                    self._snap_tx.add(peer)
                threading.Thread(target=self._send_snapshot, args=(peer, req),
                                 name=f"raft-snap-{self.id}->{peer}", daemon=True).start()
                continue
            if kind == "vote":
                pb = raft_pb.VoteRequest(term=req.term, candidate_id=req.candidate_id,
                                         last_log_index=req.last_log_index,
                                         last_log_term=req.last_log_term)
                fut = stub.RequestVote.future(pb, timeout=self.core.cfg.rpc_timeout_vote)
            else:
                pb = raft_pb.AppendEntriesRequest(
                    term=req.term, leader_id=req.leader_id, prev_log_index=req.prev_log_index,
                    prev_log_term=req.prev_log_term, entries=[to_pb_entry(x) for x in req.entries],
                    leader_commit=req.leader_commit)
                fut = stub.AppendEntries.future(pb, timeout=self.core.cfg.rpc_timeout_append)
            fut.add_done_callback(lambda f, p=peer, k=kind, r=req: self._on_reply(p, k, r, f))

    def _on_reply(self, peer, kind, req, fut) -> None:
        try:
            resp = fut.result()
        except grpc.RpcError:
            resp = None
        with self.core_lock:
            self.core.now = time.monotonic()
            if kind == "vote":
                self.core.on_vote_reply(peer, req.term, None if resp is None else
                                        VoteResp(resp.term, resp.vote_granted))
            else:
                self.core.on_append_reply(peer, req, None if resp is None else
                                          AppendResp(resp.term, resp.success))
            out = self.core.drain()
        self._send(out)

    # gRPC handlers (peer -> peer)
    def RequestVote(self, request, context):
        with self.core_lock:
            self.core.now = time.monotonic()
            r = self.core.on_request_vote(VoteReq(request.term, request.candidate_id,
                                                  request.last_log_index, request.last_log_term))
            out = self.core.drain()
        self._send(out)
        return raft_pb.VoteResponse(term=r.term, vote_granted=r.vote_granted)

    def AppendEntries(self, request, context):
        req = AppendReq(request.term, request.leader_id, request.prev_log_index,
                        request.prev_log_term, [from_pb_entry(x) for x in request.entries],
                        request.leader_commit)
        with self.core_lock:
            self.core.now = time.monotonic()
            r = self.core.on_append_entries(req)
            out = self.core.drain()
        self._send(out)
        return raft_pb.AppendEntriesResponse(term=r.term, success=r.success)

    # ------------------------------------------------------------ client API
    def is_leader(self) -> bool:
        return self.core.is_leader()

    def leader_info(self) -> dict:
        with self.core_lock:
            c = self.core
            return {"is_leader": c.is_leader(), "leader_id": c.leader_id, "term": c.term,
                    "state": c.role.value, "log": c.last_index + 1, "commit": c.commit_index,
                    "snap_index": c.snap_index}

    def propose(self, command: str, data: dict, timeout: float = 5.0) -> bool:
        """Replicate one command; True once committed and applied here."""
        payload = json.dumps(data).encode("utf-8")
        with self.core_lock:
            self.core.now = time.monotonic()
            idx, term = self.core.propose(command, payload)  # may raise NotLeaderError
            if self.core.last_applied >= idx:  # single node / local-commit mode
                return True
            w = _Waiter(term)
            self.waiters[idx] = w
            out = self.core.drain()
        self._send(out)
        if not w.event.wait(timeout):
            with self.core_lock:
                self.waiters.pop(idx, None)
            return False
        return w.ok


__all__ = ["RaftRuntime", "NotLeaderError", "GRPC_OPTS"]
