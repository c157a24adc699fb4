"""Raft consensus core: pure state transitions, no I/O, no threads.

Inputs are method calls (``tick``, ``on_request_vote``, ``on_append_entries``,
``on_vote_reply``, ``on_append_reply``, ``propose``); outputs are messages
queued in ``outbox`` and committed entries delivered through ``apply_fn``.
The node runtime (raft/node.py) drives it from gRPC threads under one short
lock and sends the outbox *outside* that lock, so no network wait ever blocks
consensus (the reference held its node lock across thread joins and RPCs:
survey quirk Q2).  Tests drive it with a virtual clock and an in-memory
network with loss/partition/reorder injection (raft/sim.py).

Behaviour vs the reference (server/raft_node.py:469-1194):
  * indices are 0-based with -1 = none, as on the reference's wire and disk;
  * AppendEntries truncates only at the first conflicting entry (§5.3), so a
    stale or reordered RPC can no longer drop newer entries (quirk Q4);
  * commit requires a majority *and* an entry of the current term; a new
    leader appends a NOOP entry so earlier-term entries commit promptly;
  * writes are acknowledged after majority commit by default; the
    reference's leader-local commit (quirk Q1) is available as
    ``RaftConfig.local_commit``;
  * AppendEntries batches are bounded in bytes (quirk Q12) and rejected
    followers are probed with exponential back-off instead of one entry
    per round trip;
  * log compaction (the reference has none, SURVEY §5 "Checkpoint"): the
    runtime snapshots the state machine at an applied index and calls
    ``compact``; entries up to it leave the log (``snap_index`` /
    ``snap_term`` remember the boundary).  A follower whose next entry was
    compacted away is sent the snapshot (``InstallSnapshot``, Raft §7)
    instead of entries.
"""
from __future__ import annotations

import enum
import random
from dataclasses import dataclass


class Role(enum.Enum):
    FOLLOWER = "follower"
    CANDIDATE = "candidate"
    LEADER = "leader"


@dataclass(frozen=True)
class Entry:
    term: int
    command: str
    data: bytes


@dataclass
class VoteReq:
    term: int
    candidate_id: int
    last_log_index: int
    last_log_term: int


@dataclass
class VoteResp:
    term: int
    vote_granted: bool


@dataclass
class AppendReq:
    term: int
    leader_id: int
    prev_log_index: int
    prev_log_term: int
    entries: list
    leader_commit: int


@dataclass
class AppendResp:
    term: int
    success: bool


@dataclass
class SnapshotReq:
    term: int
    leader_id: int
    last_index: int
    last_term: int
    data: bytes = b""   # filled in by the transport from the latest snapshot


@dataclass
class SnapshotResp:
    term: int
    success: bool


@dataclass
class RaftConfig:
    election_timeout: tuple = (1.5, 3.0)     # reference: (10.0, 15.0)
    heartbeat_interval: float = 0.05         # reference: 0.05 (raft_node.py:2356)
    rpc_timeout_vote: float = 3.0
    rpc_timeout_append: float = 2.0
    max_batch_bytes: int = 4 << 20
    max_batch_entries: int = 4096
    local_commit: bool = False
    leader_noop: bool = True

    @staticmethod
    def reference_timing() -> "RaftConfig":
        return RaftConfig(election_timeout=(10.0, 15.0))


NOOP = "NOOP"
# The leader's no-op carries "{}": a reference node replaying this log
# (ref server/raft_node.py:1196-1241) json-decodes it and logs "Unknown
# command" instead of failing on an empty payload (its except handler would
# then hit an unbound ``command`` at log index 0 and crash).
NOOP_DATA = b"{}"


@dataclass
class _Inflight:
    sent_at: float
    prev_index: int
    n_entries: int
    term: int


class MemoryStorage:
    """Volatile storage (tests); durable ones live in raft/storage.py.

    ``entries`` hold absolute indices ``snap_index + 1 ...``; ``snapshot`` is
    the last installed/compacted state-machine image."""

    def __init__(self):
        self.entries: list[Entry] = []
        self.state = {"current_term": 0, "voted_for": None, "commit_index": -1, "last_applied": -1,
                      "snap_index": -1, "snap_term": 0}
        self.snapshot: bytes | None = None

    def load(self):
        return self.state, self.entries

    def append(self, entries: list[Entry]) -> None:
        self.entries.extend(entries)

    def truncate_from(self, index: int) -> None:
        del self.entries[index - self.state["snap_index"] - 1:]

    def compact(self, index: int, term: int, data: bytes | None = None) -> None:
        del self.entries[:index - self.state["snap_index"]]
        self.state["snap_index"], self.state["snap_term"] = index, term
        if data is not None:
            self.snapshot = data

    def install_snapshot(self, index: int, term: int, data: bytes, keep: list[Entry]) -> None:
        self.entries = list(keep)
        self.state["snap_index"], self.state["snap_term"] = index, term
        self.snapshot = data

    def latest_snapshot(self):
        if self.snapshot is None:
            return None
        return self.state["snap_index"], self.state["snap_term"], self.snapshot

    def save_state(self, state: dict) -> None:
        self.state.update(state)

    def flush(self) -> None:
        pass


class RaftCore:
    def __init__(self, node_id: int, peers, storage=None, apply_fn=None,
                 config: RaftConfig | None = None, seed: int | None = None, now: float = 0.0,
                 restore_fn=None):
        self.id = node_id
        self.peers = sorted(int(p) for p in peers)
        self.cfg = config or RaftConfig()
        self.storage = storage if storage is not None else MemoryStorage()
        self.apply_fn = apply_fn or (lambda index, entry: None)
        # restore_fn(data): replace the state machine with a snapshot image
        self.restore_fn = restore_fn or (lambda data: None)
        self.rng = random.Random(seed if seed is not None else node_id * 7919 + 17)
        st, entries = self.storage.load()
        self.snap_index = int(st.get("snap_index", -1))
        self.snap_term = int(st.get("snap_term", 0))
        self.log: list[Entry] = list(entries)  # absolute indices snap_index+1 ...
        self.term = int(st.get("current_term", 0))
        self.voted_for = st.get("voted_for")
        self.commit_index = max(self.snap_index,
                                min(int(st.get("commit_index", -1)), self.last_index))
        # the state machine is rebuilt by the runtime (snapshot + replay), so
        # apply restarts from the persisted last_applied
        self.last_applied = max(self.snap_index,
                                min(int(st.get("last_applied", -1)), self.commit_index))
        self.role = Role.FOLLOWER
        self.leader_id: int | None = None
        self.votes: set[int] = set()
        self.next_index: dict[int, int] = {}
        self.match_index: dict[int, int] = {}
        self.backoff: dict[int, int] = {}
        self.inflight: dict[int, _Inflight] = {}
        self.vote_inflight: dict[int, float] = {}
        self.last_sent: dict[int, float] = {}
        self.outbox: list[tuple] = []
        self.now = now
        self.election_deadline = now + self._timeout()
        self.commit_listeners = []

    # ------------------------------------------------------------ helpers
    @property
    def majority(self) -> int:
        return (len(self.peers) + 1) // 2 + 1

    @property
    def last_index(self) -> int:
        return self.snap_index + len(self.log)

    @property
    def first_index(self) -> int:
        """Oldest index still held as an entry."""
        return self.snap_index + 1

    def entry(self, i: int) -> Entry:
        return self.log[i - self.snap_index - 1]

    def term_at(self, i: int) -> int:
        if i == self.snap_index:
            return self.snap_term
        if self.snap_index < i <= self.last_index:
            return self.log[i - self.snap_index - 1].term
        return 0

    def _timeout(self) -> float:
        a, b = self.cfg.election_timeout
        return self.rng.uniform(a, b)

    def _persist(self) -> None:
        self.storage.save_state({"current_term": self.term, "voted_for": self.voted_for,
                                 "commit_index": self.commit_index,
                                 "last_applied": self.last_applied,
                                 "snap_index": self.snap_index, "snap_term": self.snap_term})

    def _become_follower(self, term: int, leader: int | None = None) -> None:
        changed = term != self.term
        if term > self.term:
            self.term = term
            self.voted_for = None
        self.role = Role.FOLLOWER
        self.leader_id = leader
        self.inflight.clear()
        self.vote_inflight.clear()
        if changed:
            self._persist()

    def is_leader(self) -> bool:
        return self.role == Role.LEADER

    # ------------------------------------------------------------ time
    def tick(self, now: float) -> None:
        self.now = now
        if self.role == Role.LEADER:
            for p in self.peers:
                inf = self.inflight.get(p)
                if inf is not None and now - inf.sent_at > self.cfg.rpc_timeout_append:
                    del self.inflight[p]  # lost reply: resend
                    inf = None
                if inf is None and (now - self.last_sent.get(p, -1e9) >= self.cfg.heartbeat_interval
                                    or self.next_index.get(p, 0) <= self.last_index):
                    self._send_append(p)
        else:
            if now >= self.election_deadline:
                self._start_election()
            elif self.role == Role.CANDIDATE:
                for p in self.peers:
                    t = self.vote_inflight.get(p)
                    if t is not None and now - t > self.cfg.rpc_timeout_vote:
                        del self.vote_inflight[p]

    def _start_election(self) -> None:
        self.role = Role.CANDIDATE
        self.term += 1
        self.voted_for = self.id
        self.leader_id = None
        self.votes = {self.id}
        self.election_deadline = self.now + self._timeout()
        self._persist()
        if len(self.votes) >= self.majority:
            self._become_leader()
            return
        req = VoteReq(self.term, self.id, self.last_index, self.term_at(self.last_index))
        for p in self.peers:
            self.vote_inflight[p] = self.now
            self.outbox.append((p, "vote", req))

    def _become_leader(self) -> None:
        self.role = Role.LEADER
        self.leader_id = self.id
        self.inflight.clear()
        for p in self.peers:
            self.next_index[p] = self.last_index + 1
            self.match_index[p] = -1
            self.backoff[p] = 1
            self.last_sent[p] = -1e9
        if self.cfg.leader_noop:
            self._append_local([Entry(self.term, NOOP, NOOP_DATA)])
        for p in self.peers:
            self._send_append(p)
        self._advance_commit()

    # ------------------------------------------------------------ votes
    def on_request_vote(self, req: VoteReq) -> VoteResp:
        if req.term < self.term:
            return VoteResp(self.term, False)
        if req.term > self.term:
            self._become_follower(req.term)
        my_lt, my_li = self.term_at(self.last_index), self.last_index
        up_to_date = (req.last_log_term > my_lt or
                      (req.last_log_term == my_lt and req.last_log_index >= my_li))
        if self.voted_for in (None, req.candidate_id) and up_to_date:
            self.voted_for = req.candidate_id
            self.election_deadline = self.now + self._timeout()
            self._persist()
            return VoteResp(self.term, True)
        return VoteResp(self.term, False)

    def on_vote_reply(self, peer: int, req_term: int, resp: VoteResp | None) -> None:
        self.vote_inflight.pop(peer, None)
        if resp is None:
            return
        if resp.term > self.term:
            self._become_follower(resp.term)
            self.election_deadline = self.now + self._timeout()
            return
        if self.role != Role.CANDIDATE or req_term != self.term or not resp.vote_granted:
            return
        self.votes.add(peer)
        if len(self.votes) >= self.majority:
            self._become_leader()

    # ------------------------------------------------------------ replication
    def _append_local(self, entries: list[Entry]) -> int:
        self.log.extend(entries)
        self.storage.append(entries)
        return self.last_index

    def _send_append(self, p: int) -> None:
        ni = min(self.next_index.get(p, self.last_index + 1), self.last_index + 1)
        if ni <= self.snap_index:  # the entries it needs are compacted away
            req = SnapshotReq(self.term, self.id, self.snap_index, self.snap_term)
            self.inflight[p] = _Inflight(self.now, self.snap_index, 0, self.term)
            self.last_sent[p] = self.now
            self.outbox.append((p, "snapshot", req))
            return
        prev = ni - 1
        batch, size = [], 0
        for i in range(ni, self.last_index + 1):
            e = self.entry(i)
            sz = len(e.data) + len(e.command) + 16
            if batch and (size + sz > self.cfg.max_batch_bytes or len(batch) >= self.cfg.max_batch_entries):
                break
            batch.append(e)
            size += sz
        req = AppendReq(self.term, self.id, prev, self.term_at(prev), batch, self.commit_index)
        self.inflight[p] = _Inflight(self.now, prev, len(batch), self.term)
        self.last_sent[p] = self.now
        self.outbox.append((p, "append", req))

    def on_append_entries(self, req: AppendReq) -> AppendResp:
        if req.term < self.term:
            return AppendResp(self.term, False)
        if req.term > self.term or self.role != Role.FOLLOWER:
            self._become_follower(req.term, req.leader_id)
        self.leader_id = req.leader_id
        self.election_deadline = self.now + self._timeout()
        prev = req.prev_log_index
        new = list(req.entries)
        if prev < self.snap_index:
            # the prefix up to snap_index is committed (hence identical on
            # every node): drop the part of the batch the snapshot covers
            skip = self.snap_index - prev
            if skip >= len(new):
                return AppendResp(self.term, True)  # everything sent is in the snapshot
            new = new[skip:]
            prev = self.snap_index
        elif prev >= 0 and (prev > self.last_index or self.term_at(prev) != req.prev_log_term):
            return AppendResp(self.term, False)
        # §5.3: skip entries already present, truncate only at a conflict
        idx = prev + 1
        k = 0
        while k < len(new) and idx + k <= self.last_index:
            if self.term_at(idx + k) != new[k].term:
                if idx + k <= self.commit_index and not self.cfg.local_commit:
                    # never happens under Raft's safety rules; with the
                    # reference's leader-local commit it can (quirk Q1)
                    raise AssertionError("leader tried to overwrite a committed entry")
                del self.log[idx + k - self.snap_index - 1:]
                self.storage.truncate_from(idx + k)
                break
            k += 1
        if k < len(new):
            self._append_local(new[k:])
        if req.leader_commit > self.commit_index:
            self.commit_index = max(self.commit_index, min(req.leader_commit, prev + len(new)))
        if self.last_applied < self.commit_index:
            # also catches up a runtime that restarted with committed entries
            # it has not re-applied yet
            self._apply()
        return AppendResp(self.term, True)

    # ------------------------------------------------------------ snapshots
    def on_install_snapshot(self, req: SnapshotReq) -> SnapshotResp:
        """Raft §7 InstallSnapshot (whole image; the transport reassembles
        chunks before calling this)."""
        if req.term < self.term:
            return SnapshotResp(self.term, False)
        if req.term > self.term or self.role != Role.FOLLOWER:
            self._become_follower(req.term, req.leader_id)
        self.leader_id = req.leader_id
        self.election_deadline = self.now + self._timeout()
        if req.last_index <= self.commit_index:  # already have everything it covers
            return SnapshotResp(self.term, True)
        keep: list[Entry] = []
        if self.snap_index < req.last_index <= self.last_index and \
                self.term_at(req.last_index) == req.last_term:
            keep = self.log[req.last_index - self.snap_index:]  # retain the matching suffix
        self.log = list(keep)
        self.snap_index, self.snap_term = req.last_index, req.last_term
        self.storage.install_snapshot(req.last_index, req.last_term, req.data, keep)
        self.restore_fn(req.data)
        self.commit_index = max(self.commit_index, req.last_index)
        self.last_applied = req.last_index
        self._persist()
        for cb in self.commit_listeners:
            cb(self.last_applied)
        return SnapshotResp(self.term, True)

    def on_snapshot_reply(self, peer: int, req: SnapshotReq, resp: SnapshotResp | None) -> None:
        inf = self.inflight.get(peer)
        if inf is not None and inf.prev_index == req.last_index and inf.term == req.term:
            del self.inflight[peer]
        if resp is None:
            return
        if resp.term > self.term:
            self._become_follower(resp.term)
            self.election_deadline = self.now + self._timeout()
            return
        if self.role != Role.LEADER or req.term != self.term or not resp.success:
            return
        self.match_index[peer] = max(self.match_index.get(peer, -1), req.last_index)
        self.next_index[peer] = max(self.next_index.get(peer, 0), req.last_index + 1)
        self.backoff[peer] = 1
        self._advance_commit()
        if self.next_index[peer] <= self.last_index:
            self._send_append(peer)

    def compact(self, index: int, data: bytes | None = None) -> bool:
        """Drop entries up to ``index`` (<= last_applied) after the runtime has
        durably saved a state-machine snapshot taken at ``index``."""
        if index <= self.snap_index or index > self.last_applied:
            return False
        term = self.term_at(index)
        del self.log[:index - self.snap_index]
        self.snap_index, self.snap_term = index, term
        self.storage.compact(index, term, data)
        self._persist()
        return True

    def on_append_reply(self, peer: int, req: AppendReq, resp: AppendResp | None) -> None:
        inf = self.inflight.get(peer)
        if inf is not None and inf.prev_index == req.prev_log_index and inf.term == req.term:
            del self.inflight[peer]
        if resp is None or self.role != Role.LEADER:
            if resp is not None and resp.term > self.term:
                self._become_follower(resp.term)
            return
        if resp.term > self.term:
            self._become_follower(resp.term)
            self.election_deadline = self.now + self._timeout()
            return
        if req.term != self.term:
            return
        if resp.success:
            m = req.prev_log_index + len(req.entries)
            if m > self.match_index.get(peer, -1):
                self.match_index[peer] = m
            self.next_index[peer] = max(self.next_index.get(peer, 0), m + 1)
            self.backoff[peer] = 1
            self._advance_commit()
            if self.next_index[peer] <= self.last_index:
                self._send_append(peer)
        else:
            b = self.backoff.get(peer, 1)
            self.next_index[peer] = max(0, min(self.next_index.get(peer, 0), req.prev_log_index + 1) - b)
            self.backoff[peer] = min(b * 2, 1 << 16)
            self._send_append(peer)

    def _advance_commit(self) -> None:
        if self.role != Role.LEADER:
            return
        matches = sorted([self.last_index] + [self.match_index.get(p, -1) for p in self.peers],
                         reverse=True)
        n = matches[self.majority - 1]
        if n > self.commit_index and self.term_at(n) == self.term:
            self.commit_index = n
            self._apply()

    def _apply(self) -> None:
        applied = False
        while self.last_applied < self.commit_index:
            self.last_applied += 1
            e = self.entry(self.last_applied)
            self.apply_fn(self.last_applied, e)
            applied = True
        if applied:
            self._persist()
            for cb in self.commit_listeners:
                cb(self.last_applied)

    # ------------------------------------------------------------ client API
    def propose(self, command: str, data: bytes) -> tuple[int, int]:
        """Append a command (leader only). Returns (index, term)."""
        if self.role != Role.LEADER:
            raise NotLeaderError(self.leader_id)
        idx = self._append_local([Entry(self.term, command, data)])
        if self.cfg.local_commit:
            # reference behaviour (quirk Q1): commit + apply before replication
            self.commit_index = max(self.commit_index, idx)
            self._apply()
        else:
            self._advance_commit()  # single-node cluster commits immediately
        for p in self.peers:
            if p not in self.inflight:
                self._send_append(p)
        return idx, self.term

    def drain(self) -> list:
        out, self.outbox = self.outbox, []
        return out

    def status(self) -> dict:
        return {"id": self.id, "role": self.role.value, "term": self.term,
                "leader": self.leader_id, "log": self.last_index + 1, "commit": self.commit_index,
                "applied": self.last_applied, "snap_index": self.snap_index}


class NotLeaderError(Exception):
    def __init__(self, leader_id):
        super().__init__(f"not the leader (leader={leader_id})")
        self.leader_id = leader_id
