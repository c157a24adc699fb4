"""Deterministic in-memory network for RaftCore (fault-injection test harness).

The reference has no fault injection at all; this simulator
drives N cores on a virtual clock and lets tests drop, delay, duplicate and
reorder messages and partition the cluster.
"""
from __future__ import annotations

import heapq
import pickle
import random

from .core import AppendReq, MemoryStorage, RaftConfig, RaftCore, Role


class SimCluster:
    def __init__(self, n: int = 3, config: RaftConfig | None = None, seed: int = 0,
                 drop: float = 0.0, delay: tuple = (0.001, 0.005), dup: float = 0.0):
        self.rng = random.Random(seed)
        self.now = 0.0
        self.drop, self.delay, self.dup = drop, delay, dup
        self.partition: list[set] | None = None
        self.down: set[int] = set()
        self.q: list = []
        self.seq = 0
        self.applied: dict[int, list] = {}
        self.storages: dict[int, MemoryStorage] = {}
        self.cfg = config or RaftConfig(election_timeout=(0.15, 0.3), heartbeat_interval=0.02,
                                        rpc_timeout_append=0.1, rpc_timeout_vote=0.1)
        ids = list(range(1, n + 1))
        self.nodes: dict[int, RaftCore] = {}
        for i in ids:
            self.storages[i] = MemoryStorage()
            self._make(i, ids)
        self.leaders_by_term: dict[int, set] = {}

    def _make(self, i, ids) -> None:
        snap = self.storages[i].snapshot
        # the simulated state machine is the list of applied entries; its
        # snapshot image is that list (test-local data, produced here)
        self.applied[i] = pickle.loads(snap) if snap else []

        def apply(idx, e, i=i):
            self.applied[i].append((idx, e))

        def restore(data, i=i):
            self.applied[i] = pickle.loads(data)

        self.nodes[i] = RaftCore(i, [p for p in ids if p != i], self.storages[i], apply, self.cfg,
                                 seed=self.rng.randrange(1 << 30), now=self.now,
                                 restore_fn=restore)

    def compact(self, i: int) -> bool:
        """Snapshot node i's state machine at its applied index and compact."""
        n = self.nodes[i]
        data = pickle.dumps(self.applied[i])
        return n.compact(n.last_applied, data)

    # ------------------------------------------------------------- faults
    def can_talk(self, a: int, b: int) -> bool:
        if a in self.down or b in self.down:
            return False
        if self.partition is None:
            return True
        return any(a in g and b in g for g in self.partition)

    def crash(self, i: int) -> None:
        self.down.add(i)

    def restart(self, i: int) -> None:
        """Restart from durable storage (volatile state lost)."""
        self.down.discard(i)
        # the simulated state machine is volatile: restore the snapshot and
        # replay the log after it
        self.storages[i].state["last_applied"] = -1
        ids = sorted(self.nodes)
        self._make(i, ids)
        # boot replay of the committed entries, as raft/node.py does
        n = self.nodes[i]
        n.last_applied = n.snap_index
        n._apply()

    # ------------------------------------------------------------- running
    def _post(self, when, item) -> None:
        self.seq += 1
        heapq.heappush(self.q, (when, self.seq, item))

    def _flush_outboxes(self) -> None:
        for i, n in self.nodes.items():
            for dst, kind, req in n.drain():
                if i in self.down:
                    continue
                if kind == "snapshot":
                    req.data = self.storages[i].snapshot
                copies = 2 if self.rng.random() < self.dup else 1
                for _ in range(copies):
                    if self.rng.random() < self.drop:
                        continue
                    self._post(self.now + self.rng.uniform(*self.delay), ("req", i, dst, kind, req))

    def step(self, dt: float = 0.005) -> None:
        end = self.now + dt
        while self.q and self.q[0][0] <= end:
            when, _, item = heapq.heappop(self.q)
            self.now = max(self.now, when)
            typ, src, dst, kind, req = item[:5]
            if typ == "req":
                if not self.can_talk(src, dst):
                    continue
                node = self.nodes[dst]
                node.now = self.now
                if kind == "vote":
                    resp = node.on_request_vote(req)
                elif kind == "snapshot":
                    resp = node.on_install_snapshot(req)
                else:
                    resp = node.on_append_entries(req)
                if self.rng.random() >= self.drop:
                    self._post(self.now + self.rng.uniform(*self.delay), ("resp", dst, src, kind, req, resp))
            else:
                if not self.can_talk(src, dst):
                    continue
                node = self.nodes[dst]
                node.now = self.now
                resp = item[5]
                if kind == "vote":
                    node.on_vote_reply(src, req.term, resp)
                elif kind == "snapshot":
                    node.on_snapshot_reply(src, req, resp)
                else:
                    node.on_append_reply(src, req, resp)
            self._flush_outboxes()
        self.now = end
        for i, n in self.nodes.items():
            if i not in self.down:
                n.tick(self.now)
        self._flush_outboxes()
        for i, n in self.nodes.items():
            if i not in self.down and n.role == Role.LEADER:
                self.leaders_by_term.setdefault(n.term, set()).add(i)

    def run(self, seconds: float, dt: float = 0.005) -> None:
        t_end = self.now + seconds
        while self.now < t_end:
            self.step(dt)

    def leader(self) -> int | None:
        ls = [i for i, n in self.nodes.items() if i not in self.down and n.role == Role.LEADER]
        if not ls:
            return None
        return max(ls, key=lambda i: self.nodes[i].term)

    def wait_leader(self, timeout: float = 10.0) -> int:
        t_end = self.now + timeout
        while self.now < t_end:
            self.step()
            l = self.leader()
            if l is not None:
                return l
        raise TimeoutError("no leader elected")

    def propose(self, command: str, data: bytes = b"") -> tuple:
        l = self.leader()
        if l is None:
            raise RuntimeError("no leader")
        r = self.nodes[l].propose(command, data)
        self._flush_outboxes()
        return r

    def committed_commands(self, i: int) -> list:
        return [e.command for _, e in self.applied[i] if e.command != "NOOP"]


__all__ = ["SimCluster", "AppendReq"]
