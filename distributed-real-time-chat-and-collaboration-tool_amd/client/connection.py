"""Leader-aware connection to the Raft chat cluster (client side).

Discovery asks every configured node for ``GetLeaderInfo`` and follows
``leader_address`` hints (client/chat_client.py:66-145).  Calls go through
``call(name, request)``, which resolves the RPC on the *current* stub at
call time - after a redirect the call goes to the new leader (the
reference bound the method to the old stub first: survey quirk Q25) - and
retries on UNAVAILABLE/DEADLINE_EXCEEDED and on "Not the leader" replies.

Retry safety: a DEADLINE_EXCEEDED write may still commit.  The chat shell
stamps every message / DM / upload with a ``request_id`` (the server turns it
into the record id, which the state machine de-duplicates), so those retries
are idempotent; calls that cannot be made idempotent pass
``retry_deadline=False`` and are not re-sent after a deadline.

Failover: when discovery moves the session to a different leader, the
``on_leader_change(address)`` hook runs - the shell uses it to re-validate
its token, auto-logout if the new leader rejects it, and restore the current
channel by name (ref client/chat_client.py:147-228).
"""
from __future__ import annotations

import logging
import time

import grpc

from ..protos import RAFT_SERVICE, make_stub, raft_pb

log = logging.getLogger(__name__)

DEFAULT_CLUSTER = ["localhost:50051", "localhost:50052", "localhost:50053"]
CHANNEL_OPTS = [("grpc.keepalive_time_ms", 10000), ("grpc.keepalive_timeout_ms", 5000),
                ("grpc.max_send_message_length", 50 * 1024 * 1024),
                ("grpc.max_receive_message_length", 50 * 1024 * 1024)]
RETRY_CODES = (grpc.StatusCode.UNAVAILABLE, grpc.StatusCode.DEADLINE_EXCEEDED)


class ClusterUnavailable(RuntimeError):
    pass


class ClusterConnection:
    def __init__(self, nodes=None, discovery_rounds: int = 10, round_sleep: float = 0.5,
                 probe_timeout: float = 2.0):
        self.nodes = list(nodes or DEFAULT_CLUSTER)
        self.rounds = discovery_rounds
        self.round_sleep = round_sleep
        self.probe_timeout = probe_timeout
        self.address: str | None = None
        self.channel = None
        self.stub = None
        self._channels: dict[str, grpc.Channel] = {}
        self.on_leader_change = None  # callable(address) after a failover re-discovery

    def _stub_for(self, addr: str):
        ch = self._channels.get(addr)
        if ch is None:
            ch = self._channels[addr] = grpc.insecure_channel(addr, options=CHANNEL_OPTS)
        return ch, make_stub(ch, RAFT_SERVICE)

    def _use(self, addr: str) -> None:
        prev = self.address
        self.channel, self.stub = self._stub_for(addr)
        self.address = addr
        if prev is not None and prev != addr and self.on_leader_change is not None:
            self.on_leader_change(addr)

    def probe(self, addr: str):
        _, stub = self._stub_for(addr)
        return stub.GetLeaderInfo(raft_pb.GetLeaderRequest(), timeout=self.probe_timeout)

    def discover(self) -> str:
        """Connect to the leader; raise ClusterUnavailable if none is found."""
        for rnd in range(self.rounds):
            for addr in self.nodes:
                try:
                    info = self.probe(addr)
                except grpc.RpcError:
                    continue
                if info.is_leader:
                    self._use(addr)
                    return addr
                if info.leader_address:
                    try:
                        li = self.probe(info.leader_address)
                        if li.is_leader:
                            self._use(info.leader_address)
                            return info.leader_address
                    except grpc.RpcError:
                        pass
            if rnd + 1 < self.rounds:
                time.sleep(self.round_sleep)
        raise ClusterUnavailable("could not find a Raft leader")

    def node_status(self) -> list[tuple]:
        out = []
        for addr in self.nodes:
            try:
                i = self.probe(addr)
                out.append((addr, i.state, i.term, i.is_leader, i.leader_id))
            except grpc.RpcError:
                out.append((addr, "down", None, False, None))
        return out

    def ensure(self) -> None:
        if self.stub is None:
            self.discover()
            return
        try:
            info = self.stub.GetLeaderInfo(raft_pb.GetLeaderRequest(), timeout=self.probe_timeout)
            if info.is_leader:
                return
        except grpc.RpcError:
            pass
        self.discover()

    def call(self, name: str, request, timeout: float = 5.0, attempts: int = 3,
             retry_deadline: bool = True):
        last = None
        for i in range(attempts):
            if self.stub is None:
                self.discover()
            try:
                resp = getattr(self.stub, name)(request, timeout=timeout)
            except grpc.RpcError as e:
                last = e
                code = e.code()
                if code == grpc.StatusCode.DEADLINE_EXCEEDED and not retry_deadline:
                    raise
                if code in RETRY_CODES and i + 1 < attempts:
                    self.discover()
                    continue
                raise
            msg = getattr(resp, "message", "")
            if (not getattr(resp, "success", True)) and msg == "Not the leader" and i + 1 < attempts:
                self.discover()
                continue
            return resp
        if last is not None:
            raise last
        raise ClusterUnavailable("no leader accepted the request")

    def close(self) -> None:
        for ch in self._channels.values():
            ch.close()
        self._channels.clear()
