"""Local cluster harnesses (tests, demos, benchmarks).

``LocalCluster`` starts N Raft chat nodes in THIS process on ephemeral localhost ports (the
reference's manual 3-terminal setup, automated) and exposes kill/restart for failover
experiments.  ``ProcessCluster`` starts each node in its own process, as a deployment runs
them (one interpreter per node: the leader's RPC handling does not share a GIL with the
followers, the benchmark clients or an in-process LLM front-end).
"""
from __future__ import annotations

import socket
import time

import grpc

from ..protos import RAFT_SERVICE, make_stub, raft_pb
from ..raft.core import RaftConfig


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class LocalCluster:
    def __init__(self, n: int = 3, data_root: str = ".", llm_address: str | None = None,
                 raft: RaftConfig | None = None, bcrypt_rounds: int = 4, storage: str = "native",
                 **node_kw):
        from ..server.raft_service import NodeConfig

        self.n = n
        self.ports = [free_port() for _ in range(n)]
        self.peers = {i + 1: f"127.0.0.1:{p}" for i, p in enumerate(self.ports)}
        self.raft = raft or RaftConfig(election_timeout=(0.3, 0.6), heartbeat_interval=0.03)
        self.cfgs = {i: NodeConfig(node_id=i, port=self.ports[i - 1], peers=self.peers,
                                   data_root=data_root, llm_address=llm_address, raft=self.raft,
                                   bcrypt_rounds=bcrypt_rounds, advertise_host="127.0.0.1",
                                   storage=storage, **node_kw)
                     for i in self.peers}
        self.nodes: dict = {}
        self.servers: dict = {}

    def start(self) -> "LocalCluster":
        for i in self.peers:
            self.start_node(i)
        return self

    def start_node(self, i: int) -> None:
        from ..server.node import serve

        node, server = serve(self.cfgs[i], block=False, bind="127.0.0.1")
        self.nodes[i], self.servers[i] = node, server

    def kill(self, i: int) -> None:
        self.servers.pop(i).stop(0)
        self.nodes.pop(i).stop()

    def stop(self) -> None:
        for i in list(self.nodes):
            self.kill(i)

    def leader(self, timeout: float = 10.0) -> int:
        """Id of the current leader, once it has the default users/channels
        (a fresh cluster seeds them through the log right after election)."""
        t_end = time.time() + timeout
        while time.time() < t_end:
            ls = [i for i, n in self.nodes.items() if n.rt.is_leader()]
            if ls and self.nodes[ls[0]].genesis_done.is_set():
                return ls[0]
            time.sleep(0.01)
        raise TimeoutError("no leader")

    def stub(self, i: int):
        return make_stub(grpc.insecure_channel(self.peers[i]), RAFT_SERVICE)

    def addresses(self) -> list[str]:
        return list(self.peers.values())

    def login(self, i: int, user: str = "alice", pw: str | None = None) -> str:
        r = self.stub(i).Login(raft_pb.LoginRequest(username=user, password=pw or f"{user}123"))
        assert r.success, r.message
        return r.token

    def wait_applied(self, predicate, timeout: float = 5.0) -> bool:
        t_end = time.time() + timeout
        while time.time() < t_end:
            if all(predicate(n) for n in self.nodes.values()):
                return True
            time.sleep(0.02)
        return False

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False


def _node_proc(cfg, ready, stop) -> None:
    import signal as _signal

    from ..server.node import serve

    _signal.signal(_signal.SIGINT, _signal.SIG_IGN)  # the parent stops us through `stop`
    node, server = serve(cfg, block=False, bind="127.0.0.1")
    ready.set()
    stop.wait()
    server.stop(1.0)
    node.stop()


class ProcessCluster(LocalCluster):
    """LocalCluster with every node in its own (spawned) process; leader discovery and
    logins go over RPC."""

    def start(self) -> "ProcessCluster":
        import multiprocessing as mp

        ctx = mp.get_context("spawn")
        self._stop = ctx.Event()
        self.procs = {}
        readies = []
        for i in self.peers:
            r = ctx.Event()
            p = ctx.Process(target=_node_proc, args=(self.cfgs[i], r, self._stop), daemon=True)
            p.start()
            self.procs[i] = p
            readies.append(r)
        for r in readies:
            if not r.wait(120):
                self.stop()
                raise RuntimeError("a Raft node process did not start")
        return self

    def leader(self, timeout: float = 20.0) -> int:
        t_end = time.time() + timeout
        while time.time() < t_end:
            for i in self.peers:
                try:
                    r = self.stub(i).GetLeaderInfo(raft_pb.GetLeaderRequest(), timeout=1.0)
                except grpc.RpcError:
                    continue
                if r.is_leader:
                    try:  # genesis (default users / channels) applied: a login succeeds
                        self.login(i)
                        return i
                    except (AssertionError, grpc.RpcError):
                        pass
            time.sleep(0.05)
        raise TimeoutError("no leader")

    def kill(self, i: int) -> None:
        raise NotImplementedError("ProcessCluster stops all nodes together")

    def stop(self) -> None:
        if getattr(self, "_stop", None) is not None:
            self._stop.set()
        for p in getattr(self, "procs", {}).values():
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
        self.procs = {}
