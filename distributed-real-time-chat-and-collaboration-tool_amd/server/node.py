"""Raft chat node entry point: ``python -m drtc_amd.server.node --node-id 1 --port 50051``.

Defaults mirror the reference (server/raft_node.py:2358-2418): a 3-node
cluster on localhost:50051-50053, 50 MB gRPC messages, data under
``./raft_node_{id}_data``, the LLM service at localhost:50055, and a status
line every 2 s.  Everything is overridable (peers, timings, storage, LLM
address, token mode, local-commit compatibility mode).
"""
from __future__ import annotations

import argparse
import logging
import signal
import threading
from concurrent import futures

import grpc

from ..protos import RAFT_SERVICE, RAFT_SNAPSHOT_SERVICE, SERVER_QUEUE_OPTS, add_servicer
from ..raft.core import RaftConfig
from ..utils.config import parse_with_config
from ..utils.logging_utils import setup_logging
from .raft_service import ChatNode, NodeConfig

log = logging.getLogger("drtc_amd.server.node")

DEFAULT_PEERS = {1: "localhost:50051", 2: "localhost:50052", 3: "localhost:50053"}
SERVER_OPTS = [
    ("grpc.max_send_message_length", 50 * 1024 * 1024),
    ("grpc.max_receive_message_length", 50 * 1024 * 1024),
    ("grpc.keepalive_time_ms", 10000),
    ("grpc.keepalive_timeout_ms", 5000),
] + SERVER_QUEUE_OPTS


def parse_peers(s: str | None) -> dict:
    if not s:
        return dict(DEFAULT_PEERS)
    out = {}
    for part in s.split(","):
        k, v = part.split("=", 1)
        out[int(k)] = v
    return out


def serve(cfg: NodeConfig, block: bool = True, bind: str = "[::]",
          stop: threading.Event | None = None):
    """Run one node.  ``block``: serve until SIGINT / SIGTERM (or ``stop`` is set), then stop
    in order and return; the handlers are installed before the node starts (main() installs
    them even earlier, before argument-dependent start-up work)."""
    if block and stop is None:
        stop = _install_stop_handlers()
    node = ChatNode(cfg)
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=cfg.grpc_workers), options=SERVER_OPTS)
    add_servicer(server, RAFT_SERVICE, node)
    add_servicer(server, RAFT_SNAPSHOT_SERVICE, node.rt)  # log-compaction catch-up (Raft §7)
    port = server.add_insecure_port(f"{bind}:{cfg.port}")
    if port == 0:
        raise RuntimeError(f"cannot bind port {cfg.port}")
    server.start()
    node.start()
    log.info("raft chat node %d on port %d (peers %s)", cfg.node_id, cfg.port, cfg.peers)
    if not block:
        return node, server
    while not stop.wait(2.0):
        i = node.rt.leader_info()
        with node.rt.state_lock:
            nu, nc, nf = len(node.st.users), len(node.st.channels), len(node.st.files)
        role = i["state"].upper()
        lead = f"leader {i['leader_id']}" if i["leader_id"] is not None else "no leader"
        log.info("node %d %s | term %d | log %d (commit %d) | %d users | %d channels | %d files | %s",
                 cfg.node_id, role, i["term"], i["log"], i["commit"], nu, nc, nf, lead)
    # ordered stop: no new RPCs (in-flight ones get 1 s), then the Raft runtime (timer and
    # persist threads joined, state flushed, log exported and closed, channels closed)
    server.stop(1.0).wait(10)
    node.stop()
    return node, server


def _install_stop_handlers() -> threading.Event:
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *a: stop.set())
    signal.signal(signal.SIGTERM, lambda *a: _stop_once(stop))
    return stop


def _stop_once(stop: threading.Event) -> None:
    """SIGTERM: start the ordered shutdown; further SIGTERMs are ignored (CPython restores
    the default - terminate - action for Python-level handlers during finalization, so a
    repeated SIGTERM from a supervisor would otherwise kill the exiting process)."""
    stop.set()
    signal.signal(signal.SIGTERM, signal.SIG_IGN)


def main(argv=None) -> None:
    stop = _install_stop_handlers()  # a SIGTERM during start-up still ends the node in order
    ap = argparse.ArgumentParser(description="drtc_amd Raft chat node")
    ap.add_argument("--node-id", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--peers", default=None, help="id=host:port,... (default: 3 nodes on localhost)")
    ap.add_argument("--data-root", default=".")
    ap.add_argument("--storage", choices=("native", "pickle"), default="native")
    ap.add_argument("--llm", default="localhost:50055", help="LLM service address ('' disables)")
    for feat, rpc in (("smart", "GetSmartReply"), ("summary", "SummarizeConversation"),
                      ("ask", "GetLLMAnswer"), ("suggest", "GetContextSuggestions")):
        ap.add_argument(f"--llm-{feat}", default=None,
                        help=f"LLM service address for {rpc} (default: --llm)")
    ap.add_argument("--election-timeout", default="1.5,3.0", help="min,max seconds")
    ap.add_argument("--reference-timing", action="store_true", help="10-15 s election timeout")
    ap.add_argument("--heartbeat", type=float, default=0.05)
    ap.add_argument("--local-commit", action="store_true", help="reference quirk Q1 behaviour")
    ap.add_argument("--token-mode", choices=("replicated", "reference"), default="replicated")
    ap.add_argument("--bcrypt-rounds", type=int, default=12)
    ap.add_argument("--fsync", dest="fsync", action="store_true", default=True,
                    help="fsync log appends and votes before acknowledging (default)")
    ap.add_argument("--no-fsync", dest="fsync", action="store_false",
                    help="reference behaviour: no fsync (acknowledged writes can be lost)")
    ap.add_argument("--snapshot-every", type=int, default=0,
                    help="snapshot the state machine and compact the log every N entries "
                         "(native storage; 0 = keep the whole log like the reference)")
    ap.add_argument("--log-level", default="INFO")
    a = parse_with_config(ap, argv)
    setup_logging(a.log_level)
    lo, hi = (10.0, 15.0) if a.reference_timing else tuple(float(x) for x in a.election_timeout.split(","))
    cfg = NodeConfig(node_id=a.node_id, port=a.port, peers=parse_peers(a.peers), data_root=a.data_root,
                     storage=a.storage, llm_address=a.llm or None,
                     llm_smart=a.llm_smart, llm_summary=a.llm_summary, llm_ask=a.llm_ask,
                     llm_suggest=a.llm_suggest,
                     raft=RaftConfig(election_timeout=(lo, hi), heartbeat_interval=a.heartbeat,
                                     local_commit=a.local_commit),
                     token_mode=a.token_mode, bcrypt_rounds=a.bcrypt_rounds, fsync=a.fsync,
                     snapshot_every=a.snapshot_every)
    print(f"\n{'=' * 60}\n  Raft Chat Node {a.node_id}\n  Port: {a.port}\n"
          f"  Features: Consensus + Full Chat Application + on-GPU AI\n{'=' * 60}\n", flush=True)
    serve(cfg, stop=stop)


if __name__ == "__main__":
    main()
