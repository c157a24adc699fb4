"""Wire contract: raft.RaftNode, llm.LLMService, chat.ChatService (+ toy chat)."""
from .registry import (CHAT_SERVICE, CHAT_TOY_SERVICE, LLM_SERVICE, RAFT_SERVICE,
                       RAFT_SNAPSHOT_SERVICE, Method, Service, add_servicer, chat_pb, chat_toy_pb,
                       file_descriptor_protos, llm_pb, make_stub, raft_pb, raft_snap_pb)

# Server-side queue for calls that arrived before a handler picked them up.  The sync Python
# server re-posts one request slot per accepted call, so a burst of concurrent RPCs (a wave of
# ~1k clients starting together) waits in grpc-core's pending list, whose default limit (1,000)
# CANCELs the excess (measured: 1,280 concurrent smart-reply RPCs lost ~100 at start-up).
SERVER_QUEUE_OPTS = [("grpc.server.max_pending_requests", 1 << 16),
                     ("grpc.server.max_pending_requests_hard_limit", 1 << 17)]

__all__ = ["CHAT_SERVICE", "CHAT_TOY_SERVICE", "LLM_SERVICE", "RAFT_SERVICE", "RAFT_SNAPSHOT_SERVICE",
           "raft_snap_pb", "Method", "Service",
           "add_servicer", "chat_pb", "chat_toy_pb", "file_descriptor_protos", "llm_pb", "make_stub",
           "raft_pb", "SERVER_QUEUE_OPTS"]
