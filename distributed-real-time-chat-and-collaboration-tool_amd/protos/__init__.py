"""Wire contract: raft.RaftNode, llm.LLMService, chat.ChatService (+ toy chat)."""
from .registry import (CHAT_SERVICE, CHAT_TOY_SERVICE, LLM_SERVICE, RAFT_SERVICE,
                       RAFT_SNAPSHOT_SERVICE, Method, Service, add_servicer, chat_pb, chat_toy_pb,
                       file_descriptor_protos, llm_pb, make_stub, raft_pb, raft_snap_pb)

__all__ = ["CHAT_SERVICE", "CHAT_TOY_SERVICE", "LLM_SERVICE", "RAFT_SERVICE", "RAFT_SNAPSHOT_SERVICE",
           "raft_snap_pb", "Method", "Service",
           "add_servicer", "chat_pb", "chat_toy_pb", "file_descriptor_protos", "llm_pb", "make_stub",
           "raft_pb"]
