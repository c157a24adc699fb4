"""Raft consensus core, durable storage, replicated chat state machine, node runtime."""
from .core import Entry, NotLeaderError, RaftConfig, RaftCore, Role
from .state_machine import ChatState

__all__ = ["Entry", "NotLeaderError", "RaftConfig", "RaftCore", "Role", "ChatState"]
