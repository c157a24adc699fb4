"""gRPC servers: the Raft chat node (raft.RaftNode) and the legacy single-node chat.ChatService."""
