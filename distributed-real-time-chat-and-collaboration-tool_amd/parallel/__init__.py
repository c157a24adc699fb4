"""Parallelism: TP/EP process groups over RCCL (xGMI), DP replica routing."""
from .comm import ParallelContext, env_rank_world, init_distributed

__all__ = ["ParallelContext", "env_rank_world", "init_distributed"]
