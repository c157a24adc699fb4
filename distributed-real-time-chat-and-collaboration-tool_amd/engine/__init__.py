"""Serving engine: paged KV cache, continuous batching, hipGraph decode."""
from .engine import EngineLoop, LLMEngine
from .kv_cache import PagedKVCache
from .request import Request, RequestState, SamplingParams
from .tokenizer import ChatTokenizer

__all__ = ["EngineLoop", "LLMEngine", "PagedKVCache", "Request", "RequestState",
           "SamplingParams", "ChatTokenizer"]
