"""Model zoo: Llama-3 (8B/70B), Gemma-2B, Mixtral-8x7B (random-init bf16)."""
from .config import (GEMMA_2B, LLAMA3_8B, LLAMA3_70B, MIXTRAL_8X7B, REGISTRY, TINY_GEMMA,
                     TINY_LLAMA, TINY_MIXTRAL, ModelConfig, get_config)
from .transformer import DecodeMeta, PrefillMeta, TransformerLM

__all__ = ["GEMMA_2B", "LLAMA3_8B", "LLAMA3_70B", "MIXTRAL_8X7B", "REGISTRY", "TINY_GEMMA",
           "TINY_LLAMA", "TINY_MIXTRAL", "ModelConfig", "get_config", "DecodeMeta", "PrefillMeta",
           "TransformerLM"]
