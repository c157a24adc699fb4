"""Model configurations (public architecture hyper-parameters; random-init weights).

The four families BASELINE.json names for the LLM service:
  * Llama-3-8B  (smart reply / summarize, TP=1)        - flagship bench model
  * Llama-3-70B (ask-AI, TP=8 over xGMI)
  * Gemma-2B    (smart reply, TP=1; MQA, head_dim 256, GELU-tanh, (1+w) norm)
  * Mixtral-8x7B (context suggestions; top-2 of 8 experts, EP)
plus tiny variants of each for CPU tests.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass(frozen=True)
class ModelConfig:
    name: str
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    rope_theta: float = 500000.0
    rope_scaling: dict | None = field(default=None, hash=False, compare=False)
    rms_eps: float = 1e-5
    max_position: int = 8192
    act: str = "silu"                # silu | gelu_tanh
    gemma_norm: bool = False         # weight convention (1 + w)
    embed_scale: bool = False        # Gemma multiplies embeddings by sqrt(H)
    tie_embeddings: bool = False
    num_experts: int = 0             # 0 = dense MLP
    experts_per_token: int = 2
    bos_token_id: int = 1
    eos_token_id: int = 2
    init_std: float = 0.02
    query_pre_attn_scalar: float | None = None
    prefill_chunk: int = 16384       # engine prefill step, tokens (LLMEngine.prefill_chunk_tokens)

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def attn_scale(self) -> float:
        s = self.query_pre_attn_scalar or self.head_dim
        return float(s) ** -0.5

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def num_params(self) -> int:
        H, I, L, V = self.hidden_size, self.intermediate_size, self.num_layers, self.vocab_size
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        mlp = 3 * H * I * (self.num_experts if self.is_moe else 1) + (H * self.num_experts)
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


LLAMA3_8B = ModelConfig(
    name="llama-3-8b", vocab_size=128256, hidden_size=4096, intermediate_size=14336,
    num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128, rope_theta=500000.0,
    rms_eps=1e-5, max_position=8192, bos_token_id=128000, eos_token_id=128001)

LLAMA3_70B = ModelConfig(
    name="llama-3-70b", vocab_size=128256, hidden_size=8192, intermediate_size=28672,
    num_layers=80, num_heads=64, num_kv_heads=8, head_dim=128, rope_theta=500000.0,
    rms_eps=1e-5, max_position=8192, bos_token_id=128000, eos_token_id=128001,
    prefill_chunk=36864)  # a whole ask wave (256 x ~136 tokens) in one step, profiles/r6t

GEMMA_2B = ModelConfig(
    name="gemma-2b", vocab_size=256000, hidden_size=2048, intermediate_size=16384,
    num_layers=18, num_heads=8, num_kv_heads=1, head_dim=256, rope_theta=10000.0,
    rms_eps=1e-6, max_position=8192, act="gelu_tanh", gemma_norm=True, embed_scale=True,
    tie_embeddings=True, bos_token_id=2, eos_token_id=1)

MIXTRAL_8X7B = ModelConfig(
    name="mixtral-8x7b", vocab_size=32000, hidden_size=4096, intermediate_size=14336,
    num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128, rope_theta=1e6,
    rms_eps=1e-5, max_position=32768, num_experts=8, experts_per_token=2,
    bos_token_id=1, eos_token_id=2,
    prefill_chunk=32768)  # 8k rows per expert in the prefill MoE GEMMs, profiles/r6t

# Tiny shapes with the same structural features, for CPU tests and smoke runs.
TINY_LLAMA = ModelConfig(
    name="tiny-llama", vocab_size=512, hidden_size=256, intermediate_size=512,
    num_layers=2, num_heads=4, num_kv_heads=2, head_dim=64, rope_theta=10000.0,
    max_position=1024, bos_token_id=1, eos_token_id=2)

TINY_GEMMA = ModelConfig(
    name="tiny-gemma", vocab_size=512, hidden_size=256, intermediate_size=512,
    num_layers=2, num_heads=2, num_kv_heads=1, head_dim=128, rope_theta=10000.0,
    rms_eps=1e-6, max_position=1024, act="gelu_tanh", gemma_norm=True, embed_scale=True,
    tie_embeddings=True, bos_token_id=2, eos_token_id=1)

TINY_MIXTRAL = ModelConfig(
    name="tiny-mixtral", vocab_size=512, hidden_size=256, intermediate_size=256,
    num_layers=2, num_heads=4, num_kv_heads=2, head_dim=64, rope_theta=1e6,
    max_position=1024, num_experts=4, experts_per_token=2, bos_token_id=1, eos_token_id=2)

REGISTRY = {c.name: c for c in (LLAMA3_8B, LLAMA3_70B, GEMMA_2B, MIXTRAL_8X7B,
                                TINY_LLAMA, TINY_GEMMA, TINY_MIXTRAL)}


def get_config(name: str) -> ModelConfig:
    try:
        return REGISTRY[name]
    except KeyError:
        raise KeyError(f"unknown model {name!r}; known: {sorted(REGISTRY)}") from None
