"""Hot ops of the inference engine.

Each op dispatches on the tensor's device: GPU tensors run the hand-written
CDNA4 HIP kernel (``csrc/kernels``), CPU tensors run the fp32 PyTorch
reference of the same op (used by the CPU tests and as the GPU numerics
oracle).  Projection GEMMs are hipBLASLt: ``linear`` replays a measured per-shape
solution for the decode shapes in the tuning table (``ops/gemm.py``) and
falls back to ``torch.nn.functional.linear`` elsewhere; everything around
them is fused here.
"""
from ._ext import on_gpu, reference_mode
from .activation import act_glu, act_glu_ref
from .attention import (KV_BLOCK, DecodeWorkspace, decode_partitioning, paged_decode_attention,
                        paged_decode_attention_rope, set_prefill_persist,
                        paged_decode_ref, prefill_attention, prefill_attention_ref, prefill_tiles)
from .gemm import (Partials, glu_linear, linear, linear_partials, linear_residual,
                   linear_residual_rinv, mfma_gemm, norm_glu, norm_linear, residual_fusable,
                   rs_linear, w4_glu_ok)
from .moe import fused_moe, fused_moe_ref
from .norm import PendingNorm, rmsnorm, rmsnorm_partials, rmsnorm_ref
from .rope import build_rope_cache, kv_write_v, kv_write_v_ref, rope_kv_, rope_kv_ref
from .sampling import sample, sample_ref

__all__ = [
    "on_gpu", "reference_mode", "linear", "linear_partials", "Partials", "rmsnorm_partials",
    "linear_residual_rinv", "rs_linear", "norm_linear", "glu_linear", "norm_glu", "w4_glu_ok", "mfma_gemm", "linear_residual", "residual_fusable", "PendingNorm", "fused_moe", "fused_moe_ref",
    "act_glu", "act_glu_ref", "KV_BLOCK", "DecodeWorkspace", "decode_partitioning",
    "paged_decode_attention", "paged_decode_attention_rope", "paged_decode_ref", "prefill_attention", "prefill_attention_ref",
    "prefill_tiles", "rmsnorm", "rmsnorm_ref", "build_rope_cache", "rope_kv_", "rope_kv_ref",
    "kv_write_v", "kv_write_v_ref",
    "sample", "sample_ref",
]
