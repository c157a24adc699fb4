"""Hot ops of the inference engine.

Each op dispatches on the tensor's device: GPU tensors run the hand-written
CDNA4 HIP kernel (``csrc/kernels``), CPU tensors run the fp32 PyTorch
reference of the same op (used by the CPU tests and as the GPU numerics
oracle).  Projection GEMMs go through one table-driven router (``ops/gemm.py``
``route``): the hand-written 4-wave MFMA GEMM (``gemm_w4.hip``) for prefill-sized
passes and the full-batch gate_up + GLU, the skinny (``gemv.hip``) and medium-M
(``gemm_midm.hip``) decode kernels where they measured faster, and per-shape tuned
hipBLASLt solutions for the remaining decode buckets; everything around the GEMMs
is fused here.
"""
from ._ext import on_gpu, reference_mode
from .activation import act_glu, act_glu_ref
from .attention import (KV_BLOCK, DecodeWorkspace, decode_partitioning, paged_decode_attention,
                        paged_decode_attention_rope, set_prefill_persist,
                        paged_decode_ref, prefill_attention, prefill_attention_ref, prefill_tiles)
from .gemm import (fused_glu_ok, glu_linear, linear, linear_residual, mfma_gemm, norm_glu,
                   norm_linear, residual_fusable, w4_glu_ok)
from .moe import fused_moe, fused_moe_ref, router_logits
from .norm import PendingNorm, rmsnorm, rmsnorm_ref
from .rope import build_rope_cache, kv_write_v, kv_write_v_ref, rope_kv_, rope_kv_ref
from .sampling import sample, sample_ref

__all__ = [
    "on_gpu", "reference_mode", "linear", "norm_linear", "glu_linear", "norm_glu", "w4_glu_ok",
    "fused_glu_ok",
    "mfma_gemm", "linear_residual", "residual_fusable", "PendingNorm", "fused_moe", "router_logits",
    "fused_moe_ref", "act_glu", "act_glu_ref", "KV_BLOCK", "DecodeWorkspace",
    "decode_partitioning", "paged_decode_attention", "paged_decode_attention_rope",
    "paged_decode_ref", "prefill_attention", "prefill_attention_ref", "prefill_tiles",
    "set_prefill_persist", "rmsnorm", "rmsnorm_ref", "build_rope_cache", "rope_kv_",
    "rope_kv_ref", "kv_write_v", "kv_write_v_ref", "sample", "sample_ref",
]
