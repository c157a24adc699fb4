"""Rotary embedding applied in place on fused QKV, fused with the paged KV write.

HIP kernel: csrc/kernels/norm_act_rope.hip (rope_kv_kernel).

KV-cache layout (per layer):
  k_cache [num_blocks, Hkv, block_size, D]   token-major rows
  v_cache [num_blocks, Hkv, D, block_size]   storage shape; inside a block the
      tokens are 8 groups of 4, dim-major within a group ([8][D][4], see
      ``v_block_tokens`` / ``v_block_storage`` and csrc/kernels/norm_act_rope.hip)
"""
from __future__ import annotations

import math

import torch

from ._ext import check, hipk, on_gpu, ptr, stream_ptr


def build_rope_cache(max_pos: int, head_dim: int, theta: float,
                     scaling: dict | None = None, device=None) -> torch.Tensor:
    """[max_pos, head_dim] fp32 table: first half cos, second half sin.

    ``scaling`` supports the Llama-3.1 "llama3" frequency remap
    (factor / low_freq_factor / high_freq_factor / original_max_position_embeddings).
    """
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2.0 / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling["low_freq_factor"], scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    pos = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(pos, inv)
    table = torch.cat([torch.cos(ang), torch.sin(ang)], dim=-1).to(torch.float32)
    return table.to(device) if device is not None else table


V_GROUP = 4  # tokens per dim-major group of a V cache block


def v_block_tokens(vb: torch.Tensor) -> torch.Tensor:
    """V cache blocks [..., D, bs] (storage) -> token-major [..., bs, D]."""
    *lead, D, bs = vb.shape
    return vb.reshape(*lead, bs // V_GROUP, D, V_GROUP).transpose(-1, -2).reshape(*lead, bs, D)


def v_block_storage(v: torch.Tensor) -> torch.Tensor:
    """Token-major [..., bs, D] -> V cache block storage [..., D, bs]."""
    *lead, bs, D = v.shape
    return v.reshape(*lead, bs // V_GROUP, V_GROUP, D).transpose(-1, -2).reshape(*lead, D, bs)


def rope_kv_ref(qkv, positions, slots, cos_sin, Hq, Hkv, D, k_cache, v_cache, block_size):
    T = qkv.shape[0]
    nh = Hq + Hkv
    heads = qkv[:, : nh * D].reshape(T, nh, D).float()
    cs = cos_sin[positions.long()]
    c = cs[:, None, : D // 2]
    s = cs[:, None, D // 2:]
    x1, x2 = heads[..., : D // 2], heads[..., D // 2:]
    new = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(qkv.dtype)
    qkv[:, : nh * D] = new.reshape(T, nh * D)
    if slots is not None and k_cache is not None:
        sl = slots.long()
        valid = sl >= 0
        blk = torch.div(sl[valid], block_size, rounding_mode="floor")
        off = sl[valid] % block_size
        k = new[:, Hq:][valid]
        v = qkv[:, nh * D:(nh + Hkv) * D].reshape(T, Hkv, D)[valid]
        k_cache[blk, :, off, :] = k
        if v_cache is not None:
            nb, hkv, d, bs = v_cache.shape
            vg = v_cache.view(nb, hkv, bs // V_GROUP, d, V_GROUP)
            vg[blk, :, torch.div(off, V_GROUP, rounding_mode="floor"), :, off % V_GROUP] = v
    return qkv


def kv_write_v_ref(v_cache, qkv, seg_tok, seg_len, seg_blk, Hq, Hkv, D):
    bs = v_cache.shape[-1]
    for t0, n, b in zip(seg_tok.tolist(), seg_len.tolist(), seg_blk.tolist()):
        v = qkv[t0:t0 + n, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(n, Hkv, D)
        blk = torch.zeros(Hkv, bs, D, dtype=v_cache.dtype, device=v_cache.device)
        blk[:, :n] = v.permute(1, 0, 2)
        v_cache[b] = v_block_storage(blk)


def kv_write_v(v_cache: torch.Tensor, qkv: torch.Tensor, segs, Hq: int, Hkv: int, D: int) -> None:
    """Prefill V write: ``segs`` = (tok_start, n_tokens, block) int32 tensors,
    one entry per 32-token cache block of the packed prompt batch."""
    seg_tok, seg_len, seg_blk = segs
    if not on_gpu(qkv):
        kv_write_v_ref(v_cache, qkv, seg_tok, seg_len, seg_blk, Hq, Hkv, D)
        return
    nb, hkv, d, bs = v_cache.shape
    assert hkv == Hkv and d == D and v_cache.is_contiguous() and qkv.stride(1) == 1
    for t in segs:
        assert t.dtype == torch.int32 and t.is_cuda and t.numel() == seg_tok.numel()
    check(hipk().kv_write_v(v_cache.data_ptr(), qkv.data_ptr(), qkv.stride(0), seg_tok.data_ptr(),
                            seg_len.data_ptr(), seg_blk.data_ptr(), seg_tok.numel(), Hq, Hkv, D, bs,
                            stream_ptr(qkv)), "kv_write_v")


def rope_kv_(qkv: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor | None,
             cos_sin: torch.Tensor, Hq: int, Hkv: int, D: int,
             k_cache: torch.Tensor | None, v_cache: torch.Tensor | None,
             block_size: int, write_v: bool = True) -> torch.Tensor:
    """Rotate q/k heads of ``qkv`` [T, (Hq+2Hkv)*D] in place; write k (and v,
    unless ``write_v`` is False) of tokens with ``slots[t] >= 0`` into the
    paged cache."""
    if not on_gpu(qkv):
        return rope_kv_ref(qkv, positions, slots, cos_sin, Hq, Hkv, D, k_cache,
                           v_cache if write_v else None, block_size)
    T = qkv.shape[0]
    assert qkv.dtype == torch.bfloat16 and qkv.stride(1) == 1
    assert qkv.shape[1] >= (Hq + 2 * Hkv) * D
    assert positions.dtype == torch.int32 and positions.numel() >= T
    assert cos_sin.dtype == torch.float32 and cos_sin.shape[1] == D and cos_sin.is_contiguous()
    if slots is not None:
        assert slots.dtype == torch.int64 and slots.numel() >= T
        assert k_cache is not None and v_cache is not None
        assert k_cache.shape[1:] == (Hkv, block_size, D) and k_cache.is_contiguous()
        assert v_cache.shape[1:] == (Hkv, D, block_size) and v_cache.is_contiguous()
    check(hipk().rope_kv(qkv.data_ptr(), T, qkv.stride(0), positions.data_ptr(), ptr(slots),
                         cos_sin.data_ptr(), Hq, Hkv, D, ptr(k_cache), ptr(v_cache),
                         block_size, int(write_v), stream_ptr(qkv)), "rope_kv")
    return qkv
