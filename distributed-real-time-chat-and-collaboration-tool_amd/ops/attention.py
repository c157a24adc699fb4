"""Attention: varlen causal prefill and paged decode (GQA/MQA).

HIP kernels: csrc/kernels/attention_prefill.hip, csrc/kernels/attention_decode.hip.
"""
from __future__ import annotations

import math
import os

import torch

from ._ext import check, hipk, on_gpu, ptr, stream_ptr
from .rope import v_block_tokens

KV_BLOCK = 32  # tokens per cache block (fixed by the decode kernel)
PREFILL_QTILE = 64
# Prefill attention launch form (profiles/r2j_prefill_persistent.md): persistent
# workgroups win 9-10 % on chat-length prompts, one workgroup per (query tile,
# head group) wins on long prompts (4k tokens: 8 %); parity around 430 tokens.
PERSIST_MAX_LEN = 1024
_prefill_persist = [{"1": True, "0": False}.get(os.environ.get("DRTC_PREFILL_PERSIST", ""))]


def set_prefill_persist(on: bool | None) -> None:
    """Force the prefill attention launch form (None: per call, by the
    longest sequence of the batch)."""
    _prefill_persist[0] = None if on is None else bool(on)


def prefill_persist_for(max_len: int) -> bool:
    forced = _prefill_persist[0]
    return forced if forced is not None else max_len <= PERSIST_MAX_LEN


# ----------------------------------------------------------------- prefill
def prefill_tiles(cu_seqlens: list[int]) -> tuple[list[int], list[int]]:
    """Host-side 64-row query tile map for a packed batch, longest sequences
    first (causal tiles near the end of long sequences are the heaviest)."""
    seqs = []
    for s in range(len(cu_seqlens) - 1):
        n = cu_seqlens[s + 1] - cu_seqlens[s]
        for q0 in range(0, n, PREFILL_QTILE):
            seqs.append((-(q0 + PREFILL_QTILE), s, q0))
    seqs.sort()
    return [s for _, s, _ in seqs], [q for _, _, q in seqs]


def prefill_attention_ref(qkv, cu_seqlens, Hq, Hkv, D, scale, causal=True):
    T = qkv.shape[0]
    out = torch.zeros((T, Hq * D), dtype=qkv.dtype, device=qkv.device)
    G = Hq // Hkv
    cu = [int(x) for x in cu_seqlens]
    for s in range(len(cu) - 1):
        a, b = cu[s], cu[s + 1]
        if b == a:
            continue
        n = b - a
        q = qkv[a:b, : Hq * D].reshape(n, Hq, D).float().transpose(0, 1)
        k = qkv[a:b, Hq * D:(Hq + Hkv) * D].reshape(n, Hkv, D).float().transpose(0, 1)
        v = qkv[a:b, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(n, Hkv, D).float().transpose(0, 1)
        k = k.repeat_interleave(G, dim=0)
        v = v.repeat_interleave(G, dim=0)
        sc = torch.matmul(q, k.transpose(1, 2)) * scale
        if causal:
            mask = torch.ones(n, n, dtype=torch.bool, device=qkv.device).triu(1)
            sc = sc.masked_fill(mask, float("-inf"))
        o = torch.matmul(torch.softmax(sc, dim=-1), v)
        out[a:b] = o.transpose(0, 1).reshape(n, Hq * D).to(qkv.dtype)
    return out


def prefill_attention(qkv: torch.Tensor, cu_seqlens: torch.Tensor, Hq: int, Hkv: int,
                      D: int, scale: float, causal: bool = True,
                      tiles: tuple[torch.Tensor, torch.Tensor] | None = None,
                      cu_host: list[int] | None = None,
                      out: torch.Tensor | None = None,
                      max_len: int | None = None) -> torch.Tensor:
    """Packed varlen attention reading q/k/v from the fused QKV buffer.

    qkv: [T, >= (Hq + 2Hkv) * D] bf16 (RoPE already applied);
    cu_seqlens: int32 [nseq + 1]. Returns [T, Hq * D]."""
    if not on_gpu(qkv):
        return prefill_attention_ref(qkv, cu_host if cu_host is not None else cu_seqlens.tolist(),
                                     Hq, Hkv, D, scale, causal)
    assert qkv.dtype == torch.bfloat16 and qkv.stride(1) == 1
    assert qkv.shape[1] >= (Hq + 2 * Hkv) * D and Hq % Hkv == 0
    assert cu_seqlens.dtype == torch.int32 and cu_seqlens.is_cuda
    T = qkv.shape[0]
    cu = cu_host if cu_host is not None else cu_seqlens.tolist()
    if out is None:
        # rows past cu[-1] (shape padding) are not written by the kernel: zero only
        # those (zeroing the whole [T, Hq*D] output cost ~17 us per layer and chunk,
        # profiles/r2o/r2o_headline_kernel_trace.csv.gz)
        out = torch.empty((T, Hq * D), dtype=qkv.dtype, device=qkv.device)
        if cu[-1] < T:
            out[cu[-1]:].zero_()
    assert out.stride(1) == 1 and out.shape[0] == T and out.shape[1] >= Hq * D
    if tiles is None:
        assert cu[-1] <= T
        ts, tq = prefill_tiles(cu)
        dev = qkv.device
        tiles = (torch.tensor(ts, dtype=torch.int32, device=dev),
                 torch.tensor(tq, dtype=torch.int32, device=dev))
    ntiles = tiles[0].numel()
    if max_len is None and _prefill_persist[0] is None:
        max_len = max(b - a for a, b in zip(cu, cu[1:]))
    persist = prefill_persist_for(max_len or 0)
    check(hipk().prefill_attn(out.data_ptr(), out.stride(0), qkv.data_ptr(), qkv.stride(0),
                              Hq, Hkv, D, cu_seqlens.data_ptr(), tiles[0].data_ptr(),
                              tiles[1].data_ptr(), ntiles, float(scale), int(causal),
                              int(persist), stream_ptr(qkv)), "prefill_attn")
    return out


# ------------------------------------------------------------------ decode
# Decode kernel variant: 1 = workgroup per (seq, kv head, partition) with a
# 4-wave LDS merge (default); 2 = one wave per (seq, kv head, partition), no
# merge.  Measured on MI355X (scripts/decode_attn_bench.py, Llama-3-8B heads):
# equal at batch 1024 (4.8 TB/s), v1 ahead at long contexts.
# 0 = pick per shape (decode_variant); 1 / 2 / 3 force a kernel variant
DECODE_VARIANT = int(os.environ.get("DRTC_DECODE_VARIANT", "0"))


def decode_variant(batch: int, Hkv: int, D: int, max_blocks: int) -> int:
    """Kernel variant per decode shape (profiles/r2g_decode_persistent.md):
    3 (persistent waves, next item prefetched) when there are >= 4096
    (sequence, kv head) items and D <= 128 - the serving batches (B 1024 x 8
    kv heads: 141 vs 150 us); 2 (wave per item) when the context must be
    split over partitions to fill the chip (B 8 x 4k tokens: 30 vs 53 us for
    variant 1, whose in-kernel merge pays an agent-scope fence per workgroup
    across the 8 XCD L2s); 1 otherwise (B 256 x ~1k tokens: 196 vs 206 us).
    r2l (profiles/r2l_decode_geometries.md): from 2048 items v3 also wins at
    chat lengths (Mixtral / 70B heads at B 256: 38.4 vs 40.1 / 38.9 vs 41.2 us);
    at D = 256 (Gemma-2B, one kv head) v2 wins from 1024 items (B 1024: 34.2 vs
    49.5 us; v3 holds ~400 registers there and spills)."""
    if DECODE_VARIANT:
        return DECODE_VARIANT
    items = batch * Hkv
    if D <= 128 and items >= 2048:
        return 3
    if D > 128 and items >= 1024:
        return 2
    if items < 256 and max_blocks > 8:
        return 2
    return 1
# variant 1 merges split-K partitions inside the attention kernel (last
# workgroup to finish) instead of a separate decode_reduce launch
FUSED_SPLIT_MERGE = os.environ.get("DRTC_DECODE_FUSED_MERGE", "1") != "0"


def decode_partitioning(batch: int, Hkv: int, max_blocks: int, target_wgs: int = 256,
                        variant: int | None = None, D: int = 128):
    """Static (graph-capturable) split of the context into partitions.

    Returns (blocks_per_part, max_parts).  Split-K only pays when the batch
    cannot fill the chip by itself: the sweep in profiles/ shows one partition
    per sequence winning from 512 (seq, kv head) workgroups up (e.g. batch 64 x
    8 kv heads: 84 us unsplit vs 96 us in 4 parts at ~1.7k-token contexts), and
    partitions shorter than ~8 blocks losing to the merge overhead (batch 8 at
    4k tokens: 28 us with 32-block parts vs 40 us with 4-block parts)."""
    variant = variant or decode_variant(batch, Hkv, D, max_blocks)
    per_wg = 4 if variant in (2, 3) else 1
    parts_wanted = max(1, math.ceil(target_wgs * per_wg / max(1, batch * Hkv)))
    bpp = max(8, math.ceil(max_blocks / parts_wanted))
    bpp = ((bpp + 3) // 4) * 4
    max_parts = max(1, math.ceil(max_blocks / bpp))
    return bpp, max_parts


def paged_decode_ref(q, k_cache, v_cache, block_tables, context_lens, scale):
    B, Hq, D = q.shape
    Hkv, bs = k_cache.shape[1], k_cache.shape[2]
    G = Hq // Hkv
    out = torch.zeros((B, Hq, D), dtype=q.dtype, device=q.device)
    for b in range(B):
        ctx = int(context_lens[b])
        if ctx <= 0:
            continue
        nblk = (ctx + bs - 1) // bs
        blocks = block_tables[b, :nblk].long()
        k = k_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * bs, D)[:, :ctx].float()
        v = v_block_tokens(v_cache[blocks]).permute(1, 0, 2, 3).reshape(Hkv, nblk * bs, D)
        v = v[:, :ctx].float()
        qh = q[b].reshape(Hkv, G, D).float()
        s = torch.einsum("hgd,htd->hgt", qh, k) * scale
        p = torch.softmax(s, dim=-1)
        out[b] = torch.einsum("hgt,htd->hgd", p, v).reshape(Hq, D).to(q.dtype)
    return out


class DecodeWorkspace:
    """fp32 split-K partial buffers for one (batch bucket, partitioning)."""

    def __init__(self, batch: int, Hq: int, D: int, max_parts: int, device):
        self.max_parts = max_parts
        if max_parts > 1:
            self.part_o = torch.empty((batch, Hq, max_parts, D), dtype=torch.float32, device=device)
            self.part_ml = torch.empty((batch, Hq, max_parts, 2), dtype=torch.float32, device=device)
            # per-(sequence, kv head) arrival counters of the in-kernel split-K
            # merge (variant 1); each launch leaves them at zero
            self.counters = torch.zeros(batch * Hq, dtype=torch.int32, device=device)
        else:
            self.part_o = self.part_ml = self.counters = None


def paged_decode_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           block_tables: torch.Tensor, context_lens: torch.Tensor,
                           scale: float, out: torch.Tensor | None = None,
                           blocks_per_part: int | None = None,
                           workspace: DecodeWorkspace | None = None,
                           variant: int | None = None) -> torch.Tensor:
    """One query token per sequence against the paged cache.

    q: [B, Hq, D] view (row stride may exceed Hq*D, e.g. the fused QKV row);
    block_tables: int32 [B, max_blocks]; context_lens: int32 [B]."""
    if not on_gpu(q):
        r = paged_decode_ref(q, k_cache, v_cache, block_tables, context_lens, scale)
        if out is not None:
            out.copy_(r)
            return out
        return r
    B, Hq, D = q.shape
    assert q.dtype == torch.bfloat16 and q.stride(2) == 1 and q.stride(1) == D
    nb, Hkv, bs, D2 = k_cache.shape
    assert bs == KV_BLOCK and D2 == D and k_cache.is_contiguous() and v_cache.is_contiguous()
    assert v_cache.shape == (nb, Hkv, D, bs)
    assert Hq % Hkv == 0 and Hq // Hkv <= 16
    assert block_tables.dtype == torch.int32 and block_tables.stride(1) == 1
    assert context_lens.dtype == torch.int32 and context_lens.numel() >= B
    max_blocks = block_tables.shape[1]
    variant = variant or decode_variant(B, Hkv, D, block_tables.shape[1])
    if blocks_per_part is None or workspace is None:
        blocks_per_part, max_parts = decode_partitioning(B, Hkv, max_blocks, variant=variant, D=D)
        workspace = DecodeWorkspace(B, Hq, D, max_parts, q.device)
    if out is None:
        out = torch.empty((B, Hq, D), dtype=q.dtype, device=q.device)
    assert out.is_contiguous() and out.shape == (B, Hq, D)
    counters = ptr(workspace.counters) if variant == 1 and FUSED_SPLIT_MERGE else 0
    check(hipk().paged_decode(out.data_ptr(), ptr(workspace.part_o), ptr(workspace.part_ml),
                              counters, q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                              block_tables.data_ptr(), block_tables.stride(0),
                              context_lens.data_ptr(), B, Hq, Hkv, D, float(scale),
                              workspace.max_parts, blocks_per_part, variant, stream_ptr(q)),
          "paged_decode")
    return out


# RoPE + KV write fused into the persistent decode attention (attention_decode.hip
# DecodeRope): the step's q / k / v come unrotated from the QKV GEMM output; one launch
# per layer instead of rope_kv + attention.  DRTC_DECODE_FUSED_ROPE=0 keeps the two launches.
FUSED_ROPE = os.environ.get("DRTC_DECODE_FUSED_ROPE", "1") != "0"


def paged_decode_attention_rope(qkv: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor,
                                cos_sin: torch.Tensor, Hq: int, Hkv: int, D: int,
                                k_cache: torch.Tensor, v_cache: torch.Tensor,
                                block_tables: torch.Tensor, context_lens: torch.Tensor,
                                scale: float, out: torch.Tensor | None = None,
                                blocks_per_part: int | None = None,
                                workspace: DecodeWorkspace | None = None,
                                max_wgs: int = 0) -> torch.Tensor:
    """Decode-step attention from the raw QKV rows [B, (Hq + 2 Hkv) D]: rotate q / k of
    the step's token (position ``positions[b]`` = context_lens[b] - 1), write its k / v
    into the paged cache at ``slots[b]`` and attend over the whole context - the result
    of ``rope_kv_`` followed by ``paged_decode_attention``.  On the GPU the persistent
    kernel (variant 3, D <= 128) does it in one launch; other shapes run the two ops.
    ``max_wgs`` > 0 caps the persistent grid at that many 4-wave workgroups (attention on
    part of the chip, beside another stream's GEMMs; 0: two per CU)."""
    from .rope import rope_kv_

    B = qkv.shape[0]
    q = qkv.as_strided((B, Hq, D), (qkv.stride(0), D, 1))
    variant = decode_variant(B, Hkv, D, block_tables.shape[1]) if on_gpu(qkv) else 0
    if not (on_gpu(qkv) and FUSED_ROPE and variant == 3 and D <= 128):
        rope_kv_(qkv, positions, slots, cos_sin, Hq, Hkv, D, k_cache, v_cache, KV_BLOCK)
        return paged_decode_attention(q, k_cache, v_cache, block_tables, context_lens, scale,
                                      out=out, blocks_per_part=blocks_per_part,
                                      workspace=workspace)
    assert qkv.dtype == torch.bfloat16 and qkv.stride(1) == 1
    assert qkv.shape[1] >= (Hq + 2 * Hkv) * D
    nb, hkv, bs, D2 = k_cache.shape
    assert hkv == Hkv and bs == KV_BLOCK and D2 == D and k_cache.is_contiguous()
    assert v_cache.is_contiguous() and v_cache.shape == (nb, Hkv, D, bs)
    assert positions.dtype == torch.int32 and positions.numel() >= B
    assert slots.dtype == torch.int64 and slots.numel() >= B
    assert cos_sin.dtype == torch.float32 and cos_sin.shape[1] == D and cos_sin.is_contiguous()
    assert block_tables.dtype == torch.int32 and block_tables.stride(1) == 1
    assert context_lens.dtype == torch.int32 and context_lens.numel() >= B
    if blocks_per_part is None or workspace is None:
        blocks_per_part, max_parts = decode_partitioning(B, Hkv, block_tables.shape[1],
                                                         variant=variant, D=D)
        workspace = DecodeWorkspace(B, Hq, D, max_parts, qkv.device)
    if out is None:
        out = torch.empty((B, Hq, D), dtype=qkv.dtype, device=qkv.device)
    assert out.is_contiguous() and out.shape == (B, Hq, D)
    check(hipk().paged_decode_rope(out.data_ptr(), ptr(workspace.part_o), ptr(workspace.part_ml),
                                   qkv.data_ptr(), qkv.stride(0), k_cache.data_ptr(),
                                   v_cache.data_ptr(), block_tables.data_ptr(),
                                   block_tables.stride(0), context_lens.data_ptr(), B, Hq, Hkv, D,
                                   float(scale), workspace.max_parts, blocks_per_part,
                                   positions.data_ptr(), slots.data_ptr(), cos_sin.data_ptr(),
                                   int(max_wgs), stream_ptr(qkv)), "paged_decode_rope")
    return out
