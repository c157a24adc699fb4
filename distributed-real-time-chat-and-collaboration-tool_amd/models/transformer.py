"""Decoder-only transformer (Llama-3 / Gemma / Mixtral families), inference-only.

MI355X-first layout decisions
  * fused projections: one QKV GEMM and one gate|up GEMM per layer, routed by
    ``ops.linear`` (ops/gemm.py): the hand-written 4-wave MFMA GEMM (gemm_w4.hip)
    for prefill passes - gate_up with the SiLU/GELU-GLU and o / down with the
    residual add in the epilogue - and for the full-batch decode gate_up + GLU;
    skinny / medium-M hand kernels and per-shape tuned hipBLASLt solutions for
    the other decode buckets.  Between the GEMMs every op is a fused HIP kernel:
    add+RMSNorm, RoPE + paged-KV write (in place on the QKV output; in decode
    inside the attention launch), MFMA attention reading q/k/v straight out of
    the QKV buffer;
  * tensor parallel over RCCL: heads / intermediate columns sharded, one
    all-reduce after o_proj and one after down_proj (or the MoE combine),
    vocab-parallel LM head + all-gather;
  * sequence parallel TP prefill (ParallelContext.sequence_parallel): the
    o / down partial sums are reduce-scattered over tokens, norms and the
    residual stream live on T/tp rows per rank, and rows are all-gathered
    only in front of the column-parallel QKV / gate_up GEMMs;
  * expert parallel for MoE: each rank owns E/ep experts; tokens are
    dispatched to the expert owners and combined back over all-to-all
    (parallel/expert_parallel.py: exact splits in prefill, where the rows are
    already sequence-sharded; decode keeps replicated tokens + the EP
    capacity-factor all-to-all in decode too: device-planned, graph-
    capturable, overflow counted and redone at worst-case capacity by the
    engine; DRTC_EP_DECODE=allreduce keeps replicated tokens + the EP
    all-reduce);
  * decode is static-shaped (persistent metadata buffers) so the whole step
    is hipGraph-capturable by the engine.

Random-init bf16 weights (no checkpoints in this environment); a fixed seed
and ``full_then_shard=True`` make TP=N numerically comparable to TP=1.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import os

import torch
import torch.nn.functional as F

from .. import ops
from ..parallel.comm import ParallelContext, all_gather_into_tensor
from .config import ModelConfig


# EP decode: the capacity-factor all-to-all (default) or the replicated-token
# fused MoE + EP all-reduce (DRTC_EP_DECODE=allreduce); EP prefill: capacity
# form (default) or exact splits with one host sync per layer (=exact)
_EP_DECODE_A2A = os.environ.get("DRTC_EP_DECODE", "a2a") == "a2a"
_EP_PREFILL = os.environ.get("DRTC_EP_PREFILL", "cap")

# Two-stream micro-batched decode: the step's rows in two halves, one per
# stream inside the captured graph, with each half's paged attention (HBM-bound) ordered to
# run beside the other half's projections (per-CU operand-ingest bound).  DRTC_DECODE_MICRO=2
# enables it for decode batches of at least DECODE_MICRO_MIN_B rows (dense TP=1 models);
# DRTC_DECODE_MICRO_WGS caps the attention's persistent grid (0: two workgroups per CU);
# DRTC_DECODE_MICRO_PINGPONG=0 drops the cross-stream attention ordering (two free chains).
DECODE_MICRO = int(os.environ.get("DRTC_DECODE_MICRO", "0"))
DECODE_MICRO_MIN_B = int(os.environ.get("DRTC_DECODE_MICRO_MIN_B", "512"))
DECODE_MICRO_WGS = int(os.environ.get("DRTC_DECODE_MICRO_WGS", "0"))
DECODE_MICRO_PINGPONG = os.environ.get("DRTC_DECODE_MICRO_PINGPONG", "1") != "0"


@dataclass
class PrefillMeta:
    positions: torch.Tensor      # int32 [T]
    slots: torch.Tensor          # int64 [T]  (-1: do not cache)
    cu_seqlens: torch.Tensor     # int32 [n+1]
    cu_host: list
    tiles: tuple | None          # (tile_seq, tile_q0) int32 device tensors
    last_idx: torch.Tensor       # int64 [n] index of each sequence's last token
    v_segs: tuple | None = None  # (tok, len, block) int32: block-wise V write
    # mixed step (engine/engine.py::_run_mixed): rows [n_prefill, T) are one
    # decode token per running sequence, attended against the paged cache
    # with ``decode``'s block tables / context lengths
    decode: "DecodeMeta | None" = None
    n_prefill: int = 0
    max_len: int | None = None   # longest sequence (prefill attention launch form)


@dataclass
class DecodeMeta:
    positions: torch.Tensor      # int32 [B]
    slots: torch.Tensor          # int64 [B]
    block_tables: torch.Tensor   # int32 [B, max_blocks]
    context_lens: torch.Tensor   # int32 [B]
    blocks_per_part: int
    workspace: object            # ops.DecodeWorkspace


class ShardInfo:
    def __init__(self, cfg: ModelConfig, pc: ParallelContext):
        tp, r = pc.tp_size, pc.tp_rank
        assert cfg.num_heads % tp == 0, "num_heads must divide by TP"
        self.hq = cfg.num_heads // tp
        if cfg.num_kv_heads >= tp:
            assert cfg.num_kv_heads % tp == 0
            self.hkv = cfg.num_kv_heads // tp
            self.kv_heads = list(range(r * self.hkv, (r + 1) * self.hkv))
        else:  # fewer kv heads than ranks: replicate (e.g. MQA)
            self.hkv = 1
            self.kv_heads = [r * cfg.num_kv_heads // tp]
        assert cfg.intermediate_size % tp == 0 and cfg.vocab_size % tp == 0
        self.inter = cfg.intermediate_size // tp
        self.vocab = cfg.vocab_size // tp
        self.q_heads = list(range(r * self.hq, (r + 1) * self.hq))
        ep = pc.ep_size
        if cfg.is_moe:
            assert cfg.num_experts % ep == 0
            self.n_local_experts = cfg.num_experts // ep
            self.expert_offset = pc.ep_rank * self.n_local_experts
            # experts are not TP-sharded when EP is used; with EP=1 they are
            self.expert_inter = cfg.intermediate_size if ep > 1 else self.inter
        self.tp, self.rank = tp, r


class TransformerLM:
    """Weights + forward for one model shard on one device."""

    def __init__(self, cfg: ModelConfig, device: torch.device | str = "cpu",
                 pc: ParallelContext | None = None, seed: int = 0,
                 full_then_shard: bool | None = None, dtype=torch.bfloat16):
        self.cfg = cfg
        self.device = torch.device(device)
        self.pc = pc or ParallelContext.single()
        self.dtype = dtype
        self.sh = ShardInfo(cfg, self.pc)
        if full_then_shard is None:
            full_then_shard = cfg.num_params() < 200_000_000
        self._init_weights(seed, full_then_shard)
        self.cos_sin = ops.build_rope_cache(cfg.max_position, cfg.head_dim, cfg.rope_theta,
                                            cfg.rope_scaling, device=self.device)
        self.qkv_dim = (self.sh.hq + 2 * self.sh.hkv) * cfg.head_dim
        self.moe_ws = None
        if cfg.is_moe and self.device.type == "cuda":
            # one persistent scratch shared by prefill chunks and every decode
            # graph (they replay serially on one stream)
            from ..ops import moe as _moe_ops
            self.moe_ws = _moe_ops.make_workspace(_moe_ops.MOE_CHUNK, cfg.hidden_size,
                                                  self.sh.expert_inter, self.sh.n_local_experts,
                                                  cfg.experts_per_token, self.device)
        self.ep_overflow = None
        self._ep_cap_used = False
        self._side_stream = None   # micro-batched decode: second stream + its split-K workspace
        self._side_ws = None
        self._micro_metas: dict = {}
        if cfg.is_moe and self.pc.ep_size > 1:
            from ..parallel.expert_parallel import EpOverflow
            self.ep_overflow = EpOverflow(self.device)

    # ------------------------------------------------------------ weights
    def _init_weights(self, seed: int, full_then_shard: bool) -> None:
        cfg, sh, dev, dt = self.cfg, self.sh, self.device, self.dtype
        std = cfg.init_std
        H, D, I = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size
        gen = torch.Generator(device="cpu").manual_seed(seed)
        dev_gen = None
        if not full_then_shard and dev.type == "cuda":
            dev_gen = torch.Generator(device=dev).manual_seed(seed * 1000 + 7 + self.pc.tp_rank)

        def rnd(*shape):
            if full_then_shard:
                return (torch.randn(*shape, generator=gen, dtype=torch.float32) * std).to(dt)
            t = torch.empty(*shape, dtype=dt, device=dev)
            if dev_gen is not None:
                return t.normal_(0.0, std, generator=dev_gen)
            return t.normal_(0.0, std, generator=gen)

        def put(t):
            return t.to(dev).contiguous()

        def rows(t, idx_blocks, block):
            return torch.cat([t[i * block:(i + 1) * block] for i in idx_blocks], dim=0)

        def norm_w():
            if cfg.gemma_norm:
                return torch.zeros(H, dtype=dt, device=dev)  # (1 + w) = 1
            return torch.ones(H, dtype=dt, device=dev)

        self.embed = put(rnd(cfg.vocab_size, H))
        self.layers = []
        for _ in range(cfg.num_layers):
            L = {}
            if full_then_shard:
                wq = rnd(cfg.num_heads * D, H)
                wk = rnd(cfg.num_kv_heads * D, H)
                wv = rnd(cfg.num_kv_heads * D, H)
                wo = rnd(H, cfg.num_heads * D)
                L["qkv"] = put(torch.cat([rows(wq, sh.q_heads, D), rows(wk, sh.kv_heads, D),
                                          rows(wv, sh.kv_heads, D)], 0))
                cols = torch.cat([torch.arange(h * D, (h + 1) * D) for h in sh.q_heads])
                L["o"] = put(wo[:, cols])
            else:
                L["qkv"] = put(rnd((sh.hq + 2 * sh.hkv) * D, H))
                L["o"] = put(rnd(H, sh.hq * D))
            L["ln_in"] = norm_w()
            L["ln_post"] = norm_w()
            if cfg.is_moe:
                E, EI = sh.n_local_experts, sh.expert_inter
                if full_then_shard:
                    wr = rnd(cfg.num_experts, H)
                    gus, downs = [], []
                    for e in range(cfg.num_experts):
                        g, u, d = rnd(I, H), rnd(I, H), rnd(H, I)
                        if sh.expert_offset <= e < sh.expert_offset + E:
                            if self.pc.ep_size > 1 or sh.tp == 1:
                                gus.append(torch.cat([g, u], 0))
                                downs.append(d)
                            else:
                                r0 = sh.rank * sh.inter
                                gus.append(torch.cat([g[r0:r0 + sh.inter], u[r0:r0 + sh.inter]], 0))
                                downs.append(d[:, r0:r0 + sh.inter])
                    L["router"] = put(wr)
                    L["gate_up"] = put(torch.stack(gus))
                    L["down"] = put(torch.stack(downs))
                else:
                    L["router"] = put(rnd(cfg.num_experts, H))
                    L["gate_up"] = put(rnd(E, 2 * EI, H))
                    L["down"] = put(rnd(E, H, EI))
            else:
                if full_then_shard:
                    g, u, d = rnd(I, H), rnd(I, H), rnd(H, I)
                    r0 = sh.rank * sh.inter
                    L["gate_up"] = put(torch.cat([g[r0:r0 + sh.inter], u[r0:r0 + sh.inter]], 0))
                    L["down"] = put(d[:, r0:r0 + sh.inter])
                else:
                    L["gate_up"] = put(rnd(2 * sh.inter, H))
                    L["down"] = put(rnd(H, sh.inter))
            self.layers.append(L)
        self.final_norm = norm_w()
        if cfg.tie_embeddings:
            v0 = sh.rank * sh.vocab
            self.lm_head = self.embed[v0:v0 + sh.vocab]
        else:
            if full_then_shard:
                full = rnd(cfg.vocab_size, H)
                v0 = sh.rank * sh.vocab
                self.lm_head = put(full[v0:v0 + sh.vocab])
            else:
                self.lm_head = put(rnd(sh.vocab, H))

    def weight_bytes(self) -> int:
        n = self.embed.numel() + self.final_norm.numel()
        for L in self.layers:
            n += sum(t.numel() for t in L.values())
        if not self.cfg.tie_embeddings:
            n += self.lm_head.numel()
        return n * self.embed.element_size()

    # ------------------------------------------------------------ forward
    def _embed(self, ids: torch.Tensor) -> torch.Tensor:
        h = F.embedding(ids, self.embed)
        if self.cfg.embed_scale:
            # Gemma: x * sqrt(H) with the normaliser rounded to the activation
            # dtype; a python scalar keeps the op graph-capturable (no H2D copy)
            h = h * float(torch.tensor(math.sqrt(self.cfg.hidden_size), dtype=h.dtype))
        return h

    def _mlp(self, L: dict, x: ops.PendingNorm, decode: bool = False) -> torch.Tensor:
        if self.cfg.is_moe:
            return self._moe(L, x.materialize(), decode), False
        if ops.fused_glu_ok(x.x, L["gate_up"], self.cfg.act):
            # prefill / decode batches with a fused form: gate_up GEMM with the GLU in its
            # epilogue (gemm_w4, or a tuned gated gemm_xd form)
            h = ops.norm_glu(x, L["gate_up"], self.cfg.act)
            res = self._fusable_residual(h, x)
            if res is not None:
                return ops.linear_residual(h, L["down"], res), True
            y = ops.linear(h, L["down"])
        else:
            gu = ops.norm_linear(x, L["gate_up"])
            res = self._fusable_residual(gu, x)
            if res is not None:
                return ops.linear_residual(ops.act_glu(gu, self.cfg.act), L["down"], res), True
            y = ops.glu_linear(gu, L["down"], self.cfg.act)
        if decode and self.pc.tp_size > 1:
            return y, False, True  # reduced by the next norm (fused all-reduce + add + norm)
        return self.pc.all_reduce_tp(y), False

    def _fusable_residual(self, a: torch.Tensor, x: ops.PendingNorm) -> torch.Tensor | None:
        """The residual stream the o / down projection may add into inside its
        GEMM epilogue (ops.linear_residual: prefill-sized passes, TP=1, where
        the all-reduce would otherwise have to come before the add)."""
        if self.pc.tp_size != 1:
            return None
        res = x.stream()
        return res if ops.residual_fusable(a, res) else None

    def _moe_ep_a2a(self, L: dict, x_rows: torch.Tensor, static: bool) -> torch.Tensor:
        """This rank's token rows through the EP group's experts over
        all-to-all (dispatch to the expert owners, combine back)."""
        from ..parallel import expert_parallel as ep

        cfg, pc = self.cfg, self.pc
        topi, w = ep.route(x_rows, L["router"], cfg.experts_per_token)
        if static or _EP_PREFILL != "exact":
            self._ep_cap_used = True
            return ep.ep_moe_a2a_cap(x_rows, topi, w, L["gate_up"], L["down"], cfg.act,
                                     pc.ep_group, cfg.num_experts, self.moe_ws,
                                     overflow=self.ep_overflow)
        return ep.ep_moe_a2a(x_rows, topi, w, L["gate_up"], L["down"], cfg.act, pc.ep_group,
                             cfg.num_experts, self.moe_ws)

    def _ep_begin(self) -> None:
        """Start of a forward pass: zero the EP overflow counter."""
        if self.ep_overflow is not None:
            self.ep_overflow.reset()
        self._ep_cap_used = False

    def _ep_end(self, logits: torch.Tensor) -> torch.Tensor:
        """End of a forward pass: sum the dropped-pair counts over the EP group
        (every rank took the same dispatch path, so all call the collective)."""
        if self.ep_overflow is not None and self._ep_cap_used:
            self.ep_overflow.reduce(self.pc.ep_group)
        return logits

    def _moe(self, L: dict, x: torch.Tensor, decode: bool = False) -> torch.Tensor:
        """Top-k routed experts (Mixtral: softmax over the top-2 logits).

        GPU: the fused HIP MoE (ops/moe.py: device-side routing + grouped
        MFMA GEMMs, static launch shapes -> the same code runs eagerly in
        prefill and inside the decode hipGraphs).  CPU: per-expert gather
        (reference semantics).  With EP, tokens replicated over the group
        (decode / non-SP prefill) are split into per-rank slices for the
        all-to-all form and all-gathered afterwards."""
        cfg, sh, pc = self.cfg, self.sh, self.pc
        T = x.shape[0]
        a2a = (pc.ep_size > 1 and T % pc.ep_size == 0 and
               (pc.ep_combine == "a2a" if not decode else _EP_DECODE_A2A))
        if a2a:
            t = T // pc.ep_size
            rows = x[pc.ep_rank * t:(pc.ep_rank + 1) * t]
            y = self._moe_ep_a2a(L, rows, static=decode)
            out = x.new_empty((T, x.shape[1]))
            all_gather_into_tensor(out, y.contiguous(), group=pc.ep_group)
            return out
        if ops.on_gpu(x):
            logits = ops.router_logits(x, L["router"], contiguous=False)  # [E, T] read in place
            out = ops.fused_moe(x, logits, L["gate_up"], L["down"],
                                cfg.experts_per_token, cfg.act, cfg.num_experts,
                                sh.expert_offset, workspace=self.moe_ws)
            if self.pc.ep_size > 1:
                return self.pc.all_reduce_ep(out)
            return self.pc.all_reduce_tp(out)
        logits = F.linear(x, L["router"]).float()
        topv, topi = logits.topk(cfg.experts_per_token, dim=-1)
        wts = torch.softmax(topv, dim=-1)
        out = torch.zeros(x.shape[0], x.shape[1], dtype=torch.float32, device=x.device)
        for le in range(sh.n_local_experts):
            e = sh.expert_offset + le
            tok, slot = torch.nonzero(topi == e, as_tuple=True)
            if tok.numel() == 0:
                continue
            xe = x.index_select(0, tok)
            h = ops.act_glu(F.linear(xe, L["gate_up"][le]), cfg.act)
            ye = F.linear(h, L["down"][le]).float() * wts[tok, slot].unsqueeze(1)
            out.index_add_(0, tok, ye)
        out = out.to(x.dtype)
        if self.pc.ep_size > 1:
            return self.pc.all_reduce_ep(out)
        return self.pc.all_reduce_tp(out)

    def _layers(self, h: torch.Tensor, attn_fn, decode: bool = False) -> torch.Tensor:
        """Pre-norm residual stack.  Each sublayer receives its input as an
        ops.PendingNorm (norm(x + residual) not yet computed), so a small
        decode batch can fuse the norm into the first projection."""
        cfg = self.cfg
        x = ops.PendingNorm(h, None, self.layers[0]["ln_in"], cfg.rms_eps, cfg.gemma_norm)
        n = len(self.layers)
        for i, L in enumerate(self.layers):
            # (o, added[, partial]): added = the projection already added the
            # residual stream in its GEMM epilogue, o IS the new stream;
            # partial = o is still a TP partial sum - the next norm runs the
            # all-reduce fused with the residual add (ParallelContext.reduce_norm)
            o, added, *part = attn_fn(i, L, x)
            x = ops.PendingNorm(o, None if added else x.stream(), L["ln_post"], cfg.rms_eps,
                                cfg.gemma_norm, pc=self.pc if part and part[0] else None)
            m, added, *part = self._mlp(L, x, decode)
            nxt = self.layers[i + 1]["ln_in"] if i + 1 < n else self.final_norm
            x = ops.PendingNorm(m, None if added else x.stream(), nxt, cfg.rms_eps, cfg.gemma_norm,
                                pc=self.pc if part and part[0] else None)
        return x.materialize()

    def _logits(self, x: torch.Tensor) -> torch.Tensor:
        logits = ops.linear(x, self.lm_head)
        return self.pc.all_gather_tp_lastdim(logits)

    def forward_prefill(self, ids: torch.Tensor, meta: PrefillMeta, kv_caches) -> torch.Tensor:
        """Packed varlen prefill (optionally with decode rows appended, see
        PrefillMeta.decode). Returns logits of the rows in ``meta.last_idx``:
        each sequence's last token, then every decode row."""
        self._ep_begin()
        if meta.decode is None and self.pc.sp_ok(ids.shape[0]):
            return self._ep_end(self._forward_prefill_sp(ids, meta, kv_caches))
        cfg, sh = self.cfg, self.sh
        D = cfg.head_dim

        def attn(i, L, x):
            qkv = ops.norm_linear(x, L["qkv"])
            kc, vc = kv_caches[i] if kv_caches is not None else (None, None)
            blockwise_v = kc is not None and meta.v_segs is not None
            ops.rope_kv_(qkv, meta.positions, meta.slots if kc is not None else None,
                         self.cos_sin, sh.hq, sh.hkv, D, kc, vc, ops.KV_BLOCK,
                         write_v=not blockwise_v)
            if blockwise_v:
                ops.kv_write_v(vc, qkv, meta.v_segs, sh.hq, sh.hkv, D)
            if meta.decode is None:
                a = ops.prefill_attention(qkv, meta.cu_seqlens, sh.hq, sh.hkv, D,
                                          cfg.attn_scale, True, tiles=meta.tiles,
                                          cu_host=meta.cu_host, max_len=meta.max_len)
            else:
                a = self._attn_mixed(qkv, meta, kc, vc)
            if i == last:
                # Every position's K/V is cached and attended to by now; only
                # each sequence's last token feeds the logits, so the last
                # layer's o-projection, MLP and final norm run on those rows
                # alone (exact: the other rows' outputs are never read).
                a = a.index_select(0, meta.last_idx)
                x.select_rows(meta.last_idx)
            res = self._fusable_residual(a, x)
            if res is not None:
                return ops.linear_residual(a, L["o"], res), True
            return self.pc.all_reduce_tp(ops.linear(a, L["o"])), False

        last = len(self.layers) - 1
        x = self._layers(self._embed(ids), attn)
        return self._ep_end(self._logits(x))

    def _attn_mixed(self, qkv: torch.Tensor, meta: PrefillMeta, kc, vc) -> torch.Tensor:
        """Attention of a mixed step: causal varlen attention over the prefill
        rows, paged-cache attention for the decode rows (their K/V were just
        written by rope_kv_), both into one [T, hq * D] buffer."""
        cfg, sh = self.cfg, self.sh
        D, Tp, dm = cfg.head_dim, meta.n_prefill, meta.decode
        T = qkv.shape[0]
        Bd = T - Tp
        a = qkv.new_empty((T, sh.hq * D))
        ap = ops.prefill_attention(qkv[:Tp], meta.cu_seqlens, sh.hq, sh.hkv, D, cfg.attn_scale,
                                   True, tiles=meta.tiles, cu_host=meta.cu_host,
                                   max_len=meta.max_len, out=a[:Tp])
        if ap.data_ptr() != a.data_ptr():  # CPU reference returns a new tensor
            a[:Tp].copy_(ap)
        if meta.cu_host[-1] < Tp:
            a[meta.cu_host[-1]:Tp].zero_()  # shape-padding rows: never written by the kernel
        q = qkv[Tp:].as_strided((Bd, sh.hq, D), (qkv.stride(0), D, 1))
        ops.paged_decode_attention(q, kc, vc, dm.block_tables, dm.context_lens, cfg.attn_scale,
                                   out=a[Tp:].view(Bd, sh.hq, D),
                                   blocks_per_part=dm.blocks_per_part, workspace=dm.workspace)
        return a

    def _attn_prefill(self, i: int, L: dict, xn: torch.Tensor, meta: PrefillMeta, kv_caches):
        """QKV + RoPE/KV write + causal attention of a packed prefill chunk on
        this rank's heads; returns the attention output [T, hq * D]."""
        cfg, sh = self.cfg, self.sh
        D = cfg.head_dim
        qkv = ops.linear(xn, L["qkv"])
        kc, vc = kv_caches[i] if kv_caches is not None else (None, None)
        blockwise_v = kc is not None and meta.v_segs is not None
        ops.rope_kv_(qkv, meta.positions, meta.slots if kc is not None else None,
                     self.cos_sin, sh.hq, sh.hkv, D, kc, vc, ops.KV_BLOCK, write_v=not blockwise_v)
        if blockwise_v:
            ops.kv_write_v(vc, qkv, meta.v_segs, sh.hq, sh.hkv, D)
        return ops.prefill_attention(qkv, meta.cu_seqlens, sh.hq, sh.hkv, D, cfg.attn_scale,
                                     True, tiles=meta.tiles, cu_host=meta.cu_host,
                                     max_len=meta.max_len)

    def _forward_prefill_sp(self, ids: torch.Tensor, meta: PrefillMeta, kv_caches) -> torch.Tensor:
        """Sequence-parallel TP prefill (tp | T).  Rank r holds rows
        [r T/tp, (r+1) T/tp) of the residual stream; per layer:

          norm(local rows) -> all-gather -> QKV (column-parallel) -> attention
          on this rank's heads -> o_proj partial -> reduce-scatter -> + residual
          norm(local rows) -> dense MLP: all-gather -> gate_up -> act -> down ->
                              reduce-scatter;  MoE (EP): expert all-to-all of
                              the local rows only (no gather at all)

        i.e. the per-sublayer all-reduce of [T, H] becomes a reduce-scatter +
        all-gather of the same bytes, while the norms, residual adds and the
        MoE dispatch work on T/tp rows.  The last layer continues on each
        sequence's last token only (replicated, all-reduce form)."""
        cfg, pc = self.cfg, self.pc
        tp, r = pc.tp_size, pc.tp_rank
        T = ids.shape[0]
        t = T // tp
        n = len(self.layers)
        moe_a2a = cfg.is_moe and pc.ep_size > 1 and pc.ep_combine == "a2a" and \
            pc.ep_group is pc.tp_group
        x = ops.PendingNorm(self._embed(ids[r * t:(r + 1) * t]), None, self.layers[0]["ln_in"],
                            cfg.rms_eps, cfg.gemma_norm)
        for i, L in enumerate(self.layers):
            xn = pc.all_gather_rows(x.materialize())
            a = self._attn_prefill(i, L, xn, meta, kv_caches)
            if i == n - 1:
                # every position is cached: only the last token of each sequence
                # feeds the logits; finish this layer on those rows, replicated
                a = a.index_select(0, meta.last_idx)
                res = pc.all_gather_rows(x.stream()).index_select(0, meta.last_idx)
                o = pc.all_reduce_tp(ops.linear(a, L["o"]))
                xr = ops.PendingNorm(o, res, L["ln_post"], cfg.rms_eps, cfg.gemma_norm)
                m, added = self._mlp(L, xr)
                xf = ops.PendingNorm(m, None if added else xr.stream(), self.final_norm,
                                     cfg.rms_eps, cfg.gemma_norm)
                return self._logits(xf.materialize())
            o_rows = pc.reduce_scatter_rows(ops.linear(a, L["o"]))
            x = ops.PendingNorm(o_rows, x.stream(), L["ln_post"], cfg.rms_eps, cfg.gemma_norm)
            if cfg.is_moe and moe_a2a:
                m_rows = self._moe_ep_a2a(L, x.materialize(), static=False)
            elif cfg.is_moe:
                # experts TP-sharded over the intermediate dim: every rank needs
                # every token, partial outputs are reduce-scattered
                xg = pc.all_gather_rows(x.materialize())
                part = ops.fused_moe(xg, ops.router_logits(xg, L["router"], contiguous=False),
                                     L["gate_up"], L["down"], cfg.experts_per_token, cfg.act,
                                     cfg.num_experts, self.sh.expert_offset,
                                     workspace=self.moe_ws) \
                    if ops.on_gpu(xg) else ops.fused_moe_ref(
                        xg, F.linear(xg, L["router"]), L["gate_up"], L["down"],
                        cfg.experts_per_token, cfg.act, self.sh.expert_offset)
                m_rows = pc.reduce_scatter_rows(part)
            else:
                xg = pc.all_gather_rows(x.materialize())
                if ops.w4_glu_ok(xg, L["gate_up"], cfg.act):
                    h = ops.mfma_gemm(xg, L["gate_up"], cfg.act, variant=7, group_m=8)
                else:
                    h = ops.act_glu(ops.linear(xg, L["gate_up"]), cfg.act)
                m_rows = pc.reduce_scatter_rows(ops.linear(h, L["down"]))
            x = ops.PendingNorm(m_rows, x.stream(), self.layers[i + 1]["ln_in"], cfg.rms_eps,
                                cfg.gemma_norm)
        raise AssertionError("unreachable")

    def forward_decode(self, ids: torch.Tensor, meta: DecodeMeta, kv_caches,
                       attn_out: torch.Tensor | None = None) -> torch.Tensor:
        """One token per sequence; static shapes (graph-capturable)."""
        cfg, sh = self.cfg, self.sh
        D = cfg.head_dim
        B = ids.shape[0]

        def attn(i, L, x):
            qkv = ops.norm_linear(x, L["qkv"])
            kc, vc = kv_caches[i]
            # RoPE + the step's KV write inside the attention launch (persistent kernel)
            a = ops.paged_decode_attention_rope(qkv, meta.positions, meta.slots, self.cos_sin,
                                                sh.hq, sh.hkv, D, kc, vc, meta.block_tables,
                                                meta.context_lens, cfg.attn_scale, out=attn_out,
                                                blocks_per_part=meta.blocks_per_part,
                                                workspace=meta.workspace)
            o = ops.linear(a.view(B, sh.hq * D), L["o"])
            if self.pc.tp_size > 1:
                return o, False, True  # reduced by the next norm (fused all-reduce + add + norm)
            return o, False

        if self.decode_micro_ok(B):
            return self._forward_decode_micro(ids, meta, kv_caches, attn_out)
        self._ep_begin()
        x = self._layers(self._embed(ids), attn, decode=True)
        return self._ep_end(self._logits(x))

    # ------------------------------------------------------------ micro-batched decode
    def decode_micro_ok(self, B: int) -> bool:
        """Whether a decode step of B rows runs as two micro-batches on two streams."""
        return (DECODE_MICRO >= 2 and B >= DECODE_MICRO_MIN_B and B % 2 == 0
                and self.device.type == "cuda" and self.pc.tp_size == 1
                and self.pc.ep_size == 1 and not self.cfg.is_moe and self.cfg.head_dim <= 128)

    def _micro_meta(self, meta: DecodeMeta, lo: int, hi: int) -> DecodeMeta:
        """Rows [lo, hi) of a decode step's metadata (views of its persistent buffers) with
        the attention partitioning and workspace of a batch of hi - lo rows; cached per
        (buffer, range) so a graph capture reuses what the eager warm-up built."""
        key = (meta.positions.data_ptr(), meta.block_tables.data_ptr(), lo, hi)
        m = self._micro_metas.get(key)
        if m is None:
            n, sh = hi - lo, self.sh
            bt = meta.block_tables[lo:hi]
            bpp, parts = ops.decode_partitioning(n, sh.hkv, bt.shape[1], D=self.cfg.head_dim)
            ws = ops.DecodeWorkspace(n, sh.hq, self.cfg.head_dim, parts, self.device)
            m = DecodeMeta(positions=meta.positions[lo:hi], slots=meta.slots[lo:hi],
                           block_tables=bt, context_lens=meta.context_lens[lo:hi],
                           blocks_per_part=bpp, workspace=ws)
            self._micro_metas[key] = m
        return m

    def _forward_decode_micro(self, ids: torch.Tensor, meta: DecodeMeta, kv_caches,
                              attn_out: torch.Tensor | None) -> torch.Tensor:
        """forward_decode on two half-batches, one per stream: the caller's (current) stream
        runs rows [0, B/2), a side stream - forked from it and joined back, so the whole step
        stays one capturable graph - rows [B/2, B) with a private split-K workspace.  With
        ping-pong ordering half A's layer-i attention waits for half B's layer-(i-1)
        attention and B's waits for A's, so the two attentions never run together and each
        overlaps the other half's projections.  Same per-row math as forward_decode (each
        row's GEMMs, norms and attention see only that row), logits on all B rows at once."""
        cfg, sh = self.cfg, self.sh
        D = cfg.head_dim
        B = ids.shape[0]
        h = B // 2
        if self._side_stream is None:  # created by the eager warm-up, before any capture
            self._side_stream = torch.cuda.Stream(self.device)
            self._side_ws = ops.gemm.new_gemm_workspace(self.device)
        main = torch.cuda.current_stream(self.device)
        streams = (main, self._side_stream)
        wss = (None, self._side_ws)
        rows = ((0, h), (h, B))
        metas = [self._micro_meta(meta, lo, hi) for lo, hi in rows]
        outs = [attn_out[lo:hi] if attn_out is not None else None for lo, hi in rows]
        hidden = self._embed(ids)
        streams[1].wait_stream(main)
        xs = [ops.PendingNorm(hidden[lo:hi], None, self.layers[0]["ln_in"], cfg.rms_eps,
                              cfg.gemma_norm) for lo, hi in rows]
        ev_attn: list = [None, None]
        n = len(self.layers)
        for i, L in enumerate(self.layers):
            kc, vc = kv_caches[i]
            nxt = self.layers[i + 1]["ln_in"] if i + 1 < n else self.final_norm
            for j in (0, 1):
                with torch.cuda.stream(streams[j]), ops.gemm.private_workspace(wss[j]):
                    x, m = xs[j], metas[j]
                    qkv = ops.norm_linear(x, L["qkv"])
                    if DECODE_MICRO_PINGPONG and ev_attn[1 - j] is not None:
                        streams[j].wait_event(ev_attn[1 - j])
                    a = ops.paged_decode_attention_rope(
                        qkv, m.positions, m.slots, self.cos_sin, sh.hq, sh.hkv, D, kc, vc,
                        m.block_tables, m.context_lens, cfg.attn_scale, out=outs[j],
                        blocks_per_part=m.blocks_per_part, workspace=m.workspace,
                        max_wgs=DECODE_MICRO_WGS)
                    if DECODE_MICRO_PINGPONG:
                        ev = torch.cuda.Event()
                        ev.record(streams[j])
                        ev_attn[j] = ev
                    o = ops.linear(a.view(a.shape[0], sh.hq * D), L["o"])
                    x = ops.PendingNorm(o, x.stream(), L["ln_post"], cfg.rms_eps, cfg.gemma_norm)
                    mo, added, *_ = self._mlp(L, x, decode=True)
                    xs[j] = ops.PendingNorm(mo, None if added else x.stream(), nxt, cfg.rms_eps,
                                            cfg.gemma_norm)
        finals = []
        for j in (0, 1):
            with torch.cuda.stream(streams[j]), ops.gemm.private_workspace(wss[j]):
                finals.append(xs[j].materialize())
        main.wait_stream(streams[1])
        # every tensor the side stream read or wrote is still referenced here, and the main
        # stream has joined it: later main-stream reuse of that memory is ordered after it
        x = torch.cat(finals)
        del finals, xs, hidden
        return self._logits(x)

    # ------------------------------------------------------------ reference
    def forward_reference(self, ids_list: list[list[int]]) -> list[torch.Tensor]:
        """Plain full-sequence causal forward (no cache) -> per-sequence logits
        of every position; used by tests to check prefill+decode equivalence."""
        outs = []
        cfg, sh = self.cfg, self.sh
        for ids in ids_list:
            n = len(ids)
            t = torch.tensor(ids, dtype=torch.long, device=self.device)
            meta = PrefillMeta(
                positions=torch.arange(n, dtype=torch.int32, device=self.device),
                slots=torch.full((n,), -1, dtype=torch.int64, device=self.device),
                cu_seqlens=torch.tensor([0, n], dtype=torch.int32, device=self.device),
                cu_host=[0, n], tiles=None,
                last_idx=torch.arange(n, dtype=torch.int64, device=self.device))
            outs.append(self.forward_prefill(t, meta, None))
        return outs
