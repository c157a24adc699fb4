"""Paged KV cache sized for MI355X HBM (288 GB per GPU).

One contiguous allocation per engine, carved into per-layer views:
  k[layer] : [num_blocks, Hkv, 32, D]   token-major (MFMA A-operand rows)
  v[layer] : [num_blocks, Hkv, D, 32]   storage shape; a block holds 8 groups
             of 4 tokens, dim-major inside a group (P.V A-operand: 4 tokens of
             one dim = 8 contiguous bytes; a decode write spans 2*D bytes)
The block count is derived from the free HBM left after the weights
(``torch.cuda.mem_get_info``) times ``kv_fraction``; on a 288 GB MI355X with
Llama-3-8B that is ~1.5 M cached tokens.  Blocks are handed out by the
native :class:`BlockAllocator` (C++ free list, see csrc/runtime).  No
reference counterpart: the reference keeps no model state (hosted Gemini,
llm_server/llm_server.py:33); SURVEY §7.1 "paged KV allocator sized from free HBM".
"""
from __future__ import annotations

import torch

from ..ops import KV_BLOCK
from ..models.config import ModelConfig
from .block_allocator import BlockAllocator


def blocks_for_budget(cfg: ModelConfig, hkv_local: int, n_layers: int, budget_bytes: int,
                      dtype_bytes: int = 2) -> int:
    per_block = 2 * n_layers * hkv_local * KV_BLOCK * cfg.head_dim * dtype_bytes
    return max(0, budget_bytes // per_block)


class PagedKVCache:
    def __init__(self, cfg: ModelConfig, hkv_local: int, num_blocks: int,
                 device: torch.device | str, dtype=torch.bfloat16):
        self.cfg = cfg
        self.block_size = KV_BLOCK
        self.num_blocks = int(num_blocks)
        self.hkv = hkv_local
        D = cfg.head_dim
        L = cfg.num_layers
        per = self.num_blocks * hkv_local * KV_BLOCK * D
        # zero-filled: stale/uninitialised bytes in partially filled blocks
        # must never be NaN (they are multiplied by p = 0 in P.V).
        self.buffer = torch.zeros((L, 2, per), dtype=dtype, device=device)
        self.layers = []
        for l in range(L):
            k = self.buffer[l, 0].view(self.num_blocks, hkv_local, KV_BLOCK, D)
            v = self.buffer[l, 1].view(self.num_blocks, hkv_local, D, KV_BLOCK)
            self.layers.append((k, v))
        # block 0 is reserved as the padding target of graph-padded slots
        self.allocator = BlockAllocator(self.num_blocks, reserved=1)

    def __getitem__(self, i):
        return self.layers[i]

    def __len__(self):
        return len(self.layers)

    @property
    def bytes(self) -> int:
        return self.buffer.numel() * self.buffer.element_size()

    @property
    def capacity_tokens(self) -> int:
        return (self.num_blocks - 1) * KV_BLOCK

    @staticmethod
    def auto_num_blocks(cfg: ModelConfig, hkv_local: int, device, kv_fraction: float = 0.85,
                        reserve_bytes: int = 8 << 30, max_blocks: int | None = None,
                        hbm_budget: float | None = None, weight_bytes: int | None = None,
                        min_blocks: int = 0) -> int:
        """KV blocks for an engine on ``device``: ``kv_fraction`` of the HBM free beyond
        ``reserve_bytes`` (activations, GEMM workspaces, graphs) - or, with ``hbm_budget``
        (engine groups sharing a GPU, llm.server --serve ...:mem=F), what is left of
        hbm_budget x the GPU's total HBM after the group's weights (``weight_bytes``; this
        process's allocations when not given) and the reserve, whatever the other groups on the
        GPU - in other processes or in this one - hold or start in what order."""
        dev = torch.device(device)
        if dev.type == "cuda":
            # blocks the caching allocator holds but no tensor uses are free HBM here: release
            # them so that neither the free figure nor this process's own share counts them
            torch.cuda.empty_cache()
            free, total = torch.cuda.mem_get_info(dev)
            budget = int(max(0, free - reserve_bytes) * kv_fraction)
            if hbm_budget is not None:
                mine = torch.cuda.memory_reserved(dev) if weight_bytes is None else weight_bytes
                left = int(hbm_budget * total) - mine - reserve_bytes
                if blocks_for_budget(cfg, hkv_local, cfg.num_layers, max(left, 0)) < min_blocks:
                    # ``min_blocks``: the cache of one max_model_len sequence
                    raise ValueError(
                        f"{cfg.name}: an HBM budget of {hbm_budget:.2f} x {total / 1e9:.0f} GB "
                        f"on {dev} leaves {left / 1e9:.1f} GB for the KV cache after "
                        f"{mine / 1e9:.1f} GB of weights and the {reserve_bytes / 1e9:.0f} GB "
                        f"reserve: less than one {min_blocks}-block sequence needs")
                budget = min(budget, max(left, 0))
        else:
            budget = 256 << 20
        n = blocks_for_budget(cfg, hkv_local, cfg.num_layers, budget)
        if max_blocks is not None:
            n = min(n, max_blocks)
        return max(n, 2)
