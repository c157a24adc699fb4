"""Expert parallelism with token dispatch/combine over all-to-all.

Two EP forms are provided:

* ``TransformerLM`` (models/transformer.py) with ``ep_size > 1``: tokens are
  replicated across the EP group (attention is TP-sharded), every rank runs
  its E/ep experts on the tokens routed to them and one all-reduce combines -
  the form used inside decode hipGraphs (static shapes, no host sync).
* ``ep_moe_forward`` here: tokens are *partitioned* across ranks (DP
  attention); each rank routes its tokens, ``all_to_all_single`` ships every
  (token, expert) pair to the rank owning the expert, experts run on exactly
  the tokens they received, and a second all-to-all returns the outputs for
  the weighted combine.  Per-rank traffic is 2 x top_k x T_r x H elements,
  independent of the number of experts - the right shape for RCCL over the
  point-to-point xGMI mesh (7 links per GPU all used by one all-to-all).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .. import ops


def route(x: torch.Tensor, router_w: torch.Tensor, top_k: int):
    logits = F.linear(x, router_w).float()
    topv, topi = logits.topk(top_k, dim=-1)
    return topi, torch.softmax(topv, dim=-1)


def local_experts(x: torch.Tensor, expert_ids: torch.Tensor, gate_up: torch.Tensor,
                  down: torch.Tensor, expert_offset: int, act: str) -> torch.Tensor:
    """Run each local expert on the rows addressed to it."""
    y = torch.zeros(x.shape[0], down.shape[1], dtype=x.dtype, device=x.device)
    for le in range(gate_up.shape[0]):
        rows = torch.nonzero(expert_ids == expert_offset + le, as_tuple=True)[0]
        if rows.numel() == 0:
            continue
        h = ops.act_glu(F.linear(x.index_select(0, rows), gate_up[le]), act)
        y.index_copy_(0, rows, F.linear(h, down[le]))
    return y


def ep_moe_forward(x: torch.Tensor, router_w: torch.Tensor, gate_up: torch.Tensor,
                   down: torch.Tensor, top_k: int, act: str = "silu", group=None) -> torch.Tensor:
    """MoE layer for this rank's token shard ``x`` [T_r, H]; ``gate_up`` /
    ``down`` hold this rank's E/ep experts."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    E = router_w.shape[0]
    e_local = gate_up.shape[0]
    assert e_local * world == E
    T = x.shape[0]
    topi, w = route(x, router_w, top_k)
    flat_tok = torch.arange(T, device=x.device).repeat_interleave(top_k)
    flat_e = topi.reshape(-1)
    flat_w = w.reshape(-1)
    owner = torch.div(flat_e, e_local, rounding_mode="floor")
    order = torch.argsort(owner, stable=True)
    send_counts = torch.bincount(owner, minlength=world)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    send_x = x.index_select(0, flat_tok[order])
    send_e = flat_e[order].to(torch.int64)
    recv_x = x.new_empty((sum(rc), x.shape[1]))
    recv_e = send_e.new_empty(sum(rc))
    dist.all_to_all_single(recv_x, send_x, rc, sc, group=group)
    dist.all_to_all_single(recv_e, send_e, rc, sc, group=group)
    y = local_experts(recv_x, recv_e, gate_up, down, rank * e_local, act)
    back = x.new_empty((sum(sc), x.shape[1]))
    dist.all_to_all_single(back, y, sc, rc, group=group)
    out = torch.zeros(T, x.shape[1], dtype=torch.float32, device=x.device)
    out.index_add_(0, flat_tok[order], back.float() * flat_w[order].unsqueeze(1))
    return out.to(x.dtype)


def moe_reference(x, router_w, gate_up_all, down_all, top_k, act="silu"):
    """Single-process MoE over all experts (oracle for the EP tests)."""
    topi, w = route(x, router_w, top_k)
    out = torch.zeros(x.shape[0], x.shape[1], dtype=torch.float32, device=x.device)
    for e in range(router_w.shape[0]):
        tok, slot = torch.nonzero(topi == e, as_tuple=True)
        if tok.numel() == 0:
            continue
        h = ops.act_glu(F.linear(x.index_select(0, tok), gate_up_all[e]), act)
        out.index_add_(0, tok, F.linear(h, down_all[e]).float() * w[tok, slot].unsqueeze(1))
    return out.to(x.dtype)
