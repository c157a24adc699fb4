"""Expert parallelism with token dispatch/combine over all-to-all.

Served form (models/transformer.py, ``ep_size > 1``): every rank owns E/ep
experts and a SHARD of the tokens - the sequence-parallel rows of a prefill
chunk, or the ``B / ep`` slice of a decode batch.  A rank routes its own
tokens, ships every (token, expert) pair to the rank that owns the expert
(``all_to_all_single``), runs its local experts on exactly the rows it
received, ships the expert outputs back (second all-to-all) and combines them
with the router weights in fp32 in a fixed order.  Per-rank traffic is
``2 x top_k x T_r x H`` elements, independent of the number of experts: the
right shape for RCCL over the point-to-point xGMI mesh (one all-to-all keeps
all 7 links of a GPU busy), instead of an all-reduce of the full ``[T, H]``
output (ref call site replaced: llm_server/llm_server.py:403, the hosted
context-suggestion model).

Two dispatch forms:

* :func:`ep_moe_a2a` - exact splits: per-destination row counts are
  exchanged first (a tiny all-to-all, one host sync), then variable-split
  all-to-alls move only real rows.  Prefill (eager).
* :func:`ep_moe_a2a_static` - static capacity ``C = T_r * top_k`` rows per
  (source, destination) pair (the worst case: no token is ever dropped, so
  results equal the exact form), placement computed on the device with fixed
  shapes, equal-split all-to-alls: no host sync, hipGraph-capturable.  Decode.

Local experts run on the fused HIP grouped-MFMA kernel (ops.fused_moe) with
one-hot router rows (top-1, weight 1.0): it computes only this rank's experts
and only for the rows received; padding rows of the static form point at a
non-local expert, which the kernel skips.  On CPU the same math runs through
the PyTorch reference (tests over gloo).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .. import ops
from ..ops.moe import route_ref
from .comm import all_to_all_single


def route(x: torch.Tensor, router_w: torch.Tensor, top_k: int):
    """(expert ids [T, k], weights [T, k] fp32): top-k of the bf16 router logits,
    softmax over the selected k, ties to the lower id (the fused kernel's rule)."""
    return route_ref(F.linear(x, router_w), top_k)


def _one_hot_logits(expert_ids: torch.Tensor, num_experts: int, dtype) -> torch.Tensor:
    lg = torch.full((expert_ids.shape[0], num_experts), -30000.0, dtype=dtype,
                    device=expert_ids.device)
    lg.scatter_(1, expert_ids.long().unsqueeze(1), 0.0)
    return lg


def local_experts(x: torch.Tensor, expert_ids: torch.Tensor, gate_up: torch.Tensor,
                  down: torch.Tensor, expert_offset: int, act: str, num_experts: int,
                  workspace: torch.Tensor | None = None) -> torch.Tensor:
    """y[r] = expert_{expert_ids[r]}(x[r]) for the rows addressed to this
    rank's experts [expert_offset, expert_offset + E_local); rows addressed
    elsewhere (static-form padding) come back unspecified."""
    if x.shape[0] == 0:
        return x.new_empty((0, down.shape[1]))
    logits = _one_hot_logits(expert_ids, num_experts, x.dtype)
    return ops.fused_moe(x.contiguous(), logits, gate_up, down, 1, act, num_experts,
                         expert_offset, workspace=workspace)


def ep_moe_a2a(x: torch.Tensor, topi: torch.Tensor, w: torch.Tensor, gate_up: torch.Tensor,
               down: torch.Tensor, act: str = "silu", group=None, num_experts: int | None = None,
               workspace: torch.Tensor | None = None) -> torch.Tensor:
    """Exact-split EP MoE for this rank's token shard ``x`` [T_r, H] routed to
    ``topi`` / ``w`` [T_r, k]; ``gate_up`` / ``down`` hold this rank's experts."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    e_local = gate_up.shape[0]
    E = num_experts or e_local * world
    T, k = topi.shape
    flat_tok = torch.arange(T, device=x.device).repeat_interleave(k)
    flat_e = topi.reshape(-1)
    owner = torch.div(flat_e, e_local, rounding_mode="floor")
    order = torch.argsort(owner, stable=True)
    send_counts = F.one_hot(owner, world).sum(0)
    recv_counts = torch.empty_like(send_counts)
    all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    send_x = x.index_select(0, flat_tok[order])
    send_e = flat_e[order].to(torch.int32)
    recv_x = x.new_empty((sum(rc), x.shape[1]))
    recv_e = send_e.new_empty(sum(rc))
    all_to_all_single(recv_x, send_x, rc, sc, group=group)
    all_to_all_single(recv_e, send_e, rc, sc, group=group)
    y = local_experts(recv_x, recv_e, gate_up, down, rank * e_local, act, E, workspace)
    back = x.new_empty((sum(sc), x.shape[1]))
    all_to_all_single(back, y, sc, rc, group=group)
    out = torch.zeros(T, x.shape[1], dtype=torch.float32, device=x.device)
    out.index_add_(0, flat_tok[order], back.float() * w.reshape(-1)[order].unsqueeze(1))
    return out.to(x.dtype)


def ep_moe_a2a_static(x: torch.Tensor, topi: torch.Tensor, w: torch.Tensor,
                      gate_up: torch.Tensor, down: torch.Tensor, act: str = "silu", group=None,
                      num_experts: int | None = None,
                      workspace: torch.Tensor | None = None) -> torch.Tensor:
    """Static-capacity EP MoE (same result as :func:`ep_moe_a2a`): every
    shape depends only on (T_r, k, world), every index is computed on the
    device, the all-to-alls use equal splits - capturable in a hipGraph."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    e_local = gate_up.shape[0]
    E = num_experts or e_local * world
    T, k = topi.shape
    H = x.shape[1]
    C = T * k  # per-destination capacity: the worst case, nothing is dropped
    flat_e = topi.reshape(-1).long()
    owner = torch.div(flat_e, e_local, rounding_mode="floor")               # [T*k]
    oh = F.one_hot(owner, world)                                            # [T*k, world]
    slot = (oh.cumsum(0) - 1).gather(1, owner.unsqueeze(1)).squeeze(1)      # rank within dest
    dst_row = owner * C + slot                                              # row in [world*C]
    send_x = x.new_zeros((world * C, H))
    send_x.index_copy_(0, dst_row, x.repeat_interleave(k, dim=0))
    # padding rows address a non-local expert of the receiver: skipped by the kernel
    pad_e = torch.full((world * C,), -1, dtype=torch.int32, device=x.device)
    pad_e.index_copy_(0, dst_row, flat_e.to(torch.int32))
    recv_x = torch.empty_like(send_x)
    recv_e = torch.empty_like(pad_e)
    all_to_all_single(recv_x, send_x, group=group)
    all_to_all_single(recv_e, pad_e, group=group)
    foreign = (rank * e_local + e_local) % E if e_local < E else 0
    recv_e = torch.where(recv_e < 0, torch.full_like(recv_e, foreign), recv_e)
    y = local_experts(recv_x, recv_e, gate_up, down, rank * e_local, act, E, workspace)
    back = torch.empty_like(y)
    all_to_all_single(back, y, group=group)
    contrib = back.index_select(0, dst_row).float() * w.reshape(-1, 1)
    return contrib.view(T, k, H).sum(1).to(x.dtype)


def ep_moe_forward(x: torch.Tensor, router_w: torch.Tensor, gate_up: torch.Tensor,
                   down: torch.Tensor, top_k: int, act: str = "silu", group=None,
                   static: bool = False) -> torch.Tensor:
    """Route this rank's token shard with the (replicated) router, then
    dispatch / compute / combine over the EP group."""
    topi, w = route(x, router_w, top_k)
    fn = ep_moe_a2a_static if static else ep_moe_a2a
    return fn(x, topi, w, gate_up, down, act, group, router_w.shape[0])


def moe_reference(x, router_w, gate_up_all, down_all, top_k, act="silu"):
    """Single-process MoE over all experts (oracle for the EP tests)."""
    return ops.fused_moe_ref(x, F.linear(x, router_w), gate_up_all, down_all, top_k, act)
