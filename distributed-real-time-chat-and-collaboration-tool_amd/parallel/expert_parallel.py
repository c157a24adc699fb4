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

Three dispatch forms:

* :func:`ep_moe_a2a_cap` (default, prefill and decode) - capacity-factor
  splits: ``C = ceil(cf * T_r * k / world)`` rows per (source, destination)
  pair (``DRTC_EP_CF``, default 2.0), planned on the device by the HIP
  kernels of csrc/kernels/moe_ep.hip (ep_plan / ep_gather / ep_combine), equal
  splits, no host sync, hipGraph-capturable; moves ``2 cf T_r k H`` elements
  per rank instead of the worst case ``2 world T_r k H``.  A pair beyond a
  destination's capacity is dropped and counted in :class:`EpOverflow`; the
  caller (engine/decode_runner.py for decode, engine/engine.py for prefill)
  reads the EP-group sum together with the sampled tokens and re-runs the step
  at worst-case capacity (:func:`worst_case_capacity`), so results never
  depend on the capacity;
* :func:`ep_moe_a2a` - exact splits: per-destination row counts are
  exchanged first (a tiny all-to-all, one host sync), then variable-split
  all-to-alls move only real rows (``DRTC_EP_PREFILL=exact``, eager only).
* :func:`ep_moe_a2a_static` - capacity ``C = T_r * top_k`` (the worst case)
  in plain PyTorch ops; the oracle of the capacity form's redo path.

Local experts run on the fused HIP grouped-MFMA kernel (ops.fused_moe) with
one-hot router rows (top-1, weight 1.0): it computes only this rank's experts
and only for the rows received; padding rows of the static form point at a
non-local expert, which the kernel skips.  On CPU the same math runs through
the PyTorch reference (tests over gloo).
"""
from __future__ import annotations

import contextlib
import math
import os

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .. import ops
from ..ops._ext import check, hipk, on_gpu, stream_ptr
from ..ops.moe import MOE_GEMM_VARIANT, route_ref
from .comm import all_to_all_single

EP_CF = float(os.environ.get("DRTC_EP_CF", "2.0"))
_PLAN_MAX_PAIRS = 64 * 1024  # one-workgroup plan kernel: <= 64 pairs per thread
_worst_case = [False]


@contextlib.contextmanager
def worst_case_capacity():
    """Capacity ``T_r * k`` (nothing can be dropped) inside the block: the
    redo of a step whose capacity-factor dispatch overflowed."""
    prev, _worst_case[0] = _worst_case[0], True
    try:
        yield
    finally:
        _worst_case[0] = prev


def capacity(T: int, k: int, world: int, cf: float | None = None) -> int:
    """Rows per (source, destination) pair: ceil(cf T k / world), at most the
    worst case T k."""
    P = T * k
    if _worst_case[0]:
        return max(P, 1)
    return max(1, min(P, math.ceil((EP_CF if cf is None else cf) * P / world)))


class EpOverflow:
    """Device counter of pairs dropped by the capacity-factor dispatch during
    one forward pass (zeroed by :meth:`reset` at the pass start, summed over
    the EP group by :meth:`reduce` at its end; both are graph-capturable)."""

    def __init__(self, device):
        self.count = torch.zeros(1, dtype=torch.int32, device=device)

    def reset(self) -> None:
        self.count.zero_()

    def reduce(self, group) -> None:
        from .comm import _staged

        if _staged(group, self.count):
            c = self.count.cpu()
            dist.all_reduce(c, group=group)
            self.count.copy_(c)
        else:
            dist.all_reduce(self.count, group=group)


def ep_plan(topi: torch.Tensor, e_local: int, world: int, cap: int,
            overflow: torch.Tensor | None = None):
    """(dst_row [P], send_pair [world cap], send_e [world cap]) int32 of the
    capacity dispatch: pair p = t k + j goes to row owner cap + slot, slot =
    its rank among the pairs with the same owner in (token, pick) order; -1
    marks dropped pairs / padding rows.  Drops are added to ``overflow``."""
    P = topi.numel()
    dev = topi.device
    dst_row = torch.empty(P, dtype=torch.int32, device=dev)
    send_pair = torch.empty(world * cap, dtype=torch.int32, device=dev)
    send_e = torch.empty(world * cap, dtype=torch.int32, device=dev)
    if on_gpu(topi) and P <= _PLAN_MAX_PAIRS:
        ti = topi.reshape(-1).to(torch.int32).contiguous()
        check(hipk().ep_plan(ti.data_ptr(), P, e_local, world, cap, dst_row.data_ptr(),
                             send_pair.data_ptr(), send_e.data_ptr(),
                             overflow.data_ptr() if overflow is not None else 0,
                             stream_ptr(ti)), "ep_plan")
        return dst_row, send_pair, send_e
    flat_e = topi.reshape(-1).long()
    owner = torch.div(flat_e, e_local, rounding_mode="floor")
    slot = (F.one_hot(owner, world).cumsum(0) - 1).gather(1, owner.unsqueeze(1)).squeeze(1)
    keep = slot < cap
    row = owner * cap + slot
    dst_row.copy_(torch.where(keep, row, torch.full_like(row, -1)))
    send_pair.fill_(-1)
    send_e.fill_(-1)
    rk = torch.where(keep, row, torch.full_like(row, world * cap))  # dropped: a scratch row
    sp = torch.full((world * cap + 1,), -1, dtype=torch.int32, device=dev)
    se = sp.clone()
    sp.index_copy_(0, rk, torch.arange(P, dtype=torch.int32, device=dev))
    se.index_copy_(0, rk, flat_e.to(torch.int32))
    send_pair.copy_(sp[:-1])
    send_e.copy_(se[:-1])
    if overflow is not None:
        overflow.add_((~keep).sum().to(overflow.dtype))
    return dst_row, send_pair, send_e


def ep_gather(x: torch.Tensor, send_pair: torch.Tensor, k: int) -> torch.Tensor:
    """send_x [world cap, H]: row r = x[send_pair[r] // k] (padding rows unspecified)."""
    rows, H = send_pair.numel(), x.shape[1]
    out = x.new_empty((rows, H))
    if on_gpu(x) and x.stride(1) == 1:
        check(hipk().ep_gather(out.data_ptr(), x.data_ptr(), send_pair.data_ptr(), rows, k, H,
                               x.stride(0), stream_ptr(x)), "ep_gather")
        return out
    idx = torch.div(send_pair.long().clamp(min=0), k, rounding_mode="floor")
    return x.index_select(0, idx)


def ep_combine(back: torch.Tensor, dst_row: torch.Tensor, w: torch.Tensor, T: int,
               k: int) -> torch.Tensor:
    """out[t] = sum_j w[t, j] back[dst_row[t k + j]] in fp32, fixed order j;
    dropped pairs (row -1) contribute nothing."""
    H = back.shape[1]
    wf = w.reshape(-1).float().contiguous()
    if on_gpu(back):
        out = back.new_empty((T, H))
        check(hipk().ep_combine(out.data_ptr(), back.data_ptr(), dst_row.data_ptr(),
                                wf.data_ptr(), T, k, H, stream_ptr(back)), "ep_combine")
        return out
    keep = (dst_row >= 0).float()
    g = back.index_select(0, dst_row.long().clamp(min=0)).float()
    acc = torch.zeros(T, H, dtype=torch.float32, device=back.device)
    g = g.view(T, k, H) * (wf * keep).view(T, k, 1)
    for j in range(k):  # fixed order, as the kernel
        acc += g[:, j]
    return acc.to(back.dtype)


def route(x: torch.Tensor, router_w: torch.Tensor, top_k: int):
    """(expert ids [T, k], weights [T, k] fp32): top-k of the bf16 router logits,
    softmax over the selected k, ties to the lower id (the fused kernel's rule)."""
    from ..ops.moe import router_logits

    return route_ref(router_logits(x, router_w), top_k)


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


def ep_moe_a2a_cap(x: torch.Tensor, topi: torch.Tensor, w: torch.Tensor,
                   gate_up: torch.Tensor, down: torch.Tensor, act: str = "silu", group=None,
                   num_experts: int | None = None, workspace: torch.Tensor | None = None,
                   overflow: EpOverflow | None = None, cf: float | None = None) -> torch.Tensor:
    """Capacity-factor EP MoE: device-planned dispatch (ep_plan + ep_gather),
    equal-split all-to-alls of ``world * C`` rows, this rank's experts on the
    received rows (fused grouped-MFMA kernel: no host sync at any size),
    all-to-all back and a fixed-order fp32 combine (ep_combine).  Equal to
    :func:`ep_moe_a2a` whenever nothing overflows (``overflow`` stays 0)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    e_local = gate_up.shape[0]
    E = num_experts or e_local * world
    T, k = topi.shape
    C = capacity(T, k, world, cf)
    dst_row, send_pair, send_e = ep_plan(topi, e_local, world, C,
                                         overflow.count if overflow is not None else None)
    send_x = ep_gather(x, send_pair, k)
    recv_x = torch.empty_like(send_x)
    recv_e = torch.empty_like(send_e)
    all_to_all_single(recv_e, send_e, group=group)
    all_to_all_single(recv_x, send_x, group=group)
    # padding rows address a non-local expert of the receiver: skipped by the kernel
    foreign = (rank * e_local + e_local) % E if e_local < E else 0
    recv_e = torch.where(recv_e < 0, torch.full_like(recv_e, foreign), recv_e)
    if on_gpu(recv_x):
        logits = _one_hot_logits(recv_e, E, x.dtype)
        y = ops.fused_moe(recv_x, logits, gate_up, down, 1, act, E, rank * e_local,
                          workspace=workspace, variant=MOE_GEMM_VARIANT)
    else:
        y = local_experts(recv_x, recv_e, gate_up, down, rank * e_local, act, E, workspace)
    back = torch.empty_like(y)
    all_to_all_single(back, y, group=group)
    return ep_combine(back, dst_row, w, T, k)


def ep_moe_forward(x: torch.Tensor, router_w: torch.Tensor, gate_up: torch.Tensor,
                   down: torch.Tensor, top_k: int, act: str = "silu", group=None,
                   static: bool = False, form: str | None = None,
                   overflow: EpOverflow | None = None, cf: float | None = None) -> torch.Tensor:
    """Route this rank's token shard with the (replicated) router, then
    dispatch / compute / combine over the EP group (``form``: "cap" (default),
    "exact" or "static"; ``static=True`` is the old spelling of "static")."""
    topi, w = route(x, router_w, top_k)
    form = form or ("static" if static else "cap")
    if form == "cap":
        return ep_moe_a2a_cap(x, topi, w, gate_up, down, act, group, router_w.shape[0],
                              overflow=overflow, cf=cf)
    fn = ep_moe_a2a_static if form == "static" else ep_moe_a2a
    return fn(x, topi, w, gate_up, down, act, group, router_w.shape[0])


def moe_reference(x, router_w, gate_up_all, down_all, top_k, act="silu"):
    """Single-process MoE over all experts (oracle for the EP tests)."""
    return ops.fused_moe_ref(x, F.linear(x, router_w), gate_up_all, down_all, top_k, act)
