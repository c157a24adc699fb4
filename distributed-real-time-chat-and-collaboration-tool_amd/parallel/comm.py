"""Process-group plumbing: one process per GPU, torch.distributed over RCCL.

On ROCm the ``"nccl"`` backend *is* RCCL; on CPU (tests) ``"gloo"`` is used
with the same code path.  A :class:`ParallelContext` carries the tensor-
parallel (TP) and expert-parallel (EP) groups a model shard needs; the
data-parallel (DP) dimension is replica-level (one engine per GPU, requests
routed by the LLM service) and needs no collective on the hot path.
The reference has no collectives at all (gRPC only); these
are the X1-X3 rows of SURVEY §2.3.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


def env_rank_world() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_distributed(backend: str | None = None, device: torch.device | None = None) -> tuple[int, int]:
    """Initialise the default process group from torchrun's env (idempotent)."""
    rank, world, local = env_rank_world()
    if world <= 1:
        return 0, 1
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        # DRTC_DIST_BACKEND=gloo rehearses multi-rank GPU code paths with
        # several ranks on ONE GPU (RCCL refuses two ranks per device)
        backend = os.environ.get("DRTC_DIST_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local % torch.cuda.device_count())
    dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world


# ------------------------------------------------------------ collectives
# RCCL ("nccl") takes device tensors directly.  gloo implements all-to-all,
# reduce-scatter and all-gather-into only for host tensors; the one-GPU
# multi-rank rehearsals (DRTC_DIST_BACKEND=gloo, eager) stage device tensors
# through host memory here.  Production TP/EP groups are RCCL and never stage.
def _staged(group, *ts) -> bool:
    return any(t.is_cuda for t in ts) and dist.get_backend(group) == "gloo"


def all_to_all_single(out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None,
                      group=None) -> torch.Tensor:
    if _staged(group, out, inp):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
    return out


def reduce_scatter_tensor(out: torch.Tensor, inp: torch.Tensor, group=None) -> torch.Tensor:
    if _staged(group, out, inp):
        o = out.float().cpu()
        dist.reduce_scatter_tensor(o, inp.float().cpu(), group=group)
        out.copy_(o)
    else:
        dist.reduce_scatter_tensor(out, inp, group=group)
    return out


def all_gather_into_tensor(out: torch.Tensor, inp: torch.Tensor, group=None) -> torch.Tensor:
    if _staged(group, out, inp):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)
    return out


@dataclass
class ParallelContext:
    tp_size: int = 1
    tp_rank: int = 0
    tp_group: object = None
    ep_size: int = 1
    ep_rank: int = 0
    ep_group: object = None
    custom_ar: object = None     # CustomAllReduce over the TP group (decode-sized messages)
    # sequence parallelism for TP prefill: after o/down projections the partial
    # sums are reduce-scattered over tokens, norms/residuals run on T/tp rows,
    # and the rows are all-gathered before the next column-parallel GEMM
    sequence_parallel: bool = field(
        default_factory=lambda: os.environ.get("DRTC_SEQUENCE_PARALLEL", "1") != "0")
    # MoE with ep_size > 1: "a2a" = token dispatch/combine over all-to-all
    # (parallel/expert_parallel.py); "allreduce" = replicated tokens + all-reduce
    ep_combine: str = field(default_factory=lambda: os.environ.get("DRTC_EP_COMBINE", "a2a"))

    @staticmethod
    def single() -> "ParallelContext":
        return ParallelContext()

    @staticmethod
    def from_world(tp: bool = True, ep: bool = False) -> "ParallelContext":
        """Use the whole default group for TP (and/or EP)."""
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return ParallelContext()
        r, w = dist.get_rank(), dist.get_world_size()
        ctx = ParallelContext()
        if tp:
            ctx.tp_size, ctx.tp_rank, ctx.tp_group = w, r, dist.group.WORLD
        if ep:
            ctx.ep_size, ctx.ep_rank, ctx.ep_group = w, r, dist.group.WORLD
        return ctx

    def enable_custom_allreduce(self, max_bytes: int = 4 << 20) -> None:
        """Route small TP all-reduces through the one-shot IPC kernel
        (parallel/custom_allreduce.py); larger ones stay on RCCL."""
        if self.tp_size <= 1 or not torch.cuda.is_available():
            return
        from .custom_allreduce import CustomAllReduce
        ranks = dist.get_process_group_ranks(self.tp_group)
        cpu_group = dist.new_group(ranks=ranks, backend="gloo")
        self.custom_ar = CustomAllReduce(cpu_group, max_bytes=max_bytes)

    def agree_min(self, v: int) -> int:
        """MIN of an integer over every rank that runs this model in lockstep
        (TP and EP groups).  Used for host-side sizing decisions that must be
        identical on all ranks - e.g. the KV-cache block count, which each
        rank derives from its own free HBM: differing counts would make the
        SPMD schedulers admit / preempt differently and issue collectives of
        different sizes (a hang, or silent corruption with the custom
        all-reduce)."""
        groups = [g for size, g in ((self.tp_size, self.tp_group), (self.ep_size, self.ep_group))
                  if size > 1]
        for g in groups:
            dev = (torch.device("cuda", torch.cuda.current_device())
                   if dist.get_backend(g) == "nccl" else torch.device("cpu"))
            t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=g)
            v = int(t.item())
        return int(v)

    def reduce_norm(self, x: torch.Tensor, residual: torch.Tensor | None, w: torch.Tensor,
                    eps: float, gemma: bool) -> torch.Tensor:
        """norm(all_reduce_tp(x) + residual) * w, residual updated in place: one
        fused launch (custom one-shot all-reduce + add + RMSNorm) when the
        message qualifies, else the all-reduce followed by the norm kernel."""
        from .. import ops

        car = self.custom_ar
        if (self.tp_size > 1 and car is not None and residual is not None
                and car.can_fuse_norm(x, residual)):
            return car.all_reduce_rmsnorm(x, residual, w, eps, gemma)
        return ops.rmsnorm(self.all_reduce_tp(x), w, eps, gemma, residual=residual)

    def all_reduce_tp(self, x: torch.Tensor) -> torch.Tensor:
        if self.tp_size > 1:
            if self.custom_ar is not None and self.custom_ar.can(x):
                return self.custom_ar.all_reduce(x)
            dist.all_reduce(x, group=self.tp_group)
        return x

    def all_reduce_ep(self, x: torch.Tensor) -> torch.Tensor:
        if self.ep_size > 1:
            if (self.custom_ar is not None and self.ep_group is self.tp_group
                    and self.custom_ar.can(x)):
                return self.custom_ar.all_reduce(x)
            dist.all_reduce(x, group=self.ep_group)
        return x

    def sp_ok(self, T: int) -> bool:
        """Whether a prefill pass of T tokens runs sequence-parallel."""
        return self.tp_size > 1 and self.sequence_parallel and T % self.tp_size == 0

    def reduce_scatter_rows(self, x: torch.Tensor) -> torch.Tensor:
        """[T, H] partial sums -> this rank's [T / tp, H] rows of the sum."""
        out = x.new_empty((x.shape[0] // self.tp_size, x.shape[1]))
        return reduce_scatter_tensor(out, x.contiguous(), group=self.tp_group)

    def all_gather_rows(self, x: torch.Tensor) -> torch.Tensor:
        """This rank's [T / tp, H] rows -> [T, H] on every rank."""
        out = x.new_empty((x.shape[0] * self.tp_size, x.shape[1]))
        return all_gather_into_tensor(out, x.contiguous(), group=self.tp_group)

    def all_gather_tp_lastdim(self, x: torch.Tensor) -> torch.Tensor:
        if self.tp_size == 1:
            return x
        parts = [torch.empty_like(x) for _ in range(self.tp_size)]
        dist.all_gather(parts, x.contiguous(), group=self.tp_group)
        return torch.cat(parts, dim=-1)
