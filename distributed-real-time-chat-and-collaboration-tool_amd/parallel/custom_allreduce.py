"""One-/two-shot P2P all-reduce for tensor-parallel messages.

Kernel + memory protocol: csrc/kernels/allreduce.hip.  Each rank allocates
one uncached device buffer (flags + double-buffered staging), exports it as
an IPC handle, and maps every peer's buffer; the handles travel over a CPU
(gloo) group, so no RCCL call is involved.  A call is a single kernel launch
with static arguments - capturable into the decode hipGraph - and gives every
rank bit-identical sums (fixed rank order).

Used by ``ParallelContext.all_reduce_tp`` for bf16 messages up to
``max_bytes`` (default 4 MiB: decode-sized [batch, hidden] tensors); larger
messages (prefill) stay on RCCL's ring/tree algorithms.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops._ext import check, hipk, stream_ptr


class CustomAllReduce:
    def __init__(self, group=None, device: torch.device | None = None,
                 max_bytes: int = 4 << 20, two_shot_min_bytes: int = 256 << 10):
        """``group``: a CPU-capable (gloo) process group over the TP ranks."""
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("custom all-reduce supports up to 8 ranks (one xGMI hive)")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.stage_elems = max_bytes // 2
        self.max_bytes = max_bytes
        # messages from this size on use the two-shot (reduce-scatter +
        # all-gather) kernel: 2(N-1)/N of the message read per rank, not N-1x
        self.two_shot_min_bytes = two_shot_min_bytes
        lib = hipk()
        with torch.cuda.device(self.device):
            self.base = lib.ar_alloc(lib.custom_ar_buffer_bytes(self.stage_elems))
            handle = lib.ar_ipc_get(self.base)
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        self._opened = []
        bases = []
        with torch.cuda.device(self.device):
            for r, h in enumerate(handles):
                if r == self.rank:
                    bases.append(self.base)
                else:
                    p = lib.ar_ipc_open(h)
                    self._opened.append(p)
                    bases.append(p)
        self.bases = bases
        dist.barrier(group=group)

    def can(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous()
                and x.numel() % 8 == 0 and x.numel() * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None,
                   two_shot: bool | None = None) -> torch.Tensor:
        """Sum of ``x`` over the group (in place unless ``out`` is given).
        ``two_shot`` (default: by size, world > 2) picks the kernel; every
        rank of a group must make the same choice for the same call."""
        assert self.can(x), "tensor not eligible for the custom all-reduce"
        out = x if out is None else out
        if two_shot is None:
            two_shot = self.world > 2 and x.numel() * 2 >= self.two_shot_min_bytes
        check(hipk().custom_allreduce(out.data_ptr(), x.data_ptr(), x.numel(), self.bases,
                                      self.rank, self.stage_elems, int(two_shot), stream_ptr(x)),
              "custom_allreduce")
        return out

    def can_fuse_norm(self, x: torch.Tensor, residual: torch.Tensor) -> bool:
        """Whether all_reduce_rmsnorm takes [rows, H] (one-shot, rows whole in
        one block's fixed staging chunk)."""
        if not (self.can(x) and x.dim() == 2 and residual.is_contiguous()
                and residual.shape == x.shape and residual.dtype == x.dtype):
            return False
        H = x.shape[1]
        chunk = (self.stage_elems // 8 + 63) // 64
        return H % 8 == 0 and H <= 16384 and chunk >= H // 8 and \
            -(-x.shape[0] // (chunk // (H // 8))) <= 64

    def all_reduce_rmsnorm(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                           eps: float, gemma: bool = False,
                           out: torch.Tensor | None = None) -> torch.Tensor:
        """One launch: residual += sum over ranks of x (rounded to bf16 once, as
        all_reduce), returns rmsnorm(residual) * w.  Identical bits on every rank."""
        assert self.can_fuse_norm(x, residual) and w.is_contiguous()
        if out is None:
            out = torch.empty_like(x)
        check(hipk().custom_ar_rmsnorm(out.data_ptr(), residual.data_ptr(), x.data_ptr(),
                                       w.data_ptr(), x.shape[0], x.shape[1], float(eps),
                                       bool(gemma), self.bases, self.rank, self.stage_elems,
                                       stream_ptr(x)), "custom_ar_rmsnorm")
        return out

    def error(self) -> int:
        """Non-zero if a flag wait ever timed out (a peer missed a call)."""
        return hipk().ar_error(self.base)

    def close(self) -> None:
        lib = hipk()
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            lib.ar_ipc_close(p)
        self._opened = []
        if self.base:
            lib.ar_free(self.base)
            self.base = 0
