"""Static-buffer decode step with per-batch-bucket hipGraph capture.

The whole decode step - embedding, 32 x (QKV GEMM, RoPE+KV write, paged MFMA
attention, o_proj, add+norm, gate|up GEMM, act, down, add+norm), LM head and
the sampler, plus the RNG-step increment - is captured once per batch bucket
and replayed with a single ``hipGraphLaunch``.  Per step the host only
uploads three packed staging buffers (int32 / int64 / fp32) and reads back
the sampled token ids.  Steps can be pipelined: the next step's input tokens
are gathered from the previous step's samples on the device, so the engine
enqueues step t+1 before it reads step t's tokens and the host bookkeeping of
step t overlaps the GPU work of step t+1.

Expert-parallel MoE models dispatch with a capacity factor (parallel/
expert_parallel.py::ep_moe_a2a_cap).  The step's EP-group count of dropped
(token, expert) pairs comes back with the sampled tokens; when it is nonzero
:meth:`DecodeRunner.wait` re-runs that step - and every step launched after it,
whose inputs depended on it - eagerly at worst-case capacity before returning,
so the tokens never depend on the capacity.
"""
from __future__ import annotations

import bisect
import os

import numpy as np
import torch

from .. import ops
from ..utils import tracing
from ..models.transformer import DecodeMeta, TransformerLM

# hipGraph batch buckets: the decode M the GEMM tuning table measured (ops/gemm.py)
DEFAULT_BUCKETS = ops.gemm.DECODE_BUCKETS


class DecodeRunner:
    def __init__(self, model: TransformerLM, kv_cache, max_batch: int, max_blocks: int,
                 use_graphs: bool = True, seed: int = 0, buckets=DEFAULT_BUCKETS):
        self.model = model
        self.kv = kv_cache
        self.max_batch = max_batch
        self.max_blocks = max_blocks
        self.seed = seed
        dev = model.device
        self.device = dev
        self.use_graphs = bool(use_graphs and dev.type == "cuda")
        self.buckets = sorted({b for b in buckets if b < max_batch} | {max_batch})
        cfg, sh = model.cfg, model.sh
        B, MB = max_batch, max_blocks
        # ---- device buffers (persistent: graphs capture these addresses)
        n_i32 = 3 * B + B * MB + B
        self.i32 = torch.zeros(n_i32, dtype=torch.int32, device=dev)
        self.ids = self.i32[0:B]
        self.positions = self.i32[B:2 * B]
        self.ctx = self.i32[2 * B:3 * B]
        self.topk = self.i32[3 * B:4 * B]
        self.bt = self.i32[4 * B:4 * B + B * MB].view(B, MB)
        # int64 staging: KV slot per sequence | source row of the input token
        # in the previous step's sampled tokens (-1: take ``ids`` from the host)
        self.i64 = torch.full((2 * B,), -1, dtype=torch.int64, device=dev)
        self.slots = self.i64[0:B]
        self.src = self.i64[B:2 * B]
        self.f32 = torch.zeros(2 * B, dtype=torch.float32, device=dev)
        self.temp = self.f32[0:B]
        self.topp = self.f32[B:2 * B]
        self.step_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        self.out = torch.zeros(B, dtype=torch.int32, device=dev)
        self.attn_out = torch.zeros((B, sh.hq, cfg.head_dim), dtype=model.dtype, device=dev)
        # ---- pinned host staging, double-buffered: step t+1 is staged while
        # step t's copies may still be pending (pipelined decode)
        pin = dev.type == "cuda"
        self.h_i32 = [torch.zeros(n_i32, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.h_i64 = [torch.full((2 * B,), -1, dtype=torch.int64, pin_memory=pin) for _ in range(2)]
        self.h_f32 = [torch.zeros(2 * B, dtype=torch.float32, pin_memory=pin) for _ in range(2)]
        self.h_out = [torch.zeros(B, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.events = [torch.cuda.Event() if pin else None for _ in range(2)]
        self._k = 0
        self.n_i32 = n_i32
        self._metas = {}
        self._graphs = {}
        self._pool = None
        # DRTC_TIME_DECODE=1: GPU time of every replay (hipEvents), for host-
        # overhead accounting (decode wall time - GPU time)
        self.time_gpu = os.environ.get("DRTC_TIME_DECODE") == "1"
        self.gpu_ms: list[float] = []
        self._timing: dict[int, tuple] = {}  # staging set -> (start, end) events
        # EP capacity-overflow redo: the input ids each step actually used and
        # the dropped-pair count, read back with the tokens; launched steps
        # not yet waited for, in launch order
        self.ep = getattr(model, "ep_overflow", None) is not None
        self.ids_used = torch.zeros(B, dtype=torch.int32, device=dev)
        self.h_in = [torch.zeros(B, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self.h_ovf = [torch.zeros(1, dtype=torch.int32, pin_memory=pin) for _ in range(2)]
        self._pending: list[dict] = []
        self._step_no = 0
        self.redo_steps = 0
        # host mirror of ``step_ctr`` (the sampler's RNG stream position): every executed
        # _forward advances it by one - eager steps, capture warm-ups and graph replays
        # alike (a capture records the add without running it) - so a redone step can be
        # given exactly the counter value its first run sampled with
        self._ctr = 0

    # ------------------------------------------------------------------
    def bucket(self, n: int) -> int:
        i = bisect.bisect_left(self.buckets, n)
        if i >= len(self.buckets):
            raise ValueError(f"batch {n} exceeds max_batch {self.max_batch}")
        return self.buckets[i]

    def _meta(self, Bb: int) -> DecodeMeta:
        m = self._metas.get(Bb)
        if m is None:
            sh = self.model.sh
            bpp, max_parts = ops.decode_partitioning(Bb, sh.hkv, self.max_blocks,
                                                     D=self.model.cfg.head_dim)
            ws = ops.DecodeWorkspace(Bb, sh.hq, self.model.cfg.head_dim, max_parts, self.device)
            m = DecodeMeta(positions=self.positions[:Bb], slots=self.slots[:Bb],
                           block_tables=self.bt[:Bb], context_lens=self.ctx[:Bb],
                           blocks_per_part=bpp, workspace=ws)
            self._metas[Bb] = m
        return m

    def _forward(self, Bb: int) -> None:
        meta = self._meta(Bb)
        # input tokens: the previous step's samples still on the device
        # (pipelined steps, src >= 0) or host-provided ids (src = -1)
        src = self.src[:Bb]
        ids = torch.where(src >= 0, self.out[:Bb].index_select(0, src.clamp(min=0)),
                          self.ids[:Bb])
        if self.ep:
            self.ids_used[:Bb].copy_(ids)
        logits = self.model.forward_decode(ids, meta, self.kv, self.attn_out[:Bb])
        ops.sample(logits, self.temp[:Bb], self.topk[:Bb], self.topp[:Bb], seed=self.seed,
                   step=self.step_ctr, out=self.out[:Bb])
        self.step_ctr.add_(1)
        if not (self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            self._ctr += 1

    def capture(self, Bb: int) -> None:
        if not self.use_graphs or Bb in self._graphs:
            return
        # warm up on a side stream (lazy hipBLASLt / allocator init), then capture
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            self._forward(Bb)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self._pool):
            self._forward(Bb)
        torch.cuda.synchronize(self.device)
        self._graphs[Bb] = g

    def capture_all(self, up_to: int | None = None) -> None:
        for Bb in sorted(self.buckets, reverse=True):
            if up_to is None or Bb <= self.bucket(min(up_to, self.max_batch)):
                self.capture(Bb)

    # ------------------------------------------------------------------
    def launch(self, n: int, ids: np.ndarray | None, positions: np.ndarray, ctx: np.ndarray,
               slots: np.ndarray, block_rows: np.ndarray, temp: np.ndarray, topk: np.ndarray,
               topp: np.ndarray) -> tuple[int, int]:
        """Enqueue one decode step for ``n`` sequences (arrays of length n,
        block_rows [n, max_blocks]) without waiting for it.  ``ids=None``
        takes every input token from the previous step's samples on the device
        (same slot order: a pipelined step).  Returns a handle for
        :meth:`wait`."""
        Bb = self.bucket(n)
        B, MB = self.max_batch, self.max_blocks
        k = self._k
        self._k ^= 1
        hi = self.h_i32[k].numpy()
        if ids is not None:
            hi[0:n] = ids
        hi[n:Bb] = 0
        hi[B:B + n] = positions
        hi[B + n:B + Bb] = 0
        hi[2 * B:2 * B + n] = ctx
        hi[2 * B + n:2 * B + Bb] = 0
        hi[3 * B:3 * B + n] = topk
        hi[3 * B + n:3 * B + Bb] = 0
        btv = hi[4 * B:4 * B + B * MB].reshape(B, MB)
        btv[:n] = block_rows
        btv[n:Bb] = 0
        hl = self.h_i64[k].numpy()
        hl[:n] = slots
        hl[n:Bb] = -1
        hl[B:B + n] = -1 if ids is not None else np.arange(n)
        hl[B + n:B + Bb] = -1
        hf = self.h_f32[k].numpy()
        hf[:n] = temp
        hf[n:Bb] = 0.0
        hf[B:B + n] = topp
        hf[B + n:B + Bb] = 1.0
        nb = self.device.type == "cuda"
        self.i32.copy_(self.h_i32[k], non_blocking=nb)
        self.i64.copy_(self.h_i64[k], non_blocking=nb)
        self.f32.copy_(self.h_f32[k], non_blocking=nb)
        g = self._graphs.get(Bb)
        if g is None and self.use_graphs:
            self.capture(Bb)
            g = self._graphs[Bb]
        timing = nb and self.time_gpu
        if timing:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        ctr = self._ctr  # the RNG counter this step samples with
        with tracing.span("decode.graph_replay" if g is not None else "decode.eager", bucket=Bb):
            if g is not None:
                g.replay()
                self._ctr += 1
            else:
                self._forward(Bb)
        if timing:
            ev1.record()
            self._timing[k] = (ev0, ev1)
        self._readback(n, k)
        self._pending.append({"n": n, "k": k, "Bb": Bb, "step": self._step_no, "ctr": ctr})
        del self._pending[:-2]  # two staging sets: at most two steps in flight
        self._step_no += 1
        return n, k

    def _readback(self, n: int, k: int) -> None:
        nb = self.device.type == "cuda"
        self.h_out[k][:n].copy_(self.out[:n], non_blocking=nb)
        if self.ep:
            self.h_in[k][:n].copy_(self.ids_used[:n], non_blocking=nb)
            self.h_ovf[k].copy_(self.model.ep_overflow.count, non_blocking=nb)
        if nb:
            self.events[k].record()

    def _redo_from(self, i: int) -> None:
        """Re-run pending step i (its capacity dispatch dropped pairs) and
        every later pending step, eagerly at worst-case EP capacity.  Step i
        takes the input ids it used the first time; later steps take theirs
        from the re-computed samples on the device, as when pipelined."""
        from ..parallel.expert_parallel import worst_case_capacity

        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        B = self.max_batch
        saved = self._ctr
        for j, p in enumerate(self._pending[i:]):
            n, k = p["n"], p["k"]
            if j == 0:
                self.h_i32[k].numpy()[0:n] = self.h_in[k].numpy()[:n]
                self.h_i64[k].numpy()[B:B + n] = -1
            self.i32.copy_(self.h_i32[k])
            self.i64.copy_(self.h_i64[k])
            self.f32.copy_(self.h_f32[k])
            # the counter value of the step's first run: the redo samples the same RNG
            # stream, so the tokens never depend on the capacity
            self.step_ctr.fill_(p["ctr"])
            with worst_case_capacity(), tracing.span("decode.ep_redo", bucket=p["Bb"]):
                self._forward(p["Bb"])
            self._readback(n, k)
            self.redo_steps += 1
        self.step_ctr.fill_(saved)
        self._ctr = saved
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)

    def wait(self, handle: tuple[int, int]) -> np.ndarray:
        """Sampled token ids of a launched step (blocks until it is done)."""
        n, k = handle
        if self.events[k] is not None:
            self.events[k].synchronize()
        i = next(j for j, p in enumerate(self._pending) if p["k"] == k)
        if self.ep and int(self.h_ovf[k][0]) > 0:
            self._redo_from(i)
        del self._pending[i]
        ev = self._timing.pop(k, None)
        if ev is not None:
            self.gpu_ms.append(ev[0].elapsed_time(ev[1]))
        return self.h_out[k][:n].numpy().copy()
