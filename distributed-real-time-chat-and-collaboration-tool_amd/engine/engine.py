"""Continuous-batching LLM serving engine (one engine per GPU / TP group).

Scheduling (one iteration = one ``step()``):
  * prefill-first: while requests wait and the batch has free slots and KV
    blocks, admit as many as fit in ``max_prefill_tokens`` and run ONE packed
    varlen prefill for all of them (MFMA flash attention, KV written in the
    fused RoPE kernel), sampling each request's first token;
  * otherwise one decode step for every running request through the
    hipGraph of its batch bucket (engine/decode_runner.py);
  * on KV exhaustion the most recently admitted request is preempted
    (blocks freed, re-queued at the front for recomputation).

Replaces the reference's hosted model call
(``genai.GenerativeModel('gemini-2.5-flash').generate_content``,
llm_server/llm_server.py:33,167,231,287,403): the four LLM features now
generate on the node's own GPU, batched across concurrent RPCs.

Running requests occupy dense "slots" 0..n-1 whose block-table rows live in
a persistent numpy array, so building a decode step's metadata is a handful
of vectorised numpy ops (no per-request Python loops on the hot path except
token bookkeeping).
"""
from __future__ import annotations

import atexit
import collections
import itertools
import math
import os
import threading
import time
import weakref

import numpy as np
import torch

from .. import ops
from ..utils import tracing
from ..utils.metrics import METRICS
from ..models.transformer import DecodeMeta, PrefillMeta, TransformerLM
from .decode_runner import DEFAULT_BUCKETS, DecodeRunner
from .kv_cache import PagedKVCache
from .request import Request, RequestState, SamplingParams

BS = ops.KV_BLOCK


def _pad_tokens(T: int) -> int:
    """Prefill token-count bucket (< 256 padded rows above 256 tokens)."""
    if T <= 256:
        return -(-T // 32) * 32
    return -(-T // 256) * 256



def freeze_gc() -> None:
    """Move every object alive now (weights, captured graphs, caches, prepared inputs)
    into the cyclic GC's permanent generation, once per serving process after warm-up:
    full collections triggered in the request loop then walk only request-lifetime
    objects instead of the whole long-lived heap.  ``DRTC_GC_FREEZE=0`` disables it."""
    import gc

    if os.environ.get("DRTC_GC_FREEZE", "1") != "0":
        gc.collect()
        gc.freeze()

class LLMEngine:
    def __init__(self, model: TransformerLM, max_batch: int = 256, max_model_len: int = 4096,
                 max_prefill_tokens: int = 16384, num_blocks: int | None = None,
                 kv_fraction: float = 0.85, use_graphs: bool = True, seed: int = 0,
                 buckets=DEFAULT_BUCKETS, hbm_budget: float | None = None):
        self.model = model
        cfg = model.cfg
        self.cfg = cfg
        self.device = model.device
        self.max_batch = max_batch
        self.max_model_len = min(max_model_len, cfg.max_position)
        self.max_prefill_tokens = max_prefill_tokens
        # prefill launch granularity: GEMMs stay at full efficiency from ~16k
        # rows; measured on the headline batch (one MI355X), 16k / 32k / 64k
        # chunks: equal tok/s, p50 TTFT 0.85 / 1.02 / 1.37 s.  Per model
        # (ModelConfig.prefill_chunk): Mixtral 32k (the MoE layers' rows per expert),
        # Llama-3-70B 36k (one step per ask wave), profiles/r6t
        self.prefill_chunk_tokens = int(os.environ.get(
            "DRTC_PREFILL_CHUNK", str(getattr(cfg, "prefill_chunk", 16384))))
        self.max_blocks = math.ceil(self.max_model_len / BS)
        # hbm_budget: the fraction of the GPU's HBM this engine may hold (engine groups that
        # share a GPU, llm.server --serve ...:mem=F); every TP / EP rank gets the same
        # fraction and the ranks agree on the smallest resulting block count
        self.hbm_budget = hbm_budget
        if num_blocks is None:
            num_blocks = PagedKVCache.auto_num_blocks(
                cfg, model.sh.hkv, self.device, kv_fraction, hbm_budget=hbm_budget,
                weight_bytes=model.weight_bytes() if hbm_budget is not None else None,
                min_blocks=self.max_blocks)
        # lockstep (SPMD) TP/EP ranks must schedule identically: every rank
        # sizes its cache from the same (smallest) block count
        num_blocks = model.pc.agree_min(num_blocks)
        self.kv = PagedKVCache(cfg, model.sh.hkv, num_blocks, self.device, model.dtype)
        self.alloc = self.kv.allocator
        self.runner = DecodeRunner(model, self.kv, max_batch, self.max_blocks,
                                   use_graphs=use_graphs, seed=seed, buckets=buckets)
        self.seed = seed
        self._prefill_step = 0
        # EP dropped-pair count and sampler step per prefill launch
        self._h_ovf: dict[int, tuple[torch.Tensor, int]] = {}
        # slot state
        self.bt = np.zeros((max_batch, self.max_blocks), dtype=np.int32)
        self.ctx = np.zeros(max_batch, dtype=np.int32)        # tokens in the KV cache
        self.last = np.zeros(max_batch, dtype=np.int32)       # last sampled token
        self.temp = np.zeros(max_batch, dtype=np.float32)
        self.topk = np.zeros(max_batch, dtype=np.int32)
        self.topp = np.ones(max_batch, dtype=np.float32)
        # per-slot finish bookkeeping, so a decode step checks 1024 sequences
        # with a few numpy ops instead of a Python call per request
        self.gen = np.zeros(max_batch, dtype=np.int32)        # tokens generated so far
        self.max_new = np.zeros(max_batch, dtype=np.int32)
        self.eos_stop = np.zeros(max_batch, dtype=bool)       # stop on EOS (not ignore_eos)
        self.nblk = np.zeros(max_batch, dtype=np.int32)       # cache blocks held
        self.stop_ids: dict[int, tuple] = {}                  # slot -> custom stop ids
        self.running: list[Request] = []
        # pipelined decode: the launched-but-unread step, and requests that
        # finished (EOS) while a later step holding their slot was in flight
        self._inflight: dict | None = None
        self._zombies: list[Request] = []
        self.pipeline = os.environ.get("DRTC_PIPELINE_DECODE", "1") != "0"
        self.waiting: collections.deque[Request] = collections.deque()
        self.lock = threading.Lock()
        self.stats = collections.Counter()
        # admission watermark + anti-thrash latch: after a preemption no new
        # request is admitted until some running request finishes
        self.watermark = max(1, self.kv.num_blocks // 100)
        self._pressure = False
        # mixed steps: while requests are running, new prompts are prefilled
        # INSIDE decode steps, at most ``mixed_tokens`` prompt tokens per step,
        # so a new wave never stalls running decodes for a whole prefill
        # (DRTC_MIXED=0: strict prefill-first)
        self.mixed = os.environ.get("DRTC_MIXED", "1") != "0"
        self._waiting_tokens = 0  # prompt (+ recompute) tokens queued in self.waiting
        self._aborts: list[Request] = []  # abort() requests, applied at the next step
        self.mixed_tokens = int(os.environ.get("DRTC_MIXED_TOKENS", "2048"))
        # slot-bound admission groups: when the queue is longer than the free
        # batch slots, wait until at least this many slots are free and admit
        # them in one step (one larger, more GEMM-efficient prefill) instead of
        # trickling the ~max_batch/48 slots freed per step into every step;
        # the steps in between are pure, graph-replayed, pipelined decodes
        self.admit_group = int(os.environ.get("DRTC_ADMIT_GROUP", str(max(1, max_batch // 16))))
        # arrival gathering for mixed steps (off unless admit_min_tokens > 0): while requests
        # are decoding and new prompts are still arriving (last one < admit_gap_s ago), run
        # pure decode steps until the queue holds admit_min_tokens prompt tokens, at most
        # admit_max_delay_s after the oldest queued arrival - one GEMM-efficient mixed step
        # per chunk instead of a small one per step (closed-loop clients return in bursts)
        self.admit_min_tokens = int(os.environ.get("DRTC_ADMIT_MIN_TOKENS", "0"))
        self.admit_gap_s = float(os.environ.get("DRTC_ADMIT_GAP_MS", "3")) / 1000.0
        self.admit_max_delay_s = float(os.environ.get("DRTC_ADMIT_MAX_MS", "100")) / 1000.0
        self._last_arrival = 0.0
        self._steps = 0  # scheduler steps (split-K fault polls every HEALTH_EVERY)
        self._fault_watch = None
        if self.device.type == "cuda":
            from ..ops import gemm as _gemm

            self._fault_watch = _gemm.SplitKWatch(self.device)
        self.closed = False

    # ------------------------------------------------------------ API
    def add_request(self, req: Request) -> Request:
        if self.closed:
            raise RuntimeError("engine is shut down")
        n = len(req.prompt_ids)
        if n == 0:
            raise ValueError("empty prompt")
        if n >= self.max_model_len:
            raise ValueError(f"prompt of {n} tokens exceeds max_model_len {self.max_model_len}")
        if n > self.max_prefill_tokens:
            raise ValueError("prompt exceeds max_prefill_tokens")
        with self.lock:
            req.state = RequestState.WAITING
            self.waiting.append(req)
            self._waiting_tokens += n
            self._last_arrival = time.perf_counter()
        return req

    def _admit_ready(self) -> bool:
        """Whether a mixed step may admit now (see ``admit_min_tokens``)."""
        if self.admit_min_tokens <= 0 or self._waiting_tokens >= self.admit_min_tokens:
            return True
        if len(self.waiting) >= self.max_batch - len(self.running):
            return True  # slot-bound: the queue fills every free slot already
        now = time.perf_counter()
        if now - self._last_arrival >= self.admit_gap_s:
            return True  # arrivals paused: nothing more to gather
        oldest = self.waiting[0].arrival_time if self.waiting else now
        return now - oldest >= self.admit_max_delay_s

    def has_work(self) -> bool:
        return bool(self.running or self.waiting or self._inflight or self._aborts)

    def abort(self, req: Request) -> None:
        """Cancel a request (its caller gave up, e.g. an RPC deadline): it is
        dropped from the queue or finished with reason "abort" at the next
        step boundary, freeing its batch slot and KV blocks.  Thread-safe;
        a no-op for a request that already finished."""
        with self.lock:
            if req.state != RequestState.FINISHED:
                self._aborts.append(req)

    def _apply_aborts(self) -> list[Request]:
        with self.lock:
            aborts, self._aborts = self._aborts, []
            done = []
            for r in aborts:
                if r.state == RequestState.WAITING:
                    try:
                        self.waiting.remove(r)
                    except ValueError:
                        continue
                    self._waiting_tokens -= r.num_tokens
                    r.mark_finished("abort")
                    done.append(r)
        live = [r for r in aborts if r.state == RequestState.RUNNING]
        if live:
            # a launched step still holds their slots: read it first
            if self._inflight is not None:
                done += self._process_inflight()
            rel = sorted((r for r in live if r.state == RequestState.RUNNING and r.slot >= 0),
                         key=lambda r: -r.slot)
            with self.lock:
                for r in rel:
                    self._release_slot(r)
                    r.mark_finished("abort")
                    done.append(r)
            if rel:
                self._pressure = False
        self.stats["aborted"] += len([r for r in done if r.finish_reason == "abort"])
        return done

    def warmup(self, capture: bool = True, up_to: int | None = None) -> None:
        """Capture decode graphs up front (zeroed staging: no cache reads/writes), then check
        the split-K fault word of the GEMM workspaces (the capture's eager warm-up ran every
        split-K form the graphs hold)."""
        if capture and self.runner.use_graphs:
            self.runner.capture_all(up_to)
        self.check_health()

    # steps between two split-K fault polls while serving (ops.gemm.SplitKWatch: an async copy
    # of the fault words per poll, no device sync; 0 disables)
    HEALTH_EVERY = int(os.environ.get("DRTC_HEALTH_EVERY", "1"))

    def check_health(self) -> None:
        """Raise ops.gemm.SplitKFault if a split-K GEMM combine on this engine's device timed
        out since the last check (its output was wrong; the workspace counters are reset)."""
        if self.device.type == "cuda":
            from ..ops import gemm as _gemm

            _gemm.check_splitk_fault(self.device)

    def shutdown(self, reason: str = "error: shutdown") -> list[Request]:
        """Stop serving, in order: read the in-flight (pipelined) decode step, finish every
        queued and running request with ``reason`` (their waiters return at once), release
        their batch slots and KV blocks, and wait until the device has finished every kernel
        this engine issued.  Call it from the thread that drives the engine, or after that
        thread has stopped (EngineLoop.stop).  Returns the requests it finished."""
        if self.closed:
            return []
        self.closed = True
        if self._inflight is not None:
            try:
                self._process_inflight()
            except Exception:  # a failing device: still fail the requests below
                self._inflight = None
        with self.lock:
            # (finished "zombies" still hold their slots: they are in ``running`` too)
            pending = list(self.waiting) + list(self.running)
            self.waiting.clear()
            self._waiting_tokens = 0
            self._aborts = []
            for r in sorted(self.running, key=lambda r: -r.slot):
                self._release_slot(r)
            self._zombies = []
        done = []
        for r in pending:
            if r.state != RequestState.FINISHED:
                r.mark_finished(reason)
                done.append(r)
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return done

    def generate(self, prompts: list[list[int]], params: SamplingParams | list) -> list[Request]:
        if isinstance(params, SamplingParams):
            params = [params] * len(prompts)
        reqs = [self.add_request(Request(list(p), prm)) for p, prm in zip(prompts, params)]
        while any(r.state != RequestState.FINISHED for r in reqs):
            self.step()
        return reqs

    def step(self) -> list[Request]:
        """One scheduler iteration. Returns requests finished in it.  The host wall time of
        each iteration is added to ``stats[<kind>_us]`` (kind: decode / mixed / prefill /
        drain / abort): with one decode step in flight that is the step's GPU time, and it
        shows what the synchronous mixed and prefill steps cost a served engine."""
        t0 = time.perf_counter()
        done, kind = self._step()
        if kind:
            self.stats[kind + "_us"] += int(1e6 * (time.perf_counter() - t0))
            self._record(done)
        return done

    def _step(self) -> tuple[list[Request], str | None]:
        if self._aborts:
            return self._apply_aborts(), "abort"
        busy = self.running or self._inflight is not None
        if self.mixed and busy and self._could_admit() and not self._admit_ready():
            # gathering arrivals for one chunk-sized mixed step: decode meanwhile
            with tracing.span("engine.decode", batch=len(self.running)):
                return self._run_decode(), "decode"
        if self.mixed and busy and self._could_admit():
            done = self._process_inflight() if self._inflight is not None else []
            with self.lock:
                self._ensure_blocks()
                batch = self._admit(self._mixed_budget()) if self.running else self._admit()
            kind = "drain"
            if batch and self.running:
                kind = "mixed"
                with tracing.span("engine.mixed", seqs=len(batch), batch=len(self.running)):
                    done += self._run_mixed(batch)
            elif batch:
                kind = "prefill"
                with tracing.span("engine.prefill", seqs=len(batch)):
                    done += self._run_prefill(batch)
            elif self.running:
                kind = "decode"
                with tracing.span("engine.decode", batch=len(self.running)):
                    done += self._run_decode()
            return done, kind
        if self._inflight is not None and self._could_admit():
            # a prefill changes the slot layout: read the in-flight step first
            return self._process_inflight(), "drain"
        with self.lock:
            batch = self._admit() if (not self.running or self._could_admit()) else []
        if batch:
            with tracing.span("engine.prefill", seqs=len(batch)):
                return self._run_prefill(batch), "prefill"
        if self.running or self._inflight is not None:
            with tracing.span("engine.decode", batch=len(self.running)):
                return self._run_decode(), "decode"
        return [], None

    def _record(self, done: list[Request]) -> None:
        """Serving metrics: TTFT / TPOT / end-to-end latency per finished
        request, KV-cache occupancy and queue depths per step."""
        M = METRICS
        self._steps += 1
        if (self._fault_watch is not None and self.HEALTH_EVERY > 0
                and self._steps % self.HEALTH_EVERY == 0):
            self._fault_watch.poll()
        if done:
            M.observe_many("engine.ttft_s", [r.ttft for r in done])
            M.observe_many("engine.e2e_s", [r.finish_time - r.arrival_time for r in done])
            M.observe_many("engine.tpot_s", [(r.finish_time - r.first_token_time)
                                             / (len(r.output_ids) - 1)
                                             for r in done if len(r.output_ids) > 1])
            M.inc("engine.generated_tokens", sum(len(r.output_ids) for r in done))
            M.inc("engine.finished", len(done))
        used, free = self.alloc.num_used, self.alloc.num_free
        M.set_gauge("engine.kv_used_frac", used / max(1, used + free))
        M.set_gauge("engine.running", len(self.running))
        M.set_gauge("engine.waiting", len(self.waiting))

    # ------------------------------------------------------------ admission
    def _mixed_budget(self) -> int:
        """Prompt tokens a mixed step may add: ``mixed_tokens`` (keeps the
        decode rows' TPOT near a pure decode step) while the queue is short,
        growing to a quarter of the waiting prompt tokens (at most one prefill
        chunk) under a backlog, so sustained overload is drained in
        efficient large chunks - with the decode rows still riding along -
        instead of throttling admission (closed-loop service load: 309 req/s
        with the fixed budget vs 370 prefill-first)."""
        if len(self.waiting) > self.max_batch - len(self.running):
            # slot-bound: a whole admission group (_could_admit) in one step
            return self.prefill_chunk_tokens
        if self.admit_min_tokens > 0:  # gathered arrivals: admit them as one chunk
            return max(self.mixed_tokens, min(self.prefill_chunk_tokens, self._waiting_tokens))
        return max(self.mixed_tokens, min(self.prefill_chunk_tokens, self._waiting_tokens // 4))

    def _admit(self, budget: int | None = None) -> list[Request]:
        budget = self.max_prefill_tokens if budget is None else budget
        batch, tokens = [], 0
        if self._pressure and self.running:
            return batch
        self._pressure = False
        while self.waiting and len(self.running) + len(batch) < self.max_batch:
            r = self.waiting[0]
            ids = r.all_ids  # recomputation after preemption includes outputs
            n = len(ids)
            if batch and tokens + n > budget:
                break
            need = math.ceil((n + 1) / BS)
            busy = bool(self.running or batch)
            if not self.alloc.can_allocate(need + (self.watermark if busy else 0)):
                if not busy and need > self.alloc.num_blocks - 1:
                    self.waiting.popleft()
                    self._waiting_tokens -= n
                    r.mark_finished("error: request exceeds KV-cache capacity")
                    continue
                break
            self.waiting.popleft()
            self._waiting_tokens -= n
            r.blocks = list(self.alloc.allocate(need))
            batch.append(r)
            tokens += n
        return batch

    def _assign_slot(self, r: Request) -> int:
        s = len(self.running)
        self.running.append(r)
        r.slot = s
        r.state = RequestState.RUNNING
        self.bt[s, :] = 0
        self.bt[s, :len(r.blocks)] = r.blocks
        self.temp[s] = r.params.temperature
        self.topk[s] = r.params.top_k
        self.topp[s] = r.params.top_p
        self.gen[s] = len(r.output_ids)
        self.max_new[s] = r.params.max_new_tokens
        self.eos_stop[s] = not r.params.ignore_eos
        self.nblk[s] = len(r.blocks)
        if r.params.stop_token_ids and not r.params.ignore_eos:
            self.stop_ids[s] = tuple(r.params.stop_token_ids)
        return s

    def _release_slot(self, r: Request) -> None:
        s = r.slot
        last = len(self.running) - 1
        if s != last:
            m = self.running[last]
            self.running[s] = m
            m.slot = s
            for arr in (self.bt, self.ctx, self.last, self.temp, self.topk, self.topp, self.gen,
                        self.max_new, self.eos_stop, self.nblk):
                arr[s] = arr[last]
            moved = self.stop_ids.pop(last, None)
            if moved is not None:
                self.stop_ids[s] = moved
            else:
                self.stop_ids.pop(s, None)
        else:
            self.stop_ids.pop(s, None)
        self.running.pop()
        r.slot = -1
        if r.blocks:
            self.alloc.free(r.blocks)
            r.blocks = []

    def _finish_check(self, r: Request, tok: int) -> str:
        p = r.params
        if not p.ignore_eos and (tok == self.cfg.eos_token_id or tok in p.stop_token_ids):
            return "stop"
        if len(r.output_ids) >= p.max_new_tokens:
            return "length"
        if r.num_tokens >= self.max_model_len:
            return "length"
        return ""

    # ------------------------------------------------------------ prefill
    def _run_prefill(self, batch: list[Request]) -> list[Request]:
        """Packed varlen prefill of ``batch``, split into chunks of about
        ``prefill_chunk_tokens`` tokens.  Each chunk's host metadata goes
        through pinned staging and every copy is asynchronous, so the host
        prepares chunk i+1 while the GPU runs chunk i (only the first chunk's
        preparation is on the critical path); the sampled first tokens come
        back through pinned buffers and are read after the last launch."""
        # greedy, not balanced: a chunk of 16,384 tokens fills whole waves of workgroups
        # on 256 CUs in every projection GEMM (64 row tiles x 16 / 24 / 112 column tiles
        # of 256), while "balanced" 10 x ~15.2k chunks measured 5.5 % slower end to end
        # (profiles/r2o_decode_gemm_128tile.md, wave quantization)
        limit = self.prefill_chunk_tokens
        chunks, cur, tok = [], [], 0
        for r in batch:
            n = r.num_tokens
            if cur and tok + n > limit:
                chunks.append(cur)
                cur, tok = [], 0
            cur.append(r)
            tok += n
        chunks.append(cur)
        launched = [self._launch_prefill(c) for c in chunks]
        finished = []
        for reqs, lens, h_tok, ev in launched:
            if ev is not None:
                ev.synchronize()
            h_tok = self._ep_redo_prefill(reqs, 0, h_tok)
            finished += self._finish_prefill(reqs, lens, h_tok.numpy())
        return finished

    def _ep_redo_prefill(self, batch: list[Request], n_dec: int, h_tok):
        """Capacity-factor EP dispatch (parallel/expert_parallel.py): when the
        chunk's forward dropped (token, expert) pairs on any EP rank, run it
        again at worst-case capacity (same KV slots, same requests; chunks are
        independent, so the chunks launched after it stay valid)."""
        ent = self._h_ovf.pop(id(h_tok), None)
        if ent is None or int(ent[0][0]) == 0:
            return h_tok
        from ..parallel.expert_parallel import worst_case_capacity

        # the step counter this chunk's first run sampled with (chunks launched after it
        # advanced the counter already): the redo draws from the same stream
        with worst_case_capacity():
            _, _, h_tok, ev = self._launch_prefill(batch, n_dec=n_dec, step=ent[1])
        if ev is not None:
            ev.synchronize()
        self._h_ovf.pop(id(h_tok), None)
        self.stats["prefill_steps"] -= 1
        self.stats["prefill_tokens"] -= int(sum(r.num_tokens for r in batch))
        self.stats["ep_redo_steps"] = self.stats.get("ep_redo_steps", 0) + 1
        return h_tok

    def _launch_prefill(self, batch: list[Request], n_dec: int = 0, step: int | None = None):
        """Enqueue one packed prefill of ``batch``.  ``n_dec > 0`` makes it a
        mixed step: one decode row per running slot 0..n_dec-1 (padded to the
        decode bucket) rides in the same forward pass - same GEMM launches,
        paged attention for those rows - and is sampled with the prefill rows.  ``step``:
        the sampler's step counter for a redo (default: the next one)."""
        dev = self.device
        cuda = dev.type == "cuda"
        # host metadata, vectorised over the batch (a 1024-prompt prefill is
        # ~150k tokens: per-request numpy calls would idle the GPU for ~50 ms)
        seqs = [r.all_ids if r.output_ids else r.prompt_ids for r in batch]
        nseq = len(batch)
        lens_a = np.fromiter((len(x) for x in seqs), dtype=np.int64, count=nseq)
        lens = lens_a.tolist()
        cu_a = np.zeros(nseq + 1, dtype=np.int64)
        np.cumsum(lens_a, out=cu_a[1:])
        cu = cu_a.tolist()
        T = cu[-1]
        # pad the token count to a coarse bucket: hipBLASLt picks (and caches)
        # its kernels per GEMM shape, so stable shapes avoid re-heuristics and
        # first-use code-object loads on every prefill.  Padded rows carry
        # position 0 and slot -1 (no cache write) and are never attended.
        # mixed step: the prefill part is padded so that prefill + decode rows
        # land on a token bucket (stable GEMM shapes)
        Bb = self.runner.bucket(n_dec) if n_dec else 0
        Tp = _pad_tokens(T + Bb) - Bb
        ids = np.zeros(Tp, dtype=np.int32)
        ids[:T] = np.fromiter(itertools.chain.from_iterable(seqs), dtype=np.int32, count=T)
        seq_of = np.repeat(np.arange(nseq), lens_a)
        p_tok = np.arange(T, dtype=np.int64) - np.repeat(cu_a[:-1], lens_a)
        pos = np.zeros(Tp, dtype=np.int32)
        pos[:T] = p_tok
        nblk = -(-lens_a // BS)
        blk_tab = np.zeros((nseq, int(nblk.max())), dtype=np.int64)
        for i, r in enumerate(batch):
            blk_tab[i, :nblk[i]] = r.blocks[:nblk[i]]
        slots = np.full(Tp, -1, dtype=np.int64)
        slots[:T] = blk_tab[seq_of, p_tok // BS] * BS + p_tok % BS
        # one V-write segment per (sequence, cache block)
        s_seq = np.repeat(np.arange(nseq), nblk)
        s_j = np.arange(int(nblk.sum()), dtype=np.int64) - np.repeat(np.cumsum(nblk) - nblk, nblk)
        seg_tok = (cu_a[s_seq] + BS * s_j).astype(np.int32)
        seg_len = np.minimum(BS, lens_a[s_seq] - BS * s_j).astype(np.int32)
        seg_blk = blk_tab[s_seq, s_j].astype(np.int32)
        last_idx = np.asarray(cu[1:], dtype=np.int64) - 1
        ts, tq = ops.prefill_tiles(cu)
        if step is None:
            self._prefill_step += 1
            step = self._prefill_step
        params = np.array([(r.params.temperature, r.params.top_p, r.params.top_k) for r in batch],
                          dtype=np.float64).reshape(nseq, 3)
        dec_i32 = []
        if n_dec:
            # decode rows: exactly the staging of a decode step of bucket Bb
            # (padding rows: context 0, no cache write, greedy)
            n, MB = n_dec, self.max_blocks
            d_pos = self.ctx[:n]
            d_ids = np.zeros(Bb, np.int32); d_ids[:n] = self.last[:n]
            d_p = np.zeros(Bb, np.int32); d_p[:n] = d_pos
            d_slot = np.full(Bb, -1, np.int64)
            d_slot[:n] = self.bt[np.arange(n), d_pos // BS].astype(np.int64) * BS + d_pos % BS
            d_ctx = np.zeros(Bb, np.int32); d_ctx[:n] = d_pos + 1
            d_bt = np.zeros((Bb, MB), np.int32); d_bt[:n] = self.bt[:n]
            d_par = np.zeros((Bb, 3)); d_par[:, 1] = 1.0
            d_par[:n, 0], d_par[:n, 1], d_par[:n, 2] = self.temp[:n], self.topp[:n], self.topk[:n]
            ids = np.concatenate([ids, d_ids])
            pos = np.concatenate([pos, d_p])
            slots = np.concatenate([slots, d_slot])
            last_idx = np.concatenate([last_idx, Tp + np.arange(Bb, dtype=np.int64)])
            params = np.concatenate([params, d_par])
            dec_i32 = [d_ctx, d_bt.reshape(-1)]
            # the V of decode rows goes through rope_kv_'s own write
            seg_tok = seg_len = seg_blk = np.zeros(0, np.int32)
        R, ns_all = Tp + Bb, nseq + Bb
        h_i32 = torch.from_numpy(np.concatenate([
            ids, pos, np.asarray(cu, np.int32), np.asarray(ts, np.int32),
            np.asarray(tq, np.int32), seg_tok, seg_len, seg_blk,
            params[:, 2].astype(np.int32)] + dec_i32))
        h_i64 = torch.from_numpy(np.concatenate([
            slots, last_idx, np.array([step + (1 << 40)], dtype=np.int64)]))
        h_f32 = torch.from_numpy(params[:, :2].T.astype(np.float32).reshape(-1))
        if cuda:  # pinned staging: the copies stay asynchronous to the host
            h_i32, h_i64, h_f32 = h_i32.pin_memory(), h_i64.pin_memory(), h_f32.pin_memory()
        t_i32 = h_i32.to(dev, non_blocking=True)
        t_i64 = h_i64.to(dev, non_blocking=True)
        t_f32 = h_f32.to(dev, non_blocking=True)
        nt, ns = len(ts), len(seg_tok)
        o = 0
        d_ids = t_i32[o:o + R]; o += R
        d_pos = t_i32[o:o + R]; o += R
        d_cu = t_i32[o:o + nseq + 1]; o += nseq + 1
        d_ts = t_i32[o:o + nt]; o += nt
        d_tq = t_i32[o:o + nt]; o += nt
        d_segs = (t_i32[o:o + ns], t_i32[o + ns:o + 2 * ns], t_i32[o + 2 * ns:o + 3 * ns])
        o += 3 * ns
        topk = t_i32[o:o + ns_all]; o += ns_all
        dmeta = None
        if n_dec:
            rm = self.runner._meta(Bb)  # decode partitioning + workspace of bucket Bb
            ctx_d = t_i32[o:o + Bb]; o += Bb
            bt_d = t_i32[o:o + Bb * self.max_blocks].view(Bb, self.max_blocks)
            dmeta = DecodeMeta(positions=d_pos[Tp:], slots=t_i64[Tp:R], block_tables=bt_d,
                               context_lens=ctx_d, blocks_per_part=rm.blocks_per_part,
                               workspace=rm.workspace)
        meta = PrefillMeta(positions=d_pos, slots=t_i64[:R], cu_seqlens=d_cu, cu_host=cu,
                           tiles=(d_ts, d_tq), last_idx=t_i64[R:R + ns_all],
                           v_segs=None if n_dec else d_segs, decode=dmeta, n_prefill=Tp,
                           max_len=int(lens_a.max()))
        d_step = t_i64[R + ns_all:R + ns_all + 1]
        temp, topp = t_f32[:ns_all], t_f32[ns_all:]
        logits = self.model.forward_prefill(d_ids, meta, self.kv)
        toks = ops.sample(logits, temp, topk, topp, seed=self.seed, step=d_step)
        h_tok = torch.empty(ns_all, dtype=torch.int32, pin_memory=cuda)
        h_tok.copy_(toks, non_blocking=cuda)
        ovf = getattr(self.model, "ep_overflow", None)
        if ovf is not None:  # EP dropped-pair count, read with the tokens
            h_ovf = torch.empty(1, dtype=torch.int32, pin_memory=cuda)
            h_ovf.copy_(ovf.count, non_blocking=cuda)
            self._h_ovf[id(h_tok)] = (h_ovf, step)
        ev = None
        if cuda:
            ev = torch.cuda.Event()
            ev.record()
        self.stats["prefill_steps"] += 1
        self.stats["prefill_tokens"] += T
        return batch, lens, h_tok, ev

    def _finish_prefill(self, batch: list[Request], lens: list[int], toks) -> list[Request]:
        """Slot assignment + first-token bookkeeping of one prefill chunk."""
        now = time.perf_counter()
        finished = []
        for r, n, tok in zip(batch, lens, toks):
            tok = int(tok)
            s = self._assign_slot(r)
            self.ctx[s] = n
            self.last[s] = tok
            r.output_ids.append(tok)
            self.gen[s] = len(r.output_ids)
            if not r.first_token_time:
                r.first_token_time = now
            reason = self._finish_check(r, tok)
            if reason:
                self._release_slot(r)
                r.mark_finished(reason)
                finished.append(r)
        return finished

    def _run_mixed(self, batch: list[Request]) -> list[Request]:
        """One forward over [prefill rows of ``batch`` | one decode row per
        running request] (the running requests' next KV slots are already
        allocated): the decode rows share the prefill's weight reads and GEMM
        launches instead of waiting for the prefill to finish."""
        n = len(self.running)
        reqs = list(self.running)
        _, lens, h_tok, ev = self._launch_prefill(batch, n_dec=n)
        if ev is not None:
            ev.synchronize()
        h_tok = self._ep_redo_prefill(batch, n, h_tok)
        self.stats["mixed_steps"] += 1
        self.stats["decode_tokens"] += n
        self.ctx[:n] += 1
        self.gen[:n] += 1
        st = {"handle": None, "n": n, "reqs": reqs, "gen": self.gen[:n].copy(),
              "ctx": self.ctx[:n].copy()}
        if ev is not None:
            ev.synchronize()
        toks = h_tok.numpy()
        nseq = len(batch)
        st["toks"] = toks[nseq:nseq + n].copy()
        done = self._process(st, later_inflight=False)
        return done + self._finish_prefill(batch, lens, toks[:nseq])

    # ------------------------------------------------------------ decode
    def _ensure_blocks(self) -> None:
        """Give every running request room for its next token; preempt the
        newest requests when the cache is exhausted."""
        n = len(self.running)
        pos = self.ctx[:n]
        need = (pos % BS == 0) & (pos // BS >= self.nblk[:n])
        for s in np.nonzero(need)[0].tolist():
            if s >= len(self.running):
                continue
            r = self.running[s]
            while not self.alloc.can_allocate(1):
                victim = self.running[-1]
                self._preempt(victim)
                if victim is r:
                    break
            if r.slot < 0:
                continue
            b = self.alloc.allocate_one()
            r.blocks.append(b)
            self.bt[r.slot, len(r.blocks) - 1] = b
            self.nblk[r.slot] = len(r.blocks)

    def _preempt(self, r: Request) -> None:
        self._pressure = True
        self._release_slot(r)
        r.state = RequestState.WAITING
        r.num_preemptions += 1
        self.stats["preemptions"] += 1
        self.waiting.appendleft(r)
        self._waiting_tokens += r.num_tokens

    def _could_admit(self) -> bool:
        # zombies (finished, slot held until the in-flight step is read) count
        # as free: admitting drains the pipeline, which releases them
        free = self.max_batch - len(self.running) + len(self._zombies)
        if not self.waiting or free <= 0 or (self._pressure and self.running):
            return False
        # slot-bound (more queued requests than free slots): admit in groups
        return not (self.running and free < self.admit_group and len(self.waiting) > free)

    def _run_decode(self) -> list[Request]:
        """Decode with one step in flight.  While the batch composition stays
        fixed (no request can finish by length in the in-flight step, no
        pending EOS finishes, no admissions, next KV slots allocatable without
        preemption) step t+1 is enqueued - its input tokens gathered from step
        t's samples on the device - BEFORE step t's tokens are read, so the
        host bookkeeping of step t overlaps the GPU work of step t+1.  Any
        composition change drains the pipeline and re-stages from the host."""
        done: list[Request] = []
        if self._inflight is not None:
            if self._can_pipeline():
                nxt = self._launch_decode(pipelined=True)
                done = self._process(self._inflight, later_inflight=True)
                self._inflight = nxt
                return done
            done = self._process_inflight()
            if self._could_admit():
                return done  # the next step() admits and prefills
        with self.lock:
            self._ensure_blocks()
            self._sort_slots()
        if self.running:
            self._inflight = self._launch_decode(pipelined=False)
        return done

    # decode batches of at least this many rows keep their slots ordered by context length
    # (DRTC_SORT_SLOTS=0 disables): the persistent decode attention deals its (sequence,
    # kv head) items to waves round-robin with every odd round mirrored, so ordered slots give
    # each wave a balanced share of cache blocks (attention_decode.hip ``phys``)
    SORT_SLOTS_MIN = int(os.environ.get("DRTC_SORT_SLOTS", "256"))

    def _sort_slots(self) -> None:
        """Reorder the running slots by context length, longest first.  Only between steps
        with nothing in flight (a non-pipelined decode launch stages every input from the
        host); pipelined steps keep the order, since every context grows by one per step."""
        n = len(self.running)
        if self.SORT_SLOTS_MIN <= 0 or n < self.SORT_SLOTS_MIN or self._inflight is not None:
            return
        ctx = self.ctx[:n]
        if np.all(ctx[:-1] >= ctx[1:]):
            return
        order = np.argsort(-ctx, kind="stable")
        for arr in (self.bt, self.ctx, self.last, self.temp, self.topk, self.topp, self.gen,
                    self.max_new, self.eos_stop, self.nblk):
            arr[:n] = arr[:n][order]
        new_of = np.empty(n, dtype=np.int64)
        new_of[order] = np.arange(n)
        self.stop_ids = {int(new_of[s_]): v for s_, v in self.stop_ids.items()}
        self.running = [self.running[i] for i in order.tolist()]
        for s_, r in enumerate(self.running):
            r.slot = s_
        self.stats["slot_sorts"] += 1

    def _process_inflight(self) -> list[Request]:
        step, self._inflight = self._inflight, None
        return self._process(step, later_inflight=False)

    def _can_pipeline(self) -> bool:
        st = self._inflight
        n = len(self.running)
        if not self.pipeline or n != st["n"] or self._could_admit():
            return False
        if np.any(st["ctx"] + 1 >= self.max_model_len):
            return False  # no cache position left for a further step
        # Requests that finish by length in the in-flight step (or were found
        # finished earlier) ride along as zombies - their rows are computed and
        # discarded, their slots released at the next drain - as long as few
        # do: continuous traffic finishes ~max_batch/48 requests per step, and
        # draining for each would expose the host between every two steps.  A
        # closed wave finishing together drains at once (no wasted step).
        live = np.fromiter((r.state != RequestState.FINISHED for r in st["reqs"]), dtype=bool,
                           count=n)
        n_fin = int(((st["gen"] >= self.max_new[:n]) & live).sum())
        n_dead = int((~live).sum())
        if n_dead + n_fin > self.admit_group or n_dead + n_fin >= n:
            return False
        pos = self.ctx[:n]
        need = (pos % BS == 0) & (pos // BS >= self.nblk[:n])
        k = int(need.sum())
        if k == 0:
            return True
        with self.lock:
            if not self.alloc.can_allocate(k):
                return False  # would need a preemption: drain first
            for s_ in np.nonzero(need)[0].tolist():
                r = self.running[s_]
                b = self.alloc.allocate_one()
                r.blocks.append(b)
                self.bt[s_, len(r.blocks) - 1] = b
                self.nblk[s_] = len(r.blocks)
        return True

    def _launch_decode(self, pipelined: bool) -> dict:
        n = len(self.running)
        pos = self.ctx[:n].copy()
        bidx = pos // BS
        slots = self.bt[np.arange(n), bidx].astype(np.int64) * BS + pos % BS
        handle = self.runner.launch(n, None if pipelined else self.last[:n], pos, pos + 1, slots,
                                    self.bt[:n], self.temp[:n], self.topk[:n], self.topp[:n])
        self.stats["decode_steps"] += 1
        self.stats["decode_tokens"] += n
        if pipelined:
            self.stats["decode_steps_pipelined"] += 1
        self.ctx[:n] += 1
        self.gen[:n] += 1
        return {"handle": handle, "n": n, "reqs": list(self.running),
                "gen": self.gen[:n].copy(), "ctx": self.ctx[:n].copy()}

    def _process(self, st: dict, later_inflight: bool) -> list[Request]:
        """Read a launched step's tokens; finish requests.  With a later step
        in flight a finished request keeps its slot (its next token is
        discarded) until that step is read."""
        toks = st["toks"] if st.get("handle") is None else self.runner.wait(st["handle"])
        n, reqs = st["n"], st["reqs"]
        live = np.fromiter((r.state != RequestState.FINISHED for r in reqs), dtype=bool, count=n)
        for r, tok, ok in zip(reqs, toks.tolist(), live.tolist()):
            if ok:
                r.output_ids.append(tok)
        self.last[:n] = np.where(live, toks, self.last[:n])
        # finish conditions for the whole batch at once (see _finish_check)
        stop = self.eos_stop[:n] & (toks == self.cfg.eos_token_id)
        for s_, ids in self.stop_ids.items():
            if s_ < n and int(toks[s_]) in ids:
                stop[s_] = True
        length = (st["gen"] >= self.max_new[:n]) | (st["ctx"] + 1 >= self.max_model_len)
        done_idx = np.nonzero((stop | length) & live)[0].tolist()
        finished = [(reqs[i], "stop" if stop[i] else "length") for i in done_idx]
        for r, reason in finished:
            r.mark_finished(reason)
        if later_inflight:
            self._zombies.extend(r for r, _ in finished)
        else:
            # release in descending slot order: a release moves the last slot
            # into the hole, which must not be a slot still to be released
            rel = sorted([r for r, _ in finished] + self._zombies, key=lambda r: -r.slot)
            self._zombies = []
            for r in rel:
                self._release_slot(r)
        if finished:
            self._pressure = False
        return [r for r, _ in finished]


class EngineLoop:
    """Background thread that drives an engine; used by the LLM gRPC service
    so concurrent RPCs are batched together (continuous batching)."""

    # serving defaults (closed-loop service bench, profiles/r4o: 1024 clients, 10 waves, same
    # box: 89.9 % of the engine bench with neither, 94.9 % direct with both; via the Raft
    # leader 92.0 -> 94.5 % with arrival gathering at 16k tokens)
    SERVING_BURST_GAP_MS = 3.0
    SERVING_ADMIT_MIN_TOKENS = 8192

    def __init__(self, engine: LLMEngine, idle_sleep: float = 0.0005,
                 burst_gap_s: float | None = None, burst_max_s: float = 0.05):
        self.engine = engine
        self.idle_sleep = idle_sleep
        # burst gathering (DRTC_BURST_GAP_MS, 0 disables): see _hold
        if burst_gap_s is None:
            burst_gap_s = float(os.environ.get("DRTC_BURST_GAP_MS",
                                               str(self.SERVING_BURST_GAP_MS))) / 1000.0
        # arrival gathering for the mixed steps of a served engine (LLMEngine.admit_min_tokens;
        # DRTC_ADMIT_MIN_TOKENS=0 disables)
        if getattr(engine, "admit_min_tokens", None) == 0 and \
                "DRTC_ADMIT_MIN_TOKENS" not in os.environ:
            engine.admit_min_tokens = self.SERVING_ADMIT_MIN_TOKENS
        self.burst_gap_s, self.burst_max_s = burst_gap_s, burst_max_s
        self._last_submit = 0.0
        self._hold_start: float | None = None
        self._stop = threading.Event()
        self._wake = threading.Event()
        self.thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
        self.error: BaseException | None = None

    def start(self) -> "EngineLoop":
        self.thread.start()
        _LIVE_LOOPS.add(self)
        return self

    def submit(self, req: Request) -> Request:
        self.engine.add_request(req)
        self._last_submit = time.perf_counter()
        self._wake.set()
        return req

    def _hold(self) -> bool:
        """Burst gathering for closed-loop clients: while requests are still streaming in (the
        last one arrived less than ``burst_gap_s`` ago), the queue holds less than one prefill
        chunk and no large batch is decoding, let the burst gather instead of running a small
        prefill and then small decode steps for its first requests - at most ``burst_max_s``
        per burst.  A lone request waits at most ``burst_gap_s``."""
        if self.burst_gap_s <= 0:
            return False
        e = self.engine
        now = time.perf_counter()
        if (not e.waiting or e._waiting_tokens >= e.prefill_chunk_tokens
                or len(e.running) > e.max_batch // 4 or now - self._last_submit >= self.burst_gap_s):
            self._hold_start = None
            return False
        if self._hold_start is None:
            self._hold_start = now
        return now - self._hold_start < self.burst_max_s

    def alive(self) -> bool:
        return self.thread.is_alive() and self.error is None

    def _loop(self) -> None:
        try:
            while not self._stop.is_set():
                if self.engine.has_work():
                    if self._hold():
                        t0 = time.perf_counter()
                        self._wake.wait(self.burst_gap_s)
                        self._wake.clear()
                        self.engine.stats["burst_hold_us"] += int(1e6 * (time.perf_counter() - t0))
                        continue
                    self.engine.step()
                else:
                    # idle time (no request anywhere in the engine), reported in the
                    # engine counters: a closed-loop service shows its per-wave turnaround here
                    t0 = time.perf_counter()
                    self._wake.wait(0.05)
                    self._wake.clear()
                    self.engine.stats["idle_ms"] += int(1000 * (time.perf_counter() - t0))
        except BaseException as e:  # surface engine faults to callers
            self.error = e
            with self.engine.lock:
                pending = list(self.engine.waiting) + list(self.engine.running)
            for r in pending:
                r.mark_finished("error")

    def stop(self, timeout: float = 10.0) -> bool:
        """Ordered stop: end the loop at its next step boundary, join the thread, then shut
        the engine down (drain the in-flight step, fail what is still queued or running with
        "error: shutdown" so blocked callers return, wait for the device).  Returns whether the
        thread ended within ``timeout``; idempotent."""
        self._stop.set()
        self._wake.set()
        if self.thread.is_alive() and self.thread is not threading.current_thread():
            self.thread.join(timeout=timeout)
        ended = not self.thread.is_alive()
        if ended:
            try:
                self.engine.shutdown()
            except Exception:  # a dead device: nothing left to drain
                pass
        _LIVE_LOOPS.discard(self)
        return ended


# every started EngineLoop of the process: stopped in order at interpreter exit, while the
# runtime is intact - a daemon engine thread still inside HIP / torch native code when CPython
# finalizes is ended by a forced unwind through C++ frames and the process aborts
# ("terminate called without an active exception"); atexit runs before that
_LIVE_LOOPS: "weakref.WeakSet[EngineLoop]" = weakref.WeakSet()


@atexit.register
def _stop_live_loops() -> None:
    for loop in list(_LIVE_LOOPS):
        loop.stop(timeout=30.0)
