"""Text-generation backends behind the LLM service.

* ``EngineBackend``   - the on-GPU engine in this process (continuous batching
  through an EngineLoop thread; concurrent RPCs share decode steps).
* ``ReplicaRouter``   - data parallelism: N engine replicas, one process per
  GPU (``WorkerPool``), least-outstanding-requests routing.
* ``ScriptedBackend`` - deterministic, format-correct text for CPU tests and
  the "LLM disabled" plumbing configuration (no model at all).

All expose ``generate(prompts, params, timeout) -> list[str]`` - the role of
``self.model.generate_content`` in the reference's LLMServicer
(llm_server/llm_server.py:23-145, 167).
"""
from __future__ import annotations

import asyncio
import itertools
import logging
import multiprocessing as mp
import os
import queue
import threading
import time

from .prompts import fit_prompt
from ..engine.request import Request, SamplingParams

log = logging.getLogger(__name__)


class GenerationError(RuntimeError):
    pass


class ScriptedBackend:
    """Answers by prompt type with text in the contract's format."""

    def __init__(self, delay: float = 0.0):
        self.delay = delay
        self.calls = 0

    def generate(self, prompts, params, timeout=None):
        self.calls += len(prompts)
        if self.delay:
            time.sleep(self.delay)
        out = []
        for p in prompts:
            if "reply suggestions" in p:
                out.append("Sounds good to me\n- Let's do it tomorrow\n3. Thanks for the update")
            elif p.startswith("Summarize"):
                out.append("Summary: The team discussed the project plan and next steps.\n\n"
                           "Key Points:\n- Plan agreed\n- Review tomorrow\n- Deploy on friday")
            elif "COMPLETIONS:" in p:
                out.append("COMPLETIONS:\n- sounds like a plan\n- let me check\n- works for me\n\n"
                           "TOPICS:\n- deadlines\n- code review")
            else:
                out.append("Here is a short answer. It considers the context.")
        return out


class EngineBackend:
    def __init__(self, engine, tokenizer, loop=None):
        from ..engine.engine import EngineLoop

        self.engine = engine
        self.tok = tokenizer
        self.loop = loop or EngineLoop(engine).start()

    @property
    def outstanding(self) -> int:
        e = self.engine
        return len(e.running) + len(e.waiting)

    def generate(self, prompts, params, timeout=None):
        if isinstance(params, SamplingParams):
            params = [params] * len(prompts)
        reqs = []
        for p, prm in zip(prompts, params):
            ids = fit_prompt(self.tok, p, self.engine.max_model_len - prm.max_new_tokens - 1)
            reqs.append(self.loop.submit(Request(ids, prm)))
        deadline = None if timeout is None else time.monotonic() + timeout
        outs = []
        for r in reqs:
            left = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not r.wait(left):
                for q in reqs:  # the caller gives up: free their slots and KV blocks
                    self.engine.abort(q)
                raise GenerationError("generation timed out")
            if r.finish_reason.startswith("error"):
                raise GenerationError(r.finish_reason)
            outs.append(self.tok.decode(r.output_ids))
        return outs

    def close(self):
        self.loop.stop()


# ------------------------------------------------------------- DP workers
def _worker_main(rank: int, device: str, model_name: str, engine_kw: dict, inq, outqs, ctlq,
                 seed: int, hb_interval: float = 0.5):
    """One engine replica per GPU (separate process: one process per GPU).

    Requests arrive on ``inq`` as (front-end, request id, prompt ids or text, params); the
    completions of each engine step go back on ``outqs[fe]`` (one front-end, index 0, in
    this service).  Besides results, the worker sends a heartbeat with its engine
    counters every ``hb_interval`` s on ``ctlq``; the owner's health monitor evicts a replica
    whose process died or whose heartbeats stopped (SURVEY §5 failure detection: per-GPU
    replica eviction)."""
    import torch

    from ..engine.engine import EngineLoop, LLMEngine, freeze_gc
    from ..engine.tokenizer import ChatTokenizer
    from ..models import TransformerLM, get_config

    try:
        if device.startswith("cuda"):
            torch.cuda.set_device(torch.device(device))
        cfg = get_config(model_name)
        model = TransformerLM(cfg, device, seed=seed, full_then_shard=False)
        eng = LLMEngine(model, seed=rank, **engine_kw)
        # prompt text is tokenized (and replies detokenized) here, beside the engine, so the
        # gRPC front-end's single GIL only carries RPC handling (llm/backends.py ReplicaRouter)
        tok = ChatTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_id)
        eng.warmup(capture=True)
        freeze_gc()  # this process only serves the engine from here on
        loop = EngineLoop(eng).start()
        ctlq.put(("ready", rank, None))
    except BaseException as e:  # report start-up failures to the parent
        ctlq.put(("fatal", rank, repr(e)))
        return
    pending = {}
    parent = os.getppid()
    # finished requests arrive here from the engine thread (Request.on_done): the watcher
    # blocks on it instead of scanning every pending request each millisecond (a Python loop
    # over ~1k requests, 1000 times a second, that held the GIL against the engine's own
    # host work), and ships each burst of completions as ONE queue message
    done_q: queue.SimpleQueue = queue.SimpleQueue()
    text_rids: set = set()  # requests submitted as prompt text: reply with text as well
    fe_requests: dict[int, int] = {}  # requests received per front-end (heartbeat stats)

    def watcher():
        last_hb = 0.0
        while True:
            if os.getppid() != parent:
                # the parent died without closing the pool (os._exit, SIGKILL):
                # do not stay behind holding the GPU and its KV cache
                log.error("engine replica %d: parent process gone, exiting", rank)
                os._exit(0)
            batch = []
            try:
                batch.append(done_q.get(timeout=min(0.05, hb_interval)))
                while True:
                    batch.append(done_q.get_nowait())
            except queue.Empty:
                pass
            if batch:
                out: dict[int, list] = {}
                for r in batch:
                    ent = pending.pop(r.request_id, None)
                    if ent is not None:
                        text = tok.decode(r.output_ids) if r.request_id in text_rids else None
                        text_rids.discard(r.request_id)
                        out.setdefault(ent[0], []).append(
                            (r.request_id, (r.output_ids, r.finish_reason, text)))
                for fe, items in out.items():
                    outqs[fe].put(("done_batch", rank, items))
            if not loop.alive():  # engine fault: exit so the parent evicts/respawns us
                log.error("engine loop of replica %d died: %r", rank, loop.error)
                os._exit(3)
            now = time.monotonic()
            if now - last_hb >= hb_interval:
                last_hb = now
                st = dict(eng.stats)
                st.update(running=len(eng.running), waiting=len(eng.waiting),
                          pending=len(pending), alive=loop.alive(),
                          fe_requests=dict(fe_requests), kv_blocks=eng.kv.num_blocks,
                          kv_tokens=eng.kv.capacity_tokens, kv_gb=round(eng.kv.bytes / 1e9, 2),
                          hbm_budget=eng.hbm_budget)
                ctlq.put(("hb", rank, st))

    threading.Thread(target=watcher, daemon=True).start()
    while True:
        msg = inq.get()
        if msg is None:
            break
        if msg[0] == "abort":  # the caller gave up: free the slot / KV blocks
            ent = pending.get(msg[2])
            if ent is not None:
                eng.abort(ent[1])
            continue
        fe, rid, ids, prm = msg
        fe_requests[fe] = fe_requests.get(fe, 0) + 1
        if isinstance(ids, str):  # prompt text: fit + tokenize here (ReplicaRouter)
            ids = fit_prompt(tok, ids, eng.max_model_len - prm.max_new_tokens - 1)
            text_rids.add(rid)
        r = Request(ids, prm, request_id=rid, on_done=done_q.put)
        pending[rid] = (fe, r)
        try:
            loop.submit(r)
        except Exception as e:
            pending.pop(rid, None)
            outqs[fe].put(("done", rid, ([], f"error: {e}")))
    loop.stop()


class WorkerPool:
    """N engine processes (one per GPU); results and heartbeats come back on
    one queue.

    Health: a monitor thread evicts a replica when its process exits or its
    heartbeat is older than ``hb_timeout``; every request in flight on it is
    failed with ``error: replica lost`` (the router re-dispatches those), and
    with ``max_restarts > 0`` the replica is respawned on the same device and
    rejoins the pool once its engine reports ready (elastic recovery)."""

    LOST = "error: replica lost"

    def __init__(self, model_name: str, devices: list[str], engine_kw: dict, seed: int = 1234,
                 hb_interval: float = 0.5, hb_timeout: float = 30.0, max_restarts: int = 1,
                 start_timeout: float = 1800):
        self._ctx = mp.get_context("spawn")
        self.model_name, self.devices, self.engine_kw, self.seed = model_name, devices, engine_kw, seed
        self.hb_interval, self.hb_timeout, self.max_restarts = hb_interval, hb_timeout, max_restarts
        n = len(devices)
        self.outq = self._ctx.Queue()
        self.inqs = [None] * n
        self.procs = [None] * n
        self.healthy = [False] * n
        self.restarts = [0] * n
        self.last_hb = [time.monotonic()] * n
        self.worker_stats: list[dict] = [{} for _ in range(n)]
        self.evictions: list[tuple[int, str]] = []
        self.futures: dict[str, tuple] = {}
        self.load = [0] * n
        self._lock = threading.Lock()
        self._ids = itertools.count()
        self._closed = False
        for w in range(n):
            self._spawn(w)
        t_end = time.monotonic() + start_timeout
        while not all(self.healthy):
            kind, rank, info = self.outq.get(timeout=max(1.0, t_end - time.monotonic()))
            if kind == "fatal":
                self.close()
                raise GenerationError(f"engine worker {rank} failed: {info}")
            if kind == "ready":
                self.healthy[rank] = True
                self.last_hb[rank] = time.monotonic()
        self._threads = [threading.Thread(target=self._collect, daemon=True, name="pool-collect"),
                         threading.Thread(target=self._monitor, daemon=True, name="pool-monitor")]
        for t in self._threads:
            t.start()

    def _spawn(self, w: int) -> None:
        self.inqs[w] = self._ctx.Queue()
        self.procs[w] = self._ctx.Process(
            target=_worker_main, daemon=True,
            args=(w, self.devices[w], self.model_name, self.engine_kw, self.inqs[w], [self.outq],
                  self.outq, self.seed, self.hb_interval))
        self.procs[w].start()

    def _collect(self):
        while not self._closed:
            try:
                kind, rid, payload = self.outq.get(timeout=0.5)
            except queue.Empty:
                continue
            except (EOFError, OSError):
                return
            if kind == "hb":
                with self._lock:
                    self.last_hb[rid] = time.monotonic()
                    self.worker_stats[rid] = payload
                continue
            if kind == "ready":  # a respawned replica rejoins
                with self._lock:
                    self.healthy[rid] = True
                    self.last_hb[rid] = time.monotonic()
                log.info("engine replica %d back in service", rid)
                continue
            if kind == "fatal":
                log.error("engine replica %s failed to start: %s", rid, payload)
                continue
            if kind == "done":
                items = [(rid, payload)]
            elif kind == "done_batch":  # every completion of one engine step, one message
                items = payload
            else:
                continue
            ready = []
            with self._lock:
                for rid, res in items:
                    ev, slot, w = self.futures.get(rid, (None, None, None))
                    if ev is None or slot:
                        continue
                    slot.append(res)
                    self.load[w] -= 1
                    ready.append(ev)
            for ev in ready:
                ev.set()

    def _monitor(self):
        while not self._closed:
            time.sleep(min(0.25, self.hb_interval))
            now = time.monotonic()
            for w, p in enumerate(self.procs):
                if not self.healthy[w]:
                    continue
                if not p.is_alive():
                    self.evict(w, f"process exited (code {p.exitcode})")
                elif now - self.last_hb[w] > self.hb_timeout:
                    self.evict(w, f"no heartbeat for {now - self.last_hb[w]:.1f}s")

    def evict(self, w: int, reason: str) -> None:
        """Take replica ``w`` out of service and fail its in-flight requests."""
        failed = []
        with self._lock:
            if not self.healthy[w]:
                return
            self.healthy[w] = False
            self.evictions.append((w, reason))
            for rid, (ev, slot, ww) in self.futures.items():
                if ww == w and not slot:
                    slot.append(([], f"{self.LOST} ({reason})"))
                    failed.append(ev)
            self.load[w] = 0
        log.error("evicting engine replica %d: %s", w, reason)
        for ev in failed:
            ev.set()
        p = self.procs[w]
        if p.is_alive():
            p.kill()
        p.join(timeout=5)
        if not self._closed and self.restarts[w] < self.max_restarts:
            self.restarts[w] += 1
            log.info("respawning engine replica %d on %s", w, self.devices[w])
            self._spawn(w)

    def pick(self) -> int:
        with self._lock:
            live = [i for i in range(len(self.procs)) if self.healthy[i]]
            if not live:
                raise GenerationError("no healthy engine replica")
            return min(live, key=lambda i: self.load[i])

    def submit(self, worker: int, ids, params, ev=None):
        """Queue one request on replica ``worker``: ``ids`` are prompt token ids, or the
        prompt TEXT (a str), which the replica fits to its context and tokenizes itself and
        answers with the decoded text as well.  Returns (request id, event, result slot);
        ``ev`` (anything with ``set()``, e.g. a _LoopEvent) replaces the threading.Event."""
        rid = f"w{worker}-{next(self._ids)}"
        ev, slot = (ev if ev is not None else threading.Event()), []
        with self._lock:
            self.futures[rid] = (ev, slot, worker)
            self.load[worker] += 1
            if not self.healthy[worker]:  # raced with an eviction
                slot.append(([], f"{self.LOST} (not in service)"))
                ev.set()
                self.load[worker] -= 1
                return rid, ev, slot
        self.inqs[worker].put((0, rid, ids, params))
        return rid, ev, slot

    def release(self, rid):
        with self._lock:
            f = self.futures.pop(rid, None)
            if f is not None and not f[1]:  # released before its result: not in flight any more
                self.load[f[2]] -= 1

    def abort(self, rid):
        """Cancel an outstanding request on its replica, then release it."""
        with self._lock:
            f = self.futures.get(rid)
            w = f[2] if f is not None and not f[1] else None
        if w is not None and self.inqs[w] is not None:
            try:
                self.inqs[w].put(("abort", 0, rid))
            except (OSError, ValueError):
                pass
        self.release(rid)

    def health(self) -> list[dict]:
        with self._lock:
            now = time.monotonic()
            return [dict(replica=w, device=self.devices[w], healthy=self.healthy[w],
                         heartbeat_age_s=round(now - self.last_hb[w], 3), load=self.load[w],
                         restarts=self.restarts[w], **self.worker_stats[w])
                    for w in range(len(self.procs))]

    def close(self):
        """Ordered stop: no more evictions / respawns, each replica drains its engine and
        exits (killed after 10 s), every request still waiting here fails with "error:
        shutdown", and the collector / monitor threads are joined.  Idempotent."""
        if self._closed and not any(p is not None and p.is_alive() for p in self.procs):
            return
        self._closed = True
        for w, q in enumerate(self.inqs):
            if q is not None and self.procs[w] is not None and self.procs[w].is_alive():
                try:
                    q.put(None)
                except (OSError, ValueError):
                    pass
        for p in self.procs:
            if p is not None:
                p.join(timeout=10)
                if p.is_alive():
                    p.kill()
                    p.join(timeout=5)
        failed = []
        with self._lock:
            for ev, slot, _ in self.futures.values():
                if not slot:
                    slot.append(([], "error: shutdown"))
                    failed.append(ev)
        for ev in failed:
            ev.set()
        for t in getattr(self, "_threads", ()):
            if t is not threading.current_thread():
                t.join(timeout=5)


class ReplicaRouter:
    """Least-outstanding routing over the healthy replicas of a WorkerPool
    (one replica per GPU).  A request whose replica is evicted mid-flight is
    re-dispatched once to another healthy replica."""

    def __init__(self, pool: WorkerPool, tokenizer, max_model_len: int, max_redispatch: int = 1):
        self.pool = pool
        self.tok = tokenizer
        self.max_model_len = max_model_len
        self.max_redispatch = max_redispatch

    def close(self):
        """Stop the engine worker processes (and free their GPUs)."""
        self.pool.close()

    def generate(self, prompts, params, timeout=None):
        # prompts go to the replicas as text: tokenization and detokenization run in the
        # engine processes, beside their engines, not in this (gRPC front-end) process
        if isinstance(params, SamplingParams):
            params = [params] * len(prompts)
        jobs = []
        for p, prm in zip(prompts, params):
            jobs.append([p, prm, self.pool.submit(self.pool.pick(), p, prm), 0])
        deadline = None if timeout is None else time.monotonic() + timeout
        outs = []
        try:
            for job in jobs:
                while True:
                    rid, ev, slot = job[2]
                    left = None if deadline is None else max(0.0, deadline - time.monotonic())
                    if not ev.wait(left):
                        for j in jobs:  # free the replicas' slots and KV blocks
                            self.pool.abort(j[2][0])
                        raise GenerationError("generation timed out")
                    ids, reason, *text = slot[0]
                    if reason.startswith(WorkerPool.LOST) and job[3] < self.max_redispatch:
                        self.pool.release(rid)
                        job[3] += 1
                        job[2] = self.pool.submit(self.pool.pick(), job[0], job[1])
                        continue
                    if reason.startswith("error"):
                        raise GenerationError(reason)
                    outs.append(text[0] if text and text[0] is not None else self.tok.decode(ids))
                    break
        finally:
            for job in jobs:
                self.pool.release(job[2][0])
        return outs

    async def agenerate(self, prompt, params, timeout=None):
        """ReplicaRouter.generate for one prompt as a coroutine (same re-dispatch on a lost
        replica, same abort on timeout), without a thread blocked per request."""
        loop = asyncio.get_running_loop()
        pool = self.pool
        deadline = None if timeout is None else time.monotonic() + timeout
        job = pool.submit(pool.pick(), prompt, params, ev=_LoopEvent(loop))
        tries = 0
        try:
            while True:
                rid, ev, slot = job
                left = None if deadline is None else max(0.0, deadline - time.monotonic())
                try:
                    await asyncio.wait_for(ev.fut, left)
                except asyncio.TimeoutError:
                    pool.abort(rid)  # free the replica's slot and KV blocks
                    raise GenerationError("generation timed out") from None
                ids, reason, *text = slot[0]
                if reason.startswith(WorkerPool.LOST) and tries < self.max_redispatch:
                    pool.release(rid)
                    tries += 1
                    job = pool.submit(pool.pick(), prompt, params, ev=_LoopEvent(loop))
                    continue
                if reason.startswith("error"):
                    raise GenerationError(reason)
                return text[0] if text and text[0] is not None else self.tok.decode(ids)
        finally:
            pool.release(job[0])


class _LoopEvent:
    """Completion signal of one request for an asyncio caller: ``set()`` may run on any
    thread (the pool's collector, an eviction) and resolves ``fut`` on its loop."""

    __slots__ = ("loop", "fut")

    def __init__(self, loop):
        self.loop = loop
        self.fut = loop.create_future()

    def _resolve(self):
        if not self.fut.done():
            self.fut.set_result(None)

    def set(self):
        try:
            self.loop.call_soon_threadsafe(self._resolve)
        except RuntimeError:  # loop closed: nobody waits any more
            pass

    def is_set(self) -> bool:
        return self.fut.done()


def visible_gpus() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0


__all__ = ["EngineBackend", "ReplicaRouter", "ScriptedBackend", "WorkerPool", "GenerationError",
           "visible_gpus"]
