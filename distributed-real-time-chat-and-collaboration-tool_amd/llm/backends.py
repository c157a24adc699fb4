"""Text-generation backends behind the LLM service.

* ``EngineBackend``   - the on-GPU engine in this process (continuous batching
  through an EngineLoop thread; concurrent RPCs share decode steps).
* ``ReplicaRouter``   - data parallelism: N engine replicas, one process per
  GPU (``WorkerPool``), least-outstanding-requests routing.
* ``ScriptedBackend`` - deterministic, format-correct text for CPU tests and
  the "LLM disabled" plumbing configuration (no model at all).

All expose ``generate(prompts, params, timeout) -> list[str]``.
"""
from __future__ import annotations

import itertools
import logging
import multiprocessing as mp
import os
import queue
import threading
import time

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
            ids = self.tok.encode(p)
            limit = self.engine.max_model_len - prm.max_new_tokens - 1
            if len(ids) > limit:  # keep the newest context (prompts end with instructions)
                ids = ids[:1] + ids[len(ids) - limit + 1:]
            reqs.append(self.loop.submit(Request(ids, prm)))
        deadline = None if timeout is None else time.monotonic() + timeout
        outs = []
        for r in reqs:
            left = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not r.wait(left):
                raise GenerationError("generation timed out")
            if r.finish_reason.startswith("error"):
                raise GenerationError(r.finish_reason)
            outs.append(self.tok.decode(r.output_ids))
        return outs

    def close(self):
        self.loop.stop()


# ------------------------------------------------------------- DP workers
def _worker_main(rank: int, device: str, model_name: str, engine_kw: dict, inq, outq, seed: int):
    """One engine replica per GPU (separate process: one process per GPU)."""
    import torch

    from ..engine.engine import EngineLoop, LLMEngine
    from ..models import TransformerLM, get_config

    try:
        if device.startswith("cuda"):
            torch.cuda.set_device(torch.device(device))
        cfg = get_config(model_name)
        model = TransformerLM(cfg, device, seed=seed, full_then_shard=False)
        eng = LLMEngine(model, seed=rank, **engine_kw)
        eng.warmup(capture=True)
        loop = EngineLoop(eng).start()
        outq.put(("ready", rank, None))
    except BaseException as e:  # report start-up failures to the parent
        outq.put(("fatal", rank, repr(e)))
        return
    pending = {}

    def watcher():
        while True:
            for rid, r in list(pending.items()):
                if r._done.is_set():
                    pending.pop(rid, None)
                    outq.put(("done", rid, (r.output_ids, r.finish_reason)))
            time.sleep(0.001)

    threading.Thread(target=watcher, daemon=True).start()
    while True:
        msg = inq.get()
        if msg is None:
            break
        rid, ids, prm = msg
        r = Request(ids, prm, request_id=rid)
        pending[rid] = r
        try:
            loop.submit(r)
        except Exception as e:
            pending.pop(rid, None)
            outq.put(("done", rid, ([], f"error: {e}")))
    loop.stop()


class WorkerPool:
    """N engine processes; results come back on one queue."""

    def __init__(self, model_name: str, devices: list[str], engine_kw: dict, seed: int = 1234):
        ctx = mp.get_context("spawn")
        self.outq = ctx.Queue()
        self.inqs = [ctx.Queue() for _ in devices]
        self.procs = [ctx.Process(target=_worker_main, args=(i, d, model_name, engine_kw, q, self.outq, seed),
                                  daemon=True) for i, (d, q) in enumerate(zip(devices, self.inqs))]
        for p in self.procs:
            p.start()
        ready = 0
        while ready < len(self.procs):
            kind, rank, info = self.outq.get(timeout=1800)
            if kind == "fatal":
                raise GenerationError(f"engine worker {rank} failed: {info}")
            ready += 1
        self.futures: dict[str, tuple] = {}
        self.load = [0] * len(self.procs)
        self._lock = threading.Lock()
        self._ids = itertools.count()
        threading.Thread(target=self._collect, daemon=True).start()

    def _collect(self):
        while True:
            kind, rid, payload = self.outq.get()
            if kind != "done":
                continue
            with self._lock:
                ev, slot, w = self.futures.get(rid, (None, None, None))
                if ev is None:
                    continue
                slot.append(payload)
                self.load[w] -= 1
            ev.set()

    def submit(self, worker: int, ids, params):
        rid = f"w{worker}-{next(self._ids)}"
        ev, slot = threading.Event(), []
        with self._lock:
            self.futures[rid] = (ev, slot, worker)
            self.load[worker] += 1
        self.inqs[worker].put((rid, ids, params))
        return rid, ev, slot

    def release(self, rid):
        with self._lock:
            self.futures.pop(rid, None)

    def close(self):
        for q in self.inqs:
            q.put(None)
        for p in self.procs:
            p.join(timeout=10)


class ReplicaRouter:
    """Least-outstanding routing over a WorkerPool (one replica per GPU)."""

    def __init__(self, pool: WorkerPool, tokenizer, max_model_len: int):
        self.pool = pool
        self.tok = tokenizer
        self.max_model_len = max_model_len

    def generate(self, prompts, params, timeout=None):
        if isinstance(params, SamplingParams):
            params = [params] * len(prompts)
        handles = []
        for p, prm in zip(prompts, params):
            ids = self.tok.encode(p)
            limit = self.max_model_len - prm.max_new_tokens - 1
            if len(ids) > limit:
                ids = ids[:1] + ids[len(ids) - limit + 1:]
            w = min(range(len(self.pool.load)), key=lambda i: self.pool.load[i])
            handles.append(self.pool.submit(w, ids, prm))
        deadline = None if timeout is None else time.monotonic() + timeout
        outs = []
        try:
            for rid, ev, slot in handles:
                left = None if deadline is None else max(0.0, deadline - time.monotonic())
                if not ev.wait(left):
                    raise GenerationError("generation timed out")
                ids, reason = slot[0]
                if reason.startswith("error"):
                    raise GenerationError(reason)
                outs.append(self.tok.decode(ids))
        finally:
            for rid, _, _ in handles:
                self.pool.release(rid)
        return outs


def visible_gpus() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0


__all__ = ["EngineBackend", "ReplicaRouter", "ScriptedBackend", "WorkerPool", "GenerationError",
           "visible_gpus", "queue", "os"]
