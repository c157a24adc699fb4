"""Tensor-parallel serving: N lockstep engine replicas (one process per GPU).

SPMD design: every TP rank runs the *same* deterministic scheduler on the
*same* request stream, so ranks agree on every batch without exchanging
plans - only newly arrived requests are broadcast (a few bytes, over a gloo
CPU group) at each step boundary.  Inside a step the model's collectives
(all-reduce after o_proj/down_proj, all-gather of vocab-parallel logits) run
on RCCL over xGMI and are captured in the decode hipGraphs.  Logits are
bitwise identical on every rank after the all-gather and the fused sampler
is a pure function of (logits, seed, step), so every rank samples the same
tokens.  Rank 0 reports results to the front-end.
"""
from __future__ import annotations

import itertools
import multiprocessing as mp
import os
import queue
import socket
import threading
import time

from ..engine.request import Request, SamplingParams
from ..llm.prompts import fit_prompt


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def check_devices(devices: list[int], device_count: int, can_access) -> None:
    """A TP group needs one distinct GPU per rank, every pair peer-accessible over xGMI (the
    IPC all-reduce maps peer memory; RCCL uses the same links).  Raises on a violation.
    ``can_access(a, b)``: torch.cuda.can_device_access_peer (hipDeviceCanAccessPeer)."""
    if len(set(devices)) != len(devices):
        raise RuntimeError(f"TP ranks share a device: {devices}")
    bad = [d for d in devices if not 0 <= d < device_count]
    if bad:
        raise RuntimeError(f"TP devices {bad} out of range (device_count={device_count})")
    missing = [(a, b) for a in devices for b in devices if a != b and not can_access(a, b)]
    if missing:
        raise RuntimeError(f"no peer access between GPUs {missing[:4]} (hipDeviceCanAccessPeer)")


def tp_worker(rank: int, world: int, port: int, model_name: str, engine_kw: dict, inq, outq,
              custom_ar: bool = True, devices: list[int] | None = None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    from ..engine.engine import LLMEngine
    from ..models import TransformerLM, get_config
    from .comm import ParallelContext, init_distributed

    try:
        init_distributed()
        cpu = dist.new_group(backend="gloo")
        devices = list(devices) if devices is not None else list(range(world))
        dev = torch.device("cpu")
        if torch.cuda.is_available():
            n = torch.cuda.device_count()
            if n >= world:
                # one process per GPU over distinct, mutually peer-accessible devices
                check_devices(devices, n, torch.cuda.can_device_access_peer)
                dev = torch.device("cuda", devices[rank])
            else:  # rehearsal: ranks time-share the GPUs (gloo / IPC on one card)
                dev = torch.device("cuda", devices[rank] % n)
        pc = ParallelContext.from_world(tp=True)
        if custom_ar and dev.type == "cuda":
            pc.enable_custom_allreduce()
        cfg = get_config(model_name)
        model = TransformerLM(cfg, dev, pc=pc, seed=1234)
        eng = LLMEngine(model, seed=0, **engine_kw)
        # ranks finish weight init at different times; the custom all-reduce's
        # flag waits are time-bounded, so enter the captured warm-up together
        dist.barrier(group=cpu)
        eng.warmup(capture=True)
        from ..engine.engine import freeze_gc

        freeze_gc()  # this process only serves the engine from here on
        if rank == 0:
            outq.put(("ready", 0, None))
    except BaseException as e:
        outq.put(("fatal", rank, repr(e)))
        raise
    try:
        _serve_loop(rank, eng, pc, cpu, inq, outq)
    except BaseException as e:  # any rank: the front-end fails and ends the whole group
        outq.put(("fatal", rank, repr(e)))
        raise
    eng.shutdown()
    dist.barrier(group=cpu)
    dist.destroy_process_group()


def _serve_loop(rank, eng, pc, cpu, inq, outq):
    import torch.distributed as dist

    live: dict[str, Request] = {}  # request id -> Request, for aborts (same on every rank)
    while True:
        new = []
        if rank == 0:
            block = not eng.has_work()
            try:
                new.append(inq.get(timeout=0.05) if block else inq.get_nowait())
                while True:
                    new.append(inq.get_nowait())
            except queue.Empty:
                pass
        box = [new]
        dist.broadcast_object_list(box, src=0, group=cpu)
        new = box[0]
        stop = any(m is None for m in new)
        for m in new:
            if m is None:
                continue
            if m[0] == "abort":  # broadcast like a new request: every rank aborts at this step
                r = live.get(m[1])
                if r is not None:
                    eng.abort(r)
                continue
            rid, ids, prm = m
            live[rid] = eng.add_request(Request(ids, prm, request_id=rid))
        if stop:
            break
        if eng.has_work():
            done = eng.step()
            for r in done:
                live.pop(r.request_id, None)
            # a flag wait of the custom all-reduce that timed out means a peer
            # missed a call and this step summed stale staging: fail the whole
            # group (the supervisor starts fresh processes) instead of
            # returning tokens computed from wrong hidden states
            if pc.custom_ar is not None and pc.custom_ar.error():
                raise RuntimeError("custom all-reduce flag wait timed out (peer missed a call)")
            if rank == 0:
                for r in done:
                    outq.put(("done", r.request_id, (r.output_ids, r.finish_reason)))


class TPEngineGroup:
    """Front-end handle: generate() on a TP group of ``world`` GPUs."""

    def __init__(self, model_name: str, world: int, engine_kw: dict, tokenizer,
                 start_timeout: float = 1800, custom_allreduce: bool = True,
                 devices: list[int] | None = None):
        ctx = mp.get_context("spawn")
        self.inq, self.outq = ctx.Queue(), ctx.Queue()
        port = _free_port()
        # every rank reports a fatal error on outq (a split-K fault or an all-reduce flag
        # timeout seen by any rank fails the group at once); only rank 0 reports results
        self.procs = [ctx.Process(target=tp_worker, daemon=True,
                                  args=(r, world, port, model_name, engine_kw,
                                        self.inq if r == 0 else None, self.outq,
                                        custom_allreduce, devices))
                      for r in range(world)]
        for p in self.procs:
            p.start()
        kind, _, info = self.outq.get(timeout=start_timeout)
        if kind != "ready":
            raise RuntimeError(f"TP engine failed to start: {info}")
        self.tok = tokenizer
        self.max_model_len = engine_kw.get("max_model_len", 4096)
        self._futs: dict[str, tuple] = {}
        self.error = None
        self._lock = threading.Lock()
        self._ids = itertools.count()
        self._closed = False
        self._collector = threading.Thread(target=self._collect, daemon=True, name="tp-collect")
        self._collector.start()

    def _fail_all(self, reason: str) -> None:
        with self._lock:
            futs, self._futs = list(self._futs.values()), {}
        for ev, slot in futs:
            slot.append(([], reason))
            ev.set()

    def _collect(self):
        while not self._closed:
            try:
                kind, rid, payload = self.outq.get(timeout=0.5)
            except queue.Empty:
                continue
            except (EOFError, OSError):
                return
            if kind == "fatal":  # the group died: fail every outstanding request
                with self._lock:
                    self.error = payload
                self._fail_all(f"error: TP group failed: {payload}")
                # the other ranks may sit in a collective with the failed one: end them all
                for p in self.procs:
                    if p.is_alive():
                        p.kill()
                continue
            with self._lock:
                f = self._futs.pop(rid, None)
            if f is not None:
                f[1].append(payload)
                f[0].set()

    def generate(self, prompts, params, timeout=None):
        if isinstance(params, SamplingParams):
            params = [params] * len(prompts)
        hs, rids = [], []
        for p, prm in zip(prompts, params):
            ids = fit_prompt(self.tok, p, self.max_model_len - prm.max_new_tokens - 1)
            rid = f"tp-{next(self._ids)}"
            ev, slot = threading.Event(), []
            with self._lock:
                if self.error is not None:
                    raise RuntimeError(f"TP group failed: {self.error}")
                self._futs[rid] = (ev, slot)
            self.inq.put((rid, ids, prm))
            hs.append((ev, slot))
            rids.append((rid, ev, slot))
        deadline = None if timeout is None else time.monotonic() + timeout
        out = []
        for ev, slot in hs:
            left = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not ev.wait(left):
                with self._lock:  # the caller gives up: abort what is still running
                    pending = [rid for rid, _, _ in rids if rid in self._futs]
                    for rid in pending:
                        self._futs.pop(rid, None)
                for rid in pending:
                    self.inq.put(("abort", rid))
                raise TimeoutError("generation timed out")
            ids, reason = slot[0]
            if reason.startswith("error"):
                raise RuntimeError(reason)
            out.append(self.tok.decode(ids))
        return out

    def close(self):
        """Ordered stop: rank 0 broadcasts the stop, every rank drains its engine and leaves
        the process group (killed after 30 s); waiting requests fail; the collector ends."""
        if self._closed:
            return
        try:
            self.inq.put(None)
        except (OSError, ValueError):
            pass
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join(timeout=5)
        self._closed = True
        self._fail_all("error: shutdown")
        if self._collector is not threading.current_thread():
            self._collector.join(timeout=5)
