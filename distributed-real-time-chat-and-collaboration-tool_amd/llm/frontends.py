"""Several gRPC front-end processes over one set of engine replicas.

One Python process serving the LLM service handles every RPC of a closed-loop wave under one
GIL: when 1024 smart-reply requests finish together, their replies leave and the next 1024
requests arrive through that single interpreter (~0.2-0.3 s per wave on MI355X hosts, during
which the engine waits for work: profiles/r3o, docs/ROUND3_STATUS.md row 6).  Here the
service runs as K front-end processes that bind the SAME port (SO_REUSEPORT: the kernel
spreads client connections over them) and share the engine replicas (one process per GPU):

    clients --TCP--> front-end 0 ... K-1 (gRPC + prompt building + reply parsing)
                          |  request queue per replica (shared by every front-end)
                          v
                     engine replica w (llm/backends.py _worker_main: tokenize, engine,
                          |            detokenize; completions back per front-end)
                          +--> result queue of front-end f

The fleet (this module's ``EngineFleet``, in the parent process) owns the replicas: it
spawns them, watches their heartbeats, evicts a dead or silent replica (its front-ends fail
the requests in flight on it, which their routers re-dispatch once) and respawns it.
Each front-end routes with ``ReplicaRouter`` over a ``FleetClient`` (the WorkerPool request
interface against the shared queues); replica health is a shared byte array (``in_service``).
"""
from __future__ import annotations

import itertools
import logging
import multiprocessing as mp
import queue
import signal
import threading
import time

from .backends import GenerationError, ReplicaRouter, WorkerPool, _worker_main

log = logging.getLogger(__name__)


class EngineFleet:
    """Engine replica processes shared by ``n_frontends`` front-end processes."""

    def __init__(self, model_name: str, devices: list[str], engine_kw: dict, n_frontends: int,
                 seed: int = 1234, hb_interval: float = 0.5, hb_timeout: float = 30.0,
                 max_restarts: int = 1, start_timeout: float = 1800):
        self._ctx = mp.get_context("spawn")
        self.model_name, self.devices, self.engine_kw, self.seed = model_name, devices, engine_kw, seed
        self.hb_interval, self.hb_timeout, self.max_restarts = hb_interval, hb_timeout, max_restarts
        n = len(devices)
        self.ctlq = self._ctx.Queue()
        self.outqs = [self._ctx.Queue() for _ in range(n_frontends)]
        self.inqs = [self._ctx.Queue() for _ in range(n)]  # kept across respawns (front-ends hold them)
        self.in_service = self._ctx.Array("b", n)  # 1 = in service
        self.procs: list = [None] * n
        self.restarts = [0] * n
        self.last_hb = [time.monotonic()] * n
        self.worker_stats: list[dict] = [{} for _ in range(n)]
        self.evictions: list[tuple[int, str]] = []
        self._closed = False
        self._lock = threading.Lock()
        for w in range(n):
            self._spawn(w)
        t_end = time.monotonic() + start_timeout
        while not all(self.in_service[:]):
            kind, rank, info = self.ctlq.get(timeout=max(1.0, t_end - time.monotonic()))
            if kind == "fatal":
                self.close()
                raise GenerationError(f"engine worker {rank} failed: {info}")
            if kind == "ready":
                self.in_service[rank] = 1
                self.last_hb[rank] = time.monotonic()
        threading.Thread(target=self._control, daemon=True).start()
        threading.Thread(target=self._monitor, daemon=True).start()

    def handles(self, f: int) -> tuple:
        """What front-end ``f`` needs (picklable: passed to its process)."""
        return self.inqs, self.outqs[f], self.in_service, f

    def _spawn(self, w: int) -> None:
        self.procs[w] = self._ctx.Process(
            target=_worker_main, daemon=True,
            args=(w, self.devices[w], self.model_name, self.engine_kw, self.inqs[w], self.outqs,
                  self.ctlq, self.seed, self.hb_interval))
        self.procs[w].start()

    def _control(self):
        while not self._closed:
            try:
                kind, rank, info = self.ctlq.get(timeout=0.5)
            except queue.Empty:
                continue
            except (EOFError, OSError):
                return
            with self._lock:
                if kind == "hb":
                    self.last_hb[rank] = time.monotonic()
                    self.worker_stats[rank] = info
                elif kind == "ready":  # a respawned replica rejoins
                    self.last_hb[rank] = time.monotonic()
                    self.in_service[rank] = 1
                    log.info("engine replica %d back in service", rank)
                elif kind == "fatal":
                    log.error("engine replica %s failed to start: %s", rank, info)

    def _monitor(self):
        while not self._closed:
            time.sleep(min(0.25, self.hb_interval))
            now = time.monotonic()
            for w, p in enumerate(self.procs):
                if not self.in_service[w]:
                    continue
                if not p.is_alive():
                    self.evict(w, f"process exited (code {p.exitcode})")
                elif now - self.last_hb[w] > self.hb_timeout:
                    self.evict(w, f"no heartbeat for {now - self.last_hb[w]:.1f}s")

    def evict(self, w: int, reason: str) -> None:
        """Take replica ``w`` out of service: every front-end fails its requests in flight
        there (its router re-dispatches them), then the replica is respawned."""
        with self._lock:
            if not self.in_service[w]:
                return
            self.in_service[w] = 0
            self.evictions.append((w, reason))
        log.error("evicting engine replica %d: %s", w, reason)
        for q in self.outqs:
            q.put(("lost", w, reason))
        p = self.procs[w]
        if p.is_alive():
            p.kill()
        p.join(timeout=5)
        if not self._closed and self.restarts[w] < self.max_restarts:
            self.restarts[w] += 1
            log.info("respawning engine replica %d on %s", w, self.devices[w])
            self._spawn(w)

    def health(self) -> list[dict]:
        with self._lock:
            now = time.monotonic()
            return [dict(replica=w, device=self.devices[w], healthy=bool(self.in_service[w]),
                         heartbeat_age_s=round(now - self.last_hb[w], 3),
                         restarts=self.restarts[w], **self.worker_stats[w])
                    for w in range(len(self.procs))]

    def close(self):
        self._closed = True
        for w, q in enumerate(self.inqs):
            if self.procs[w] is not None and self.procs[w].is_alive():
                q.put(None)
        for p in self.procs:
            if p is not None:
                p.join(timeout=10)
                if p.is_alive():
                    p.kill()


class FleetClient:
    """The request side of ``WorkerPool`` (pick / submit / release / abort) inside one
    front-end process, against the fleet's shared replica queues."""

    LOST = WorkerPool.LOST

    def __init__(self, inqs, outq, in_service, fe: int):
        self.inqs, self.outq, self.in_service, self.fe = inqs, outq, in_service, fe
        n = len(inqs)
        self.load = [0] * n
        self.futures: dict[str, tuple] = {}
        self._lock = threading.Lock()
        self._ids = itertools.count()
        self._closed = False
        threading.Thread(target=self._collect, daemon=True).start()

    def _collect(self):
        while not self._closed:
            try:
                kind, key, payload = self.outq.get(timeout=0.5)
            except queue.Empty:
                continue
            except (EOFError, OSError):
                return
            ready = []
            with self._lock:
                if kind == "lost":  # the fleet evicted replica `key`
                    for rid, (ev, slot, w) in self.futures.items():
                        if w == key and not slot:
                            slot.append(([], f"{self.LOST} ({payload})"))
                            ready.append(ev)
                    self.load[key] = 0
                else:
                    items = [(key, payload)] if kind == "done" else payload
                    for rid, res in items:
                        ev, slot, w = self.futures.get(rid, (None, None, None))
                        if ev is None or slot:
                            continue
                        slot.append(res)
                        self.load[w] -= 1
                        ready.append(ev)
            for ev in ready:
                ev.set()

    def pick(self) -> int:
        with self._lock:
            live = [i for i in range(len(self.inqs)) if self.in_service[i]]
            if not live:
                raise GenerationError("no healthy engine replica")
            return min(live, key=lambda i: self.load[i])

    def submit(self, worker: int, ids, params, ev=None):
        rid = f"f{self.fe}-w{worker}-{next(self._ids)}"
        ev, slot = (ev if ev is not None else threading.Event()), []
        with self._lock:
            self.futures[rid] = (ev, slot, worker)
            self.load[worker] += 1
        self.inqs[worker].put((self.fe, rid, ids, params))
        return rid, ev, slot

    def release(self, rid):
        with self._lock:
            f = self.futures.pop(rid, None)
            if f is not None and not f[1]:
                self.load[f[2]] -= 1

    def abort(self, rid):
        with self._lock:
            f = self.futures.get(rid)
            w = f[2] if f is not None and not f[1] else None
        if w is not None:
            try:
                self.inqs[w].put(("abort", self.fe, rid))
            except (OSError, ValueError):
                pass
        self.release(rid)

    def close(self):
        self._closed = True


def _frontend_main(handles, port: int, bind: str, workers: int, tokenizer_spec, max_model_len: int,
                   ready, stop, params=None):
    """One gRPC front-end process: FleetClient + ReplicaRouter + LLMServicer on the shared
    port (SO_REUSEPORT)."""
    from ..engine import ChatTokenizer
    from .server import serve

    signal.signal(signal.SIGINT, signal.SIG_IGN)  # the parent stops us through `stop`
    client = FleetClient(*handles)
    router = ReplicaRouter(client, ChatTokenizer(*tokenizer_spec), max_model_len)
    server = serve(router, port, workers, bind=bind, params=params, reuse_port=True)
    ready.set()
    stop.wait()
    server.stop(1.0).wait(5.0)
    client.close()


class FrontendGroup:
    """K front-end processes serving the LLM service on one port over an EngineFleet."""

    def __init__(self, fleet: EngineFleet, n: int, port: int, tokenizer_spec: tuple,
                 max_model_len: int, workers: int = 256, bind: str = "[::]",
                 start_timeout: float = 120, params=None):
        ctx = mp.get_context("spawn")
        self.fleet = fleet
        self.stop_ev = ctx.Event()
        self.procs = []
        readies = []
        for f in range(n):
            r = ctx.Event()
            p = ctx.Process(target=_frontend_main, daemon=True,
                            args=(fleet.handles(f), port, bind, workers, tokenizer_spec,
                                  max_model_len, r, self.stop_ev, params))
            p.start()
            self.procs.append(p)
            readies.append(r)
        for f, r in enumerate(readies):
            if not r.wait(start_timeout):
                self.stop()
                raise RuntimeError(f"LLM front-end {f} did not start")

    def stop(self, grace=None):
        self.stop_ev.set()
        for p in self.procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
        self.fleet.close()
        ev = threading.Event()
        ev.set()
        return ev


def serve_fleet(model_name: str, devices: list[str], engine_kw: dict, n_frontends: int,
                port: int, tokenizer_spec: tuple, max_model_len: int, workers: int = 256,
                bind: str = "[::]", params=None) -> FrontendGroup:
    """Engine replicas on ``devices`` behind ``n_frontends`` gRPC front-end processes on
    ``port``; ``stop()`` on the result shuts everything down."""
    fleet = EngineFleet(model_name, devices, engine_kw, n_frontends)
    try:
        return FrontendGroup(fleet, n_frontends, port, tokenizer_spec, max_model_len, workers,
                             bind, params=params)
    except BaseException:
        fleet.close()
        raise


__all__ = ["EngineFleet", "FleetClient", "FrontendGroup", "serve_fleet"]
