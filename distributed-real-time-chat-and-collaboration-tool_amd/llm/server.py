"""LLM service entry point: ``python -m drtc_amd.llm.server``.

Replaces the reference's Gemini proxy (llm_server/llm_server.py:476-523) with
on-node inference:

  --backend engine   (default) random-init model on the local MI355X GPUs;
                     ``--gpus N`` runs N data-parallel engine replicas, one
                     process per GPU (also for N = 1, unless --in-process),
                     behind a least-outstanding router with health checks;
                     ``--tp N`` runs one tensor-parallel engine over N GPUs
                     (RCCL all-reduce over xGMI), e.g. Llama-3-70B TP=8;
  --backend scripted deterministic format-correct text (no model; CPU tests).
  --serve FEATURE=MODEL[@GPUS][:tpN] (repeatable) hosts one engine group per feature
                     on its own GPUs of the node: the per-feature model matrix of
                     BASELINE.json (Gemma-2B smart reply, Llama-3-8B summarize,
                     Llama-3-70B TP=8 ask-AI, Mixtral suggestions) behind ONE service
                     address, e.g. --serve smart=gemma-2b@0 --serve summary=llama-3-8b@1
                     --serve answer=llama-3-70b@0-7:tp8 --serve suggest=mixtral-8x7b@2,3
                     (features without a --serve use --model).

Port 50055 and the thread-pool server match the reference.
"""
from __future__ import annotations

import asyncio
import argparse
import logging
import signal
import threading
from concurrent import futures

import grpc

from ..protos import LLM_SERVICE, add_servicer
from ..utils.config import parse_with_config
from ..utils.logging_utils import setup_logging
from .backends import ScriptedBackend
from .service import AsyncLLMServicer, LLMServicer

log = logging.getLogger("drtc_amd.llm.server")


# Engine batch (max concurrent requests per replica) when --max-batch is not given: the
# measured throughput knee on one MI355X that still answers inside the reference's
# per-feature node->LLM deadlines (20 s smart reply / suggestions, 10 s summarize and
# ask-AI: ref server/raft_node.py:2018,2084,2126,2187).  BASELINE.md: Llama-3-8B smart
# reply at 1024 (p50 2.5 s; 1536 adds ~1 %), Gemma-2B at 2048 (p50 1.5 s, +7.7 % over 1024),
# Mixtral suggestions at 1024 (p50 8.9 s, +11 % over 512, +40 % over 256), Llama-3-70B
# ask-AI on one GPU at 224 (p50 9.15 s, 3,663 tok/s; 256: p50 9.83 s, too close to the 10 s
# deadline; profiles/r4ab).
DEFAULT_MAX_BATCH = {"llama-3-8b": 1024, "gemma-2b": 2048, "mixtral-8x7b": 1024,
                     "llama-3-70b": 224}


def default_max_batch(model: str, tp: int = 1) -> int:
    """Engine batch for ``model`` when the operator did not choose one (256 for
    models without a measurement; a TP group has tp x the compute of one GPU)."""
    b = DEFAULT_MAX_BATCH.get(model, 256)
    return b if tp <= 1 else max(b, 256)


def build_backend(args, devices: list[int] | None = None):
    """Backend of one model: ``devices`` pins its GPUs (default 0 .. gpus-1 / tp-1)."""
    if args.backend == "scripted" or args.model == "scripted":
        return ScriptedBackend()
    from ..engine import ChatTokenizer
    from ..models import get_config

    cfg = get_config(args.model)
    tok = ChatTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_id)
    engine_kw = dict(max_batch=args.max_batch, max_model_len=args.max_model_len,
                     use_graphs=not args.no_graphs)
    if args.tp > 1:
        from ..parallel.tp_engine import TPEngineGroup

        return TPEngineGroup(args.model, args.tp, engine_kw, tok,
                             custom_allreduce=args.custom_allreduce, devices=devices)
    import torch

    n = len(devices) if devices else args.gpus
    if n <= 1 and (getattr(args, "in_process", False) or not torch.cuda.is_available()):
        from ..engine.engine import LLMEngine
        from ..models import TransformerLM
        from .backends import EngineBackend

        dev = f"cuda:{devices[0] if devices else 0}" if torch.cuda.is_available() else "cpu"
        model = TransformerLM(cfg, dev, seed=1234, full_then_shard=False)
        eng = LLMEngine(model, **engine_kw)
        eng.warmup(capture=True)
        return EngineBackend(eng, tok)
    from .backends import ReplicaRouter, WorkerPool

    # engines run in their own processes (one per GPU), so the gRPC handlers,
    # prompt building and tokenization here never contend for the engine
    # loop's GIL (scripts/service_bench.py: in-process 16.4k vs 17.7k tok/s)
    pool = WorkerPool(args.model, [f"cuda:{i}" for i in (devices or range(max(1, n)))], engine_kw)
    return ReplicaRouter(pool, tok, args.max_model_len)


FEATURES = ("smart", "summary", "answer", "suggest")
_FEATURE_ALIAS = {"smart_reply": "smart", "summarize": "summary", "ask": "answer",
                  "suggestions": "suggest"}


def parse_serve(spec: str) -> tuple[str, str, list[int] | None, int]:
    """``FEATURE=MODEL[@GPUS][:tpN]`` -> (feature, model, devices or None, tp); GPUS is a
    comma list of ids and ranges ("0", "1,2", "0-7")."""
    feat, eq, rest = spec.partition("=")
    feat = _FEATURE_ALIAS.get(feat.strip(), feat.strip())
    if not eq or feat not in FEATURES or not rest:
        raise ValueError(f"--serve {spec!r}: expected FEATURE=MODEL[@GPUS][:tpN], "
                         f"FEATURE in {FEATURES}")
    tp = 1
    if ":tp" in rest:
        rest, _, t = rest.rpartition(":tp")
        tp = int(t)
    model, _, gpus = rest.partition("@")
    devices = None
    if gpus:
        devices = []
        for part in gpus.split(","):
            a, _, b = part.partition("-")
            devices += list(range(int(a), int(b) + 1)) if b else [int(a)]
        if len(set(devices)) != len(devices):
            raise ValueError(f"--serve {spec!r}: a GPU is listed twice")
        if tp > 1 and len(devices) != tp:
            raise ValueError(f"--serve {spec!r}: tp{tp} needs exactly {tp} GPUs")
    return feat, model.strip(), devices, tp


def build_feature_backends(args, specs: list[str]):
    """One backend per distinct (model, GPUs, tp) of the ``--serve`` specs, routed per
    feature; features without a spec share the ``--model`` backend of ``build_backend``."""
    from .service import FeatureRouter

    parsed = [parse_serve(s) for s in specs]
    seen = set()
    for f, *_ in parsed:
        if f in seen:
            raise ValueError(f"feature {f!r} given twice")
        seen.add(f)
    made: dict = {}
    by_feature = {}
    for feat, model, devices, tp in parsed:
        key = (model, tuple(devices) if devices else None, tp)
        if key not in made:
            sub = argparse.Namespace(**vars(args))
            sub.model, sub.tp = model, tp
            sub.gpus = len(devices) if devices and tp == 1 else (1 if tp == 1 else args.gpus)
            sub.max_batch = args.max_batch or default_max_batch(model, tp)
            made[key] = build_backend(sub, devices=devices)
        by_feature[feat] = made[key]
    default = None
    if len(by_feature) < len(FEATURES):
        sub = argparse.Namespace(**vars(args))
        sub.max_batch = args.max_batch or default_max_batch(args.model, args.tp)
        default = build_backend(sub)
    return FeatureRouter(by_feature, default)


def serve(backend, port: int = 50055, workers: int = 64, bind: str = "[::]", params=None,
          reuse_port: bool = False):
    """Thread-pool gRPC server of the four RPCs over ``backend``.  ``reuse_port``: several
    front-end processes bind the same port (SO_REUSEPORT, llm/frontends.py); off by default
    so that a second server on a taken port fails instead of silently sharing it."""
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers),
                         options=[("grpc.so_reuseport", 1 if reuse_port else 0)])
    add_servicer(server, LLM_SERVICE, LLMServicer(backend, params))
    if server.add_insecure_port(f"{bind}:{port}") == 0:
        raise RuntimeError(f"cannot bind port {port}")
    server.start()
    return server


class AioServer:
    """``grpc.aio`` server on its own event-loop thread (the front-end of
    ``--frontend aio``): every in-flight RPC is a coroutine of that one thread instead of a
    pool thread blocked on its generation, so 1k concurrent requests cost no thread
    switching under the GIL.  ``stop(grace)`` mirrors grpc.Server.stop."""

    def __init__(self, backend, port: int, bind: str, params=None):
        self.loop = asyncio.new_event_loop()
        self._ready = threading.Event()
        self._err = None
        self._server = None
        self._thread = threading.Thread(target=self._run, args=(backend, port, bind, params),
                                        daemon=True, name="llm-aio")
        self._thread.start()
        self._ready.wait()
        if self._err is not None:
            raise self._err

    def _run(self, backend, port, bind, params):
        asyncio.set_event_loop(self.loop)

        async def start():
            srv = grpc.aio.server()
            add_servicer(srv, LLM_SERVICE, AsyncLLMServicer(backend, params))
            if srv.add_insecure_port(f"{bind}:{port}") == 0:
                raise RuntimeError(f"cannot bind port {port}")
            await srv.start()
            return srv

        try:
            self._server = self.loop.run_until_complete(start())
        except Exception as e:  # surfaced to the constructor's caller
            self._err = e
            self._ready.set()
            return
        self._ready.set()
        self.loop.run_forever()

    def stop(self, grace=None) -> threading.Event:
        done = threading.Event()
        if self._server is not None:
            fut = asyncio.run_coroutine_threadsafe(self._server.stop(grace), self.loop)
            try:
                fut.result(timeout=(grace or 0) + 10)
            finally:
                self.loop.call_soon_threadsafe(self.loop.stop)
                self._thread.join(timeout=10)
                self._server = None
        done.set()
        return done


def serve_aio(backend, port: int = 50055, bind: str = "[::]", params=None) -> AioServer:
    return AioServer(backend, port, bind, params)


def main(argv=None):
    ap = argparse.ArgumentParser(description="drtc_amd LLM service (on-GPU inference)")
    ap.add_argument("--port", type=int, default=50055)
    ap.add_argument("--backend", choices=("engine", "scripted"), default="engine")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--gpus", type=int, default=1, help="data-parallel replicas (1 process/GPU)")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree")
    ap.add_argument("--custom-allreduce", dest="custom_allreduce", action="store_true",
                    default=True,
                    help="one-shot IPC all-reduce (+ fused residual/RMSNorm) for decode-sized "
                         "TP messages, RCCL above the threshold (default)")
    ap.add_argument("--rccl-only", dest="custom_allreduce", action="store_false")
    ap.add_argument("--max-batch", type=int, default=0,
                    help="engine batch per replica (default: per model, DEFAULT_MAX_BATCH)")
    ap.add_argument("--max-model-len", type=int, default=4096)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--in-process", action="store_true",
                    help="1 GPU: run the engine in the server process (default: a worker process)")
    ap.add_argument("--workers", type=int, default=None,
                    help="gRPC handler threads; each blocks on one generation (default: "
                         "max-batch x replicas + 16, so the engine batch can fill)")
    ap.add_argument("--frontend", choices=("threads", "aio"), default="threads",
                    help="gRPC front-end: a handler thread per in-flight RPC, or grpc.aio "
                         "coroutines on one event-loop thread")
    ap.add_argument("--frontends", type=int, default=1,
                    help="gRPC front-end processes sharing the port (SO_REUSEPORT) over the "
                         "engine replicas (llm/frontends.py); 1 = this process")
    ap.add_argument("--serve", action="append", default=[], metavar="FEATURE=MODEL[@GPUS][:tpN]",
                    help="host FEATURE (smart | summary | answer | suggest) on its own engine "
                         "group (repeatable; see the module docstring)")
    ap.add_argument("--log-level", default="INFO")
    args = parse_with_config(ap, argv)
    setup_logging(args.log_level)
    if args.frontends > 1 and not args.serve and args.backend == "engine" and args.tp == 1:
        import torch

        from ..models import get_config
        from .frontends import serve_fleet

        if not args.max_batch:
            args.max_batch = default_max_batch(args.model, args.tp)
        cfg = get_config(args.model)
        n = max(1, args.gpus)
        devices = [f"cuda:{i}" for i in range(n)] if torch.cuda.is_available() else ["cpu"] * n
        group = serve_fleet(args.model, devices,
                            dict(max_batch=args.max_batch, max_model_len=args.max_model_len,
                                 use_graphs=not args.no_graphs),
                            args.frontends, args.port,
                            (cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_id),
                            args.max_model_len,
                            workers=args.workers or args.max_batch * n // args.frontends + 64)
        log.info("LLM server on port %d: %d front-end processes over %d engine replicas (%s)",
                 args.port, args.frontends, n, args.model)
        stop = threading.Event()
        signal.signal(signal.SIGINT, lambda *a: stop.set())
        signal.signal(signal.SIGTERM, lambda *a: stop.set())
        stop.wait()
        group.stop()
        return
    if args.serve:
        backend = build_feature_backends(args, args.serve)
        # a handler thread per request any of the engine groups can hold at once
        groups = {(m, tuple(d or ()), tp) for _, m, d, tp in map(parse_serve, args.serve)}
        slots = sum((args.max_batch or default_max_batch(m, tp)) * (len(d) if d and tp == 1 else 1)
                    for m, d, tp in groups)
        workers = args.workers or slots + 16
    else:
        if not args.max_batch:
            args.max_batch = default_max_batch(args.model, args.tp)
        backend = build_backend(args)
        workers = args.workers or args.max_batch * max(1, args.gpus) + 16
    server = (serve_aio(backend, args.port) if args.frontend == "aio"
              else serve(backend, args.port, workers))
    log.info("LLM server on port %d (backend=%s model=%s gpus=%d tp=%d)", args.port, args.backend,
             args.model, args.gpus, args.tp)
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *a: stop.set())
    signal.signal(signal.SIGTERM, lambda *a: stop.set())
    stop.wait()
    server.stop(1.0)


if __name__ == "__main__":
    main()
