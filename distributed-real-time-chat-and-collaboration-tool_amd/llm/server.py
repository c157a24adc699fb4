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
  --serve FEATURE=MODEL[@GPUS][:tpN][:mem=F] (repeatable) hosts one engine group per
                     feature on GPUs of the node: the per-feature model matrix of
                     BASELINE.json (Gemma-2B smart reply, Llama-3-8B summarize,
                     Llama-3-70B TP=8 ask-AI, Mixtral suggestions) behind ONE service
                     address (features without a --serve use --model).  Groups may share
                     a GPU only with an explicit HBM budget each (mem=F: the fraction of
                     the GPU's total HBM the group may hold - weights, KV cache,
                     workspaces; at most 0.95 per GPU in all), so the split does not
                     depend on start order.  The five BASELINE configs on one 8-GPU node:
                       --serve answer=llama-3-70b@0-7:tp8:mem=0.35
                       --serve smart=gemma-2b@0,4:mem=0.6
                       --serve summary=llama-3-8b@1,5:mem=0.6
                       --serve suggest=mixtral-8x7b@2,3,6,7:mem=0.6
                     (the 70B TP group holds 101 GB of every GPU: 17.6 GB of weight shard
                     and ~80 GB of KV cache; each data-parallel replica beside it 173 GB;
                     the Raft cluster of the first config needs no GPU).

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

from ..protos import LLM_SERVICE, SERVER_QUEUE_OPTS, add_servicer
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
    if getattr(args, "hbm_budget", None):
        engine_kw["hbm_budget"] = float(args.hbm_budget)
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


def parse_serve(spec: str) -> tuple[str, str, list[int] | None, int, float | None]:
    """``FEATURE=MODEL[@GPUS][:tpN][:mem=F]`` -> (feature, model, devices or None, tp, HBM
    budget fraction or None); GPUS is a comma list of ids and ranges ("0", "1,2", "0-7")."""
    feat, eq, rest = spec.partition("=")
    feat = _FEATURE_ALIAS.get(feat.strip(), feat.strip())
    if not eq or feat not in FEATURES or not rest:
        raise ValueError(f"--serve {spec!r}: expected FEATURE=MODEL[@GPUS][:tpN][:mem=F], "
                         f"FEATURE in {FEATURES}")
    tp, mem = 1, None
    head, *opts = rest.split(":")
    for o in opts:
        if o.startswith("tp") and o[2:].isdigit():
            tp = int(o[2:])
        elif o.startswith("mem="):
            try:
                mem = float(o[4:])
            except ValueError:
                raise ValueError(f"--serve {spec!r}: bad mem={o[4:]!r}") from None
            if not 0.0 < mem <= 0.95:
                raise ValueError(f"--serve {spec!r}: mem must be in (0, 0.95]")
        else:
            raise ValueError(f"--serve {spec!r}: unknown option {o!r}")
    model, _, gpus = head.partition("@")
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
    return feat, model.strip(), devices, tp, mem


def _group_devices(devices: list[int] | None, tp: int, gpus: int) -> list[int]:
    """GPUs an engine group occupies (the defaults of build_backend when none are named)."""
    if devices:
        return list(devices)
    return list(range(tp if tp > 1 else max(1, gpus)))


def check_placement(groups: list[tuple[str, list[int], float | None]]) -> dict[int, float]:
    """Validate the GPU placement of engine groups [(name, devices, mem fraction or None)]:
    a GPU shared by several groups needs an explicit budget for every one of them, and the
    budgets on a GPU add up to at most 0.95.  Returns {gpu: budgeted fraction}."""
    on: dict[int, list[tuple[str, float | None]]] = {}
    for name, devs, mem in groups:
        for d in devs:
            on.setdefault(d, []).append((name, mem))
    used = {}
    for d, gs in sorted(on.items()):
        if len(gs) > 1 and any(m is None for _, m in gs):
            raise ValueError(f"GPU {d} is shared by {[n for n, _ in gs]}: give every group on "
                             "a shared GPU an HBM budget (:mem=F)")
        tot = sum(m or 0.0 for _, m in gs)
        if tot > 0.95 + 1e-9:
            raise ValueError(f"GPU {d}: HBM budgets of {[n for n, _ in gs]} add up to "
                             f"{tot:.2f} > 0.95")
        used[d] = tot
    return used


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
    # one engine group per distinct (model, GPUs, tp, budget); validate the placement of all
    # of them (and of the --model group serving the remaining features) before building any
    groups: dict = {}
    for feat, model, devices, tp, mem in parsed:
        groups.setdefault((model, tuple(devices) if devices else None, tp, mem), []).append(feat)
    need_default = len(seen) < len(FEATURES)
    gpu_free = args.backend == "scripted"  # scripted stand-ins hold no GPU memory
    # one rule for the GPUs of a --serve group, used by both the placement check and the build:
    # the named GPUs, else GPU 0 (tp1: one replica) or GPUs 0 .. tp-1 (a TP group)
    group_devs = {key: _group_devices(list(key[1]) if key[1] else None, key[2], 1)
                  for key in groups}
    placement = [(f"{'+'.join(fs)}={key[0]}", group_devs[key], key[3])
                 for key, fs in groups.items() if not (gpu_free or key[0] == "scripted")]
    if need_default and not (gpu_free or args.model == "scripted"):
        placement.append((f"default={args.model}", _group_devices(None, args.tp, args.gpus),
                          getattr(args, "hbm_budget", None)))
    check_placement(placement)
    made: dict = {}
    by_feature = {}
    for feat, model, devices, tp, mem in parsed:
        key = (model, tuple(devices) if devices else None, tp, mem)
        if key not in made:
            sub = argparse.Namespace(**vars(args))
            sub.model, sub.tp, sub.hbm_budget = model, tp, mem
            devs = group_devs[key]
            sub.gpus = len(devs) if tp == 1 else args.gpus
            sub.max_batch = args.max_batch or default_max_batch(model, tp)
            made[key] = build_backend(sub, devices=devs if (devices or tp == 1) else None)
        by_feature[feat] = made[key]
    default = None
    if need_default:
        sub = argparse.Namespace(**vars(args))
        sub.max_batch = args.max_batch or default_max_batch(args.model, args.tp)
        default = build_backend(sub)
    return FeatureRouter(by_feature, default)


def serve(backend, port: int = 50055, workers: int = 64, bind: str = "[::]", params=None):
    """Thread-pool gRPC server of the four RPCs over ``backend`` (SO_REUSEPORT off: a second
    server on a taken port fails instead of silently sharing it)."""
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=workers),
                         options=[("grpc.so_reuseport", 0)] + SERVER_QUEUE_OPTS)
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
            srv = grpc.aio.server(options=SERVER_QUEUE_OPTS)
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


def _stop_once(stop: threading.Event) -> None:
    """SIGTERM: start the ordered shutdown; further SIGTERMs are ignored (CPython restores
    the default - terminate - action for Python-level handlers during finalization, so a
    repeated SIGTERM from a supervisor would otherwise kill the exiting process)."""
    stop.set()
    signal.signal(signal.SIGTERM, signal.SIG_IGN)


def main(argv=None):
    # installed first: a SIGTERM while the engines load still ends the service in order
    stop = threading.Event()
    signal.signal(signal.SIGINT, lambda *a: stop.set())
    signal.signal(signal.SIGTERM, lambda *a: _stop_once(stop))
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
    ap.add_argument("--frontend", choices=("threads", "aio"), default=None,
                    help="gRPC front-end: a handler thread per in-flight RPC, or grpc.aio "
                         "coroutines on one event-loop thread (default: aio when the engines "
                         "run in worker processes - 94.0-94.9 %% of the engine vs 92.5 %% with "
                         "threads, 1,024 closed-loop clients, profiles/r6k, r6n - threads for "
                         "--in-process, whose engine thread would share the GIL with the loop)")
    ap.add_argument("--serve", action="append", default=[],
                    metavar="FEATURE=MODEL[@GPUS][:tpN][:mem=F]",
                    help="host FEATURE (smart | summary | answer | suggest) on its own engine "
                         "group (repeatable; see the module docstring)")
    ap.add_argument("--hbm-budget", type=float, default=None, metavar="F",
                    help="fraction of each GPU's HBM the --model engine group may hold "
                         "(default: 85 %% of what is free when it starts)")
    ap.add_argument("--log-level", default="INFO")
    args = parse_with_config(ap, argv)
    setup_logging(args.log_level)
    if args.serve:
        backend = build_feature_backends(args, args.serve)
        # a handler thread per request any of the engine groups can hold at once
        groups = {(m, tuple(d or ()), tp, mem) for _, m, d, tp, mem in map(parse_serve, args.serve)}
        slots = sum((args.max_batch or default_max_batch(m, tp)) * (len(d) if d and tp == 1 else 1)
                    for m, d, tp, _ in groups)
        workers = args.workers or slots + 16
    else:
        if not args.max_batch:
            args.max_batch = default_max_batch(args.model, args.tp)
        backend = build_backend(args)
        workers = args.workers or args.max_batch * max(1, args.gpus) + 16
    frontend = args.frontend or ("threads" if args.in_process else "aio")
    server = (serve_aio(backend, args.port) if frontend == "aio"
              else serve(backend, args.port, workers))
    log.info("LLM server on port %d (backend=%s model=%s gpus=%d tp=%d)", args.port, args.backend,
             args.model, args.gpus, args.tp)
    stop.wait()
    shutdown(server, backend)


def shutdown(server, backend, grace: float = 1.0) -> None:
    """Ordered stop of the service (SIGTERM / SIGINT): stop accepting RPCs (in-flight ones get
    ``grace`` seconds), stop the engine groups - loop threads joined, in-flight steps drained,
    unfinished requests failed so their handlers return the canned fallback, worker processes
    joined, devices synchronized - then wait for the RPC server to finish."""
    log.info("LLM server shutting down")
    done = server.stop(grace)
    close = getattr(backend, "close", None)
    if close is not None:
        close()
    if done is not None:
        done.wait(grace + 10)


if __name__ == "__main__":
    main()
