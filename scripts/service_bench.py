#!/usr/bin/env python3
"""End-to-end service load driver (SURVEY §4.2 "Benchmarks").

Drives smart-reply RPCs the way the product does:

* ``--mode direct``: clients -> llm.LLMService/GetSmartReply (5 recent
  messages per request, the reference's contract);
* ``--mode raft``: clients -> raft.RaftNode/GetSmartReply on the leader of a
  3-node local cluster (token check, last-5 channel messages from the
  replicated state, node -> LLM proxy), i.e. the CLI's ``smart_reply`` path.

The LLM service runs in-process on the in-tree engine (``--backend engine``,
one GPU, random-init weights) or the scripted backend (CPU plumbing).
Reports one JSON line: requests/s, generated tokens/s, p50/p99 latency.

  python scripts/service_bench.py --model llama-3-8b --requests 2048 --concurrency 512
  python scripts/service_bench.py --backend scripted --mode raft --requests 200
"""
import argparse
import collections
import json
import multiprocessing as mp
import os
import random
import statistics
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import grpc  # noqa: E402

from drtc_amd.llm.server import serve as serve_llm, serve_aio  # noqa: E402
from drtc_amd.llm.service import FeatureParams  # noqa: E402
from drtc_amd.protos import LLM_SERVICE, RAFT_SERVICE, llm_pb, make_stub, raft_pb  # noqa: E402
from drtc_amd.utils.cluster import LocalCluster, ProcessCluster, free_port  # noqa: E402
from drtc_amd.utils.metrics import METRICS  # noqa: E402
from drtc_amd.utils.synthetic import channel_history  # noqa: E402


def build_backend(args):
    if args.backend == "scripted":
        from drtc_amd.llm.backends import ScriptedBackend
        return ScriptedBackend(), None
    if args.backend == "pool":  # engine in its own process (as llm/server.py runs N GPUs)
        from drtc_amd.engine import ChatTokenizer
        from drtc_amd.llm.backends import ReplicaRouter, WorkerPool
        from drtc_amd.models import get_config

        cfg = get_config(args.model)
        pool = WorkerPool(args.model, ["cuda:0"], dict(max_batch=args.max_batch, max_model_len=2048))
        tok = ChatTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_id)
        return ReplicaRouter(pool, tok, 2048), None
    import torch

    from drtc_amd.engine import ChatTokenizer, LLMEngine
    from drtc_amd.llm.backends import EngineBackend
    from drtc_amd.models import TransformerLM, get_config

    cfg = get_config(args.model)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    model = TransformerLM(cfg, dev, seed=1234, full_then_shard=False)
    eng = LLMEngine(model, max_batch=args.max_batch, max_model_len=2048,
                    use_graphs=dev == "cuda")
    eng.warmup(capture=True)
    return EngineBackend(eng, ChatTokenizer(cfg.vocab_size, cfg.bos_token_id,
                                            cfg.eos_token_id)), eng


# one HTTP/2 connection per stub (no shared subchannel): a service with several front-end
# processes on one port (SO_REUSEPORT) balances per connection
_OPTS = [("grpc.use_local_subchannel_pool", 1)]


def run_load(target, n_requests: int, threads: int, seed: int, ready=None, go=None):
    """``threads`` client threads issue ``n_requests`` GetSmartReply RPCs in
    total; returns (latencies s, errors, wall start, wall end, finish wall times).
    ``ready`` / ``go`` (multiprocessing primitives): the client processes connect their
    channels, report ready and wait for one common start, so the load window starts with
    every client (as bench.py's waves do) instead of with process-spawn skew."""
    mode, address, token = target
    rng = random.Random(seed)
    if mode == "raft":
        def one(stub):
            r = stub.GetSmartReply(raft_pb.SmartReplyRequest(token=token, channel_id="general"),
                                   timeout=120)
            assert r.success and len(r.suggestions) == 3
        service = RAFT_SERVICE
    else:
        histories = [[llm_pb.Message(sender=m.sender, content=m.content)
                      for m in channel_history(rng, 5)] for _ in range(64)]

        def one(stub):
            r = stub.GetSmartReply(llm_pb.SmartReplyRequest(
                recent_messages=histories[rng.randrange(len(histories))]), timeout=120)
            assert len(r.suggestions) == 3
        service = LLM_SERVICE
    chans = [grpc.insecure_channel(address, options=_OPTS) for _ in range(8)]
    stubs = [make_stub(ch, service) for ch in chans]
    lat, errors, lock, it = [], [], threading.Lock(), iter(range(n_requests))
    fin = []

    def worker(k):
        stub = stubs[k % len(stubs)]
        while True:
            with lock:
                if next(it, None) is None:
                    return
            t = time.perf_counter()
            try:
                one(stub)
            except (grpc.RpcError, AssertionError) as e:
                with lock:
                    errors.append(f"{repr(e)[:400]} (at {time.time() - t_start:.1f} s)")
                continue
            with lock:
                lat.append(time.perf_counter() - t)
                fin.append(time.time())
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(threads)]
    if go is not None:
        for ch in chans:
            grpc.channel_ready_future(ch).result(timeout=60)
        ready.release()
        go.wait()
    t_start = time.time()
    [t.start() for t in ths]
    [t.join() for t in ths]
    return lat, errors, t_start, time.time(), fin


def run_open_loop(target, n_requests: int, rate: float, seed: int):
    """Open loop: RPCs issued as a Poisson process at ``rate`` req/s (gRPC
    futures, one dispatcher thread), whatever the service's progress; latency
    counts from each request's SCHEDULED send time.  Returns (latencies s,
    errors, wall start, wall end)."""
    mode, address, token = target
    rng = random.Random(seed)
    if mode == "raft":
        stubs = [make_stub(grpc.insecure_channel(address, options=_OPTS), RAFT_SERVICE) for _ in range(8)]

        def req(stub):
            return stub.GetSmartReply.future(
                raft_pb.SmartReplyRequest(token=token, channel_id="general"), timeout=120)
    else:
        histories = [[llm_pb.Message(sender=m.sender, content=m.content)
                      for m in channel_history(rng, 5)] for _ in range(64)]
        stubs = [make_stub(grpc.insecure_channel(address, options=_OPTS), LLM_SERVICE) for _ in range(8)]

        def req(stub):
            return stub.GetSmartReply.future(llm_pb.SmartReplyRequest(
                recent_messages=histories[rng.randrange(len(histories))]), timeout=120)
    lat, errors, lock = [], [], threading.Lock()
    done = threading.Semaphore(0)

    def on_done(fut, t_sched):
        try:
            r = fut.result()
            ok = len(r.suggestions) == 3 and (mode != "raft" or r.success)
            with lock:
                (lat.append(time.perf_counter() - t_sched) if ok
                 else errors.append("bad response"))
        except grpc.RpcError as e:
            with lock:
                errors.append(repr(e)[:200])
        done.release()

    t_start = time.time()
    t0 = time.perf_counter()
    t = 0.0
    for i in range(n_requests):
        t += rng.expovariate(rate)
        d = t0 + t - time.perf_counter()
        if d > 0:
            time.sleep(d)
        f = req(stubs[i % len(stubs)])
        f.add_done_callback(lambda fut, ts=t0 + t: on_done(fut, ts))
    for _ in range(n_requests):
        done.acquire()
    return lat, errors, t_start, time.time(), []


def _delta(before, pool):
    """Per-replica counter increments since ``before`` (WorkerPool.health() snapshots)."""
    time.sleep(2 * pool.hb_interval)
    out = []
    for b, a in zip(before, pool.health()):
        out.append({k: a[k] - b.get(k, 0) for k in ("idle_ms", "burst_hold_us", "prefill_steps", "prefill_tokens",
                                                   "decode_steps", "mixed_steps", "decode_tokens",
                                                   "decode_us", "mixed_us", "prefill_us",
                                                   "drain_us")
                    if isinstance(a.get(k), int)})
    return out


def _client_main(target, n_requests, threads, seed, q, ready, go):
    q.put(run_load(target, n_requests, threads, seed, ready, go))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=("engine", "pool", "scripted"), default="engine",
                    help="engine: in-process engine; pool: engine in a worker process")
    ap.add_argument("--client-procs", type=int, default=0,
                    help="run the load clients in this many separate processes (0: threads here)")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--mode", choices=("direct", "raft"), default="direct")
    ap.add_argument("--frontend", choices=("threads", "aio"), default=None,
                    help="LLM service front-end (llm/server.py --frontend; default as there: "
                         "aio, threads for the in-process engine backend)")
    ap.add_argument("--in-process-nodes", action="store_true",
                    help="--mode raft: run the 3 Raft nodes in this process (default: one "
                         "process per node, as deployed)")
    ap.add_argument("--requests", type=int, default=1024)
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--max-batch", type=int, default=512)
    ap.add_argument("--arrival-rate", type=float, default=0.0, metavar="REQ_PER_S",
                    help="open loop: Poisson arrivals at this rate (instead of --concurrency "
                         "closed-loop clients); reports p50/p99 latency and engine TPOT")
    args = ap.parse_args()

    fp = FeatureParams(ignore_eos=True)  # full 48-token budget per reply (random weights)
    port = free_port()
    backend, eng = build_backend(args)
    if args.frontend is None:
        args.frontend = "threads" if args.backend == "engine" else "aio"
    if args.frontend == "aio":
        llm_srv = serve_aio(backend, port=port, bind="127.0.0.1", params=fp)
    else:
        llm_srv = serve_llm(backend, port=port, bind="127.0.0.1", params=fp,
                            workers=args.concurrency + 8)
    rng = random.Random(0)
    cluster = None
    tmp = tempfile.TemporaryDirectory()
    try:
        if args.mode == "raft":
            cls = LocalCluster if args.in_process_nodes else ProcessCluster
            cluster = cls(3, data_root=tmp.name, llm_address=f"127.0.0.1:{port}",
                          grpc_workers=args.concurrency + 16).start()
            leader = cluster.leader()
            token = cluster.login(leader)
            st = cluster.stub(leader)
            for m in channel_history(rng, 5):
                st.SendMessage(raft_pb.SendMessageRequest(token=token, channel_id="general",
                                                          content=m.content))
            target = (args.mode, cluster.peers[leader], token)
        else:
            target = (args.mode, f"127.0.0.1:{port}", None)

        # warm-up (graph buckets, first-use GEMM kernels)
        run_load(target, 16, 16, 0)
        if eng is not None:
            eng.stats.clear()
        METRICS.reset()
        pool = getattr(backend, "pool", None)
        if pool is not None:  # replica counters arrive with the heartbeats
            time.sleep(2 * pool.hb_interval)
        rs0 = pool.health() if pool is not None else None
        if args.arrival_rate > 0:
            lat, errors, t_s, t_e, fin = run_open_loop(target, args.requests, args.arrival_rate, 1)
            dt = t_e - t_s
        elif args.client_procs > 0:  # clients outside this process (no shared GIL)
            ctx = mp.get_context("spawn")
            q = ctx.Queue()
            k = args.client_procs
            ready, go = ctx.Semaphore(0), ctx.Event()
            procs = [ctx.Process(target=_client_main,
                                 args=(target, args.requests // k + (i < args.requests % k),
                                       args.concurrency // k + (i < args.concurrency % k), i + 1, q,
                                       ready, go))
                     for i in range(k)]
            [p.start() for p in procs]
            for _ in procs:
                ready.acquire()
            if pool is not None:  # counters from the common start on (not process spawn)
                time.sleep(2 * pool.hb_interval)
                rs0 = pool.health()
            go.set()
            lat, errors, starts, ends, fin = [], [], [], [], []
            for _ in procs:
                la, er, t_s, t_e, fi = q.get()
                lat += la
                errors += er
                fin += fi
                starts.append(t_s)
                ends.append(t_e)
            [p.join() for p in procs]
            t_s = min(starts)
            dt = max(ends) - t_s
        else:
            lat, errors, t_s, t_e, fin = run_load(target, args.requests, args.concurrency, 1)
            dt = t_e - t_s
        # steady-state service rate: completions in the 20-90 % part of the run (the
        # whole-run rate also counts the clients' ramp-up and the drain of the last batch)
        w0, w1 = t_s + 0.2 * dt, t_s + 0.9 * dt
        steady = sum(1 for f in fin if w0 <= f < w1) / (w1 - w0) if fin else None
        lat.sort()
        gen_tokens = (len(lat) * fp.smart.max_new_tokens) if args.backend != "scripted" else 0
        hist = METRICS.snapshot()["histograms"]
        tpot = hist.get("engine.tpot_s", {})
        out = {
            "metric": f"service smart-reply ({args.mode}) requests/s + latency" +
                      (f", open loop at {args.arrival_rate:g} req/s" if args.arrival_rate else ""),
            "load": (f"open-loop poisson {args.arrival_rate:g} req/s" if args.arrival_rate
                     else f"closed-loop, {args.concurrency} clients"),
            "p50_tpot_ms": round(1000 * tpot["p50"], 1) if "p50" in tpot else None,
            "p99_tpot_ms": round(1000 * tpot["p99"], 1) if "p99" in tpot else None,
            "backend": args.backend, "frontend": args.frontend, "model": args.model if args.backend != "scripted" else None,
            "client_procs": args.client_procs,
            "requests": len(lat), "errors": len(errors), "concurrency": args.concurrency, "seconds": round(dt, 3),
            "error_kinds": dict(collections.Counter(e.split(" (at ")[0] for e in errors).most_common(5)),
            "error_times_s": sorted(float(e.rsplit("(at ", 1)[1][:-3]) for e in errors)[:20],
            "requests_per_s": round(len(lat) / dt, 2),
            "gen_tokens_per_s": round(gen_tokens / dt, 1) if gen_tokens else None,
            "steady_requests_per_s": round(steady, 2) if steady else None,
            "steady_gen_tokens_per_s": (round(steady * fp.smart.max_new_tokens, 1)
                                        if steady and args.backend != "scripted" else None),
            "p50_latency_ms": round(1000 * statistics.median(lat), 1),
            "p99_latency_ms": round(1000 * lat[min(len(lat) - 1, int(0.99 * (len(lat) - 1)))], 1),
            "engine_stats": dict(eng.stats) if eng else None,
            # pool mode: the replicas' counters over the run (idle_ms: time the engine had no
            # request at all - the closed loop's per-wave turnaround)
            "replica_delta": _delta(rs0, pool) if pool is not None else None,
            "rpc_metrics": {k: v for k, v in METRICS.snapshot()["histograms"].items()
                            if "SmartReply" in k or k.startswith("engine.")},
        }
        print(json.dumps(out), flush=True)
    finally:
        if cluster is not None:
            cluster.stop()
        llm_srv.stop(0).wait(10)
        if hasattr(backend, "close"):
            backend.close()
        tmp.cleanup()


if __name__ == "__main__":
    main()
    sys.stdout.flush()
    sys.stderr.flush()
    # grpc's C++ core and the engine's graph pools are torn down by the OS:
    # interpreter finalisation with live grpc completion-queue threads can
    # std::terminate after the results are out.
    os._exit(0)
