#!/usr/bin/env python3
"""Headline benchmark: smart-reply serving throughput on MI355X.

Metric (BASELINE.json): "smart-reply tokens/sec (whole node) + p50 suggestion
latency, Llama-3-8B TP=1".

Workload per GPU (one engine replica per GPU, DP over the node = weak
scaling): each timed *step* serves ``--batch`` smart-reply requests end to
end through the continuous-batching engine - tokenization of the reference's
smart-reply prompt over a synthetic 5-message channel history, one packed
varlen prefill, then hipGraph-replayed decode steps until every request has
produced ``--max-new-tokens`` tokens (EOS ignored: random-init weights never
stop on their own; the reference's contract is 3 lines of < 10 words).
Sampling uses the hosted backend's defaults (temperature 1.0, top-k 64,
top-p 0.95) through the fused HIP sampler.

``value`` = generated tokens / s over all ranks (max wall time over ranks);
``p50_latency_ms`` = median request latency (arrival -> last token).

Launch: ``python bench.py`` (1 GPU); ``python bench.py --gpus N`` starts N rank
processes itself (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their
environment, RCCL) before the parent touches the GPU, prints rank 0's JSON line
and exits non-zero if any rank fails; under torchrun (WORLD_SIZE set) the ranks
are torchrun's and WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from drtc_amd.engine import ChatTokenizer, LLMEngine, Request, SamplingParams  # noqa: E402
from drtc_amd.engine.engine import freeze_gc  # noqa: E402
from drtc_amd.llm import prompts as P  # noqa: E402
from drtc_amd.llm.service import FeatureParams  # noqa: E402
from drtc_amd.models import TransformerLM, get_config  # noqa: E402
from drtc_amd.parallel import init_distributed  # noqa: E402
from drtc_amd.utils.synthetic import channel_history  # noqa: E402

METRIC = "smart-reply tokens/sec (whole node) + p50 suggestion latency, Llama-3-8B TP=1"

# workload -> (history messages per request, prompt builder, FeatureParams attribute)
WORKLOADS = {
    "smart_reply": (5, lambda h, rng: P.smart_reply_prompt(h), "smart"),
    "summarize": (20, lambda h, rng: P.summarize_prompt(h, 200), "summary"),
    "suggest": (5, lambda h, rng: P.suggestions_prompt(h, rng.choice(["I think", "maybe we", "sure"])),
                "suggest"),
    "ask": (5, lambda h, rng: P.answer_prompt(rng.choice(h).content + "?", [m.content for m in h]),
            "answer"),
}


def log(rank: int, *a) -> None:
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))] if xs else 0.0


def open_loop(args, eng, make_prompts, params, rank, world, tp, device, cfg) -> None:
    """Open-loop serving: requests arrive as a Poisson process at
    ``--arrival-rate`` req/s (per replica) whatever the engine's progress, the
    way chat users issue smart-reply RPCs; latency counts from the SCHEDULED
    arrival, so queueing behind a busy step is included.  Reports p50/p99 of
    end-to-end latency, TTFT and TPOT (time per output token after the first)."""
    import random

    rate = args.arrival_rate
    n_req = args.requests or int(rate * 20)
    prompts = []
    s = 0
    while len(prompts) < n_req:
        prompts += make_prompts(1000 + s)
        s += 1
    prompts = prompts[:n_req]
    rng = random.Random(17 + rank)
    arr, t = [], 0.0
    for _ in range(n_req):
        t += rng.expovariate(rate)
        arr.append(t)
    eng.stats.clear()
    if world > 1:
        dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    reqs, i = [], 0
    t0 = time.perf_counter()
    while i < n_req or eng.has_work():
        now = time.perf_counter() - t0
        while i < n_req and arr[i] <= now:
            r = Request(prompts[i], params)
            r.arrival_time = t0 + arr[i]
            reqs.append(eng.add_request(r))
            i += 1
        if eng.has_work():
            eng.step()
        elif i < n_req:
            time.sleep(min(0.002, max(0.0, arr[i] - now)))
    if device.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    lat = [r.latency for r in reqs]
    ttft = [r.ttft for r in reqs]
    tpot = [(r.finish_time - r.first_token_time) / (len(r.output_ids) - 1)
            for r in reqs if len(r.output_ids) > 1]
    gen = sum(len(r.output_ids) for r in reqs)
    # service rate in the steady part of the arrival window (30-90 % of it): the
    # whole-run rate above also counts the ramp-up and the drain after the last
    # arrival, so under overload it understates what the engine sustains
    w0, w1 = t0 + 0.3 * arr[-1], t0 + 0.9 * arr[-1]
    fin = [r for r in reqs if w0 <= r.finish_time < w1]
    st = torch.tensor([elapsed, gen, _pct(lat, .5), _pct(lat, .99), _pct(ttft, .5),
                       _pct(ttft, .99), _pct(tpot, .5), _pct(tpot, .99)], dtype=torch.float64,
                      device=device)
    steady = torch.tensor([len(fin) / (w1 - w0), sum(len(r.output_ids) for r in fin) / (w1 - w0)],
                          dtype=torch.float64, device=device)
    if world > 1:
        g = st[1].clone()
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        if tp == 1:
            dist.all_reduce(g)
            dist.all_reduce(steady)
        st[1] = g
    el, gen = float(st[0]), float(st[1])
    if rank == 0:
        ms = [round(1000 * float(v), 1) for v in st[2:]]
        print(json.dumps({
            "metric": f"{args.workload} open-loop latency at {rate:g} req/s per replica, "
                      f"{cfg.name} TP={tp}",
            "mode": "open-loop", "arrival": "poisson", "arrival_rate_per_replica": rate,
            "n_gpus": world, "requests_per_replica": n_req,
            "achieved_req_per_s": round(n_req * (world // tp) / el, 1),
            "gen_tokens_per_s": round(gen / el, 1),
            "steady_req_per_s": round(float(steady[0]), 1),
            "steady_gen_tokens_per_s": round(float(steady[1]), 1),
            "p50_latency_ms": ms[0], "p99_latency_ms": ms[1],
            "p50_ttft_ms": ms[2], "p99_ttft_ms": ms[3],
            "p50_tpot_ms": ms[4], "p99_tpot_ms": ms[5],
            "p99_over_p50_tpot": round(ms[5] / max(ms[4], 1e-9), 2),
            "scheduler": ("mixed, %d prompt tokens/step" % eng.mixed_tokens) if eng.mixed
            else "prefill-first",
            "max_new_tokens": params.max_new_tokens, "dtype": "bf16",
            "data": "synthetic chat logs, random-init weights",
            "engine_stats": dict(eng.stats)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n: int) -> int:
    """Run this script as ``n`` rank processes (no torchrun in the parent, no GPU call
    in the parent: children are started with subprocess, never exec).  Rank 0's
    stdout (the JSON line) is forwarded; every rank's stderr goes to ours.  When a
    rank fails the others are stopped and its exit status is returned."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                      env=env, stdout=subprocess.PIPE if r == 0 else
                                      subprocess.DEVNULL))
    rc = 0
    try:
        while True:
            alive = [p for p in procs if p.poll() is None]
            bad = [p for p in procs if p.poll() not in (None, 0)]
            if bad:
                rc = bad[0].returncode
                break
            if not alive:
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    out = procs[0].stdout.read().decode() if procs[0].stdout else ""
    sys.stdout.write(out)
    sys.stdout.flush()
    return rc if rc else (0 if any(ln.startswith("{") for ln in out.splitlines()) else 1)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch", type=int, default=1024, help="requests per GPU per step")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="smart_reply")
    ap.add_argument("--max-new-tokens", type=int, default=None,
                    help="default: the feature's output budget (smart reply 48)")
    ap.add_argument("--history", type=int, default=None)
    ap.add_argument("--greedy", action="store_true")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--max-model-len", type=int, default=2048)
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (= WORLD_SIZE)")
    ap.add_argument("--trace", default=None, metavar="PATH",
                    help="record engine/graph spans (roctx + Chrome trace JSON at PATH)")
    ap.add_argument("--kv-fraction", type=float, default=0.85,
                    help="fraction of the free HBM (after weights) given to the paged KV cache")
    ap.add_argument("--custom-allreduce", dest="custom_allreduce", action="store_true",
                    default=True,
                    help="TP: one-shot IPC all-reduce (fused with the residual add + RMSNorm) "
                         "for decode-sized messages, RCCL above the size threshold (default)")
    ap.add_argument("--rccl-only", dest="custom_allreduce", action="store_false",
                    help="TP: every all-reduce on RCCL")
    ap.add_argument("--arrival-rate", type=float, default=0.0, metavar="REQ_PER_S",
                    help="open-loop mode: Poisson arrivals at this rate per replica; reports "
                         "p50/p99 latency, TTFT and TPOT instead of the closed-wave headline")
    ap.add_argument("--requests", type=int, default=0,
                    help="open-loop: requests per replica (default: 20 s of arrivals)")
    ap.add_argument("--mixed-tokens", type=int, default=None,
                    help="prompt-token budget of a mixed prefill+decode step")
    ap.add_argument("--no-mixed", action="store_true", help="strict prefill-first scheduling")
    args = ap.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(self_launch(args.gpus))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE {os.environ.get('WORLD_SIZE')}",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if args.trace:
        from drtc_amd.utils import tracing
        tracing.enable(True)

    rank, world = init_distributed()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        local %= torch.cuda.device_count()  # several ranks per GPU only in rehearsals
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")

    # self-verification of the multi-GPU run: which device every rank drives, over which
    # collective backend, in a communicator of how many ranks.  Under nccl (RCCL) every rank
    # must own a distinct GPU; rehearsals that time-share one GPU run on gloo.
    backend = dist.get_backend() if world > 1 else "none"
    rccl_world = dist.get_world_size() if world > 1 else 1
    devices = [device.index if device.type == "cuda" else -1]
    if world > 1:
        devices = [None] * world
        dist.all_gather_object(devices, device.index if device.type == "cuda" else -1)
        if backend == "nccl" and len(set(devices)) != world:
            log(rank, f"error: ranks share a GPU under nccl: devices {devices}")
            sys.exit(3)

    cfg = get_config(args.model)
    t0 = time.perf_counter()
    tp = args.tp
    if tp > 1:
        assert tp == world, "--tp must equal WORLD_SIZE (one TP group per node)"
        from drtc_amd.parallel import ParallelContext
        pc = ParallelContext.from_world(tp=True, ep=cfg.is_moe)
        if args.custom_allreduce:
            pc.enable_custom_allreduce()
    else:
        pc = None
    dp_rank = 0 if tp > 1 else rank
    model = TransformerLM(cfg, device, pc=pc, seed=1234, full_then_shard=False)
    eng = LLMEngine(model, max_batch=args.batch, max_model_len=args.max_model_len,
                    max_prefill_tokens=max(16384, args.batch * 400),
                    kv_fraction=args.kv_fraction, use_graphs=not args.no_graphs, seed=dp_rank)
    if args.no_mixed:
        eng.mixed = False
    if args.mixed_tokens:
        eng.mixed_tokens = args.mixed_tokens
    if world > 1:
        dist.barrier()  # TP: the custom all-reduce's flag waits are time-bounded
    eng.warmup(capture=True)
    if device.type == "cuda":
        torch.cuda.synchronize()
    log(rank, f"model {cfg.name} {model.weight_bytes() / 1e9:.1f} GB, kv {eng.kv.bytes / 1e9:.1f} GB "
              f"({eng.kv.capacity_tokens} tokens), init {time.perf_counter() - t0:.1f}s")

    tok = ChatTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_id)
    n_hist, build, feat = WORKLOADS[args.workload]
    n_hist = args.history or n_hist
    params = getattr(FeatureParams(ignore_eos=True), feat)
    if args.max_new_tokens:
        params.max_new_tokens = args.max_new_tokens
    if args.greedy:
        params = SamplingParams.greedy(params.max_new_tokens, ignore_eos=True)
    args.max_new_tokens = params.max_new_tokens

    def make_prompts(step: int) -> list[list[int]]:
        import random
        rng = random.Random(dp_rank * 100003 + step)
        return [tok.encode(build(channel_history(rng, n_hist), rng)) for _ in range(args.batch)]

    def serve(prompts):
        reqs = [eng.add_request(Request(p, params)) for p in prompts]
        while eng.has_work():
            eng.step()
        return reqs

    for w in range(args.warmup):
        serve(make_prompts(-1 - w))
    if args.arrival_rate > 0:
        freeze_gc()
        open_loop(args, eng, make_prompts, params, rank, world, tp, device, cfg)
        return
    prompts = [make_prompts(s) for s in range(args.steps)]
    prompt_tokens = sum(len(p) for ps in prompts for p in ps)
    freeze_gc()  # as a serving process after warm-up (DRTC_GC_FREEZE=0: off)

    if world > 1:
        dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t_start = time.perf_counter()
    lat, r_ttft, gen = [], [], 0
    for s in range(args.steps):
        reqs = serve(prompts[s])
        lat.extend(r.latency for r in reqs)
        r_ttft.extend(r.ttft for r in reqs)
        gen += sum(len(r.output_ids) for r in reqs)
    if device.type == "cuda":
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start

    p50 = statistics.median(lat)
    p99 = sorted(lat)[min(len(lat) - 1, int(round(0.99 * (len(lat) - 1))))]
    ttft50 = statistics.median(r_ttft)
    stats = torch.tensor([elapsed, float(gen), float(prompt_tokens), p50, p99, ttft50],
                         dtype=torch.float64,
                         device=device)
    if world > 1:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, p50, p99, ttft50 = float(mx[0]), float(mx[3]), float(mx[4]), float(mx[5])
        if tp == 1:  # DP replicas serve different requests; TP ranks serve the same ones
            gen, prompt_tokens = float(sm[1]), float(sm[2])
    tps = gen / elapsed
    if rank == 0:
        out = {
            "metric": METRIC if (args.workload, args.model, tp) == ("smart_reply", "llama-3-8b", 1) else
            f"{args.workload} tokens/sec (whole node) + p50 latency, {cfg.name} TP={tp}",
            "value": round(tps, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 2),
            "higher_is_better": True,
            "scaling": "strong" if tp > 1 else "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": f"synthetic chat logs ({n_hist}-message {args.workload} contexts), random-init weights",
            "config": {"model": cfg.name, "global_batch": args.batch * (world // tp),
                       # tokens per sequence: the average prompt plus the generated tokens
                       "seq_len": round(prompt_tokens / (args.batch * (world // tp) * args.steps)
                                        + args.max_new_tokens),
                       "parallelism": f"tp{tp}" if tp > 1 else f"dp{world}",
                       "max_new_tokens": args.max_new_tokens,
                       "avg_prompt_tokens": round(prompt_tokens / (args.batch * (world // tp) * args.steps), 1),
                       "sampling": "greedy" if args.greedy else
                       f"t={params.temperature},top_k={params.top_k},top_p={params.top_p}",
                       "graphs": not args.no_graphs},
            "devices": devices,
            "backend": backend,
            "rccl_world": rccl_world,
            "p50_latency_ms": round(1000 * p50, 1),
            "p99_latency_ms": round(1000 * p99, 1),
            "p50_ttft_ms": round(1000 * ttft50, 1),
            "total_tokens_per_s": round((gen + prompt_tokens) / elapsed, 1),
            "engine_stats": dict(eng.stats),
        }
        print(json.dumps(out), flush=True)
        if eng.runner.gpu_ms:
            g = sorted(eng.runner.gpu_ms)
            log(rank, f"decode graph GPU time: median {g[len(g) // 2]:.3f} ms over {len(g)} steps")
        if args.trace:
            from drtc_amd.utils import tracing
            n = tracing.dump_chrome_trace(args.trace)
            log(rank, f"wrote {n} trace spans to {args.trace}")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
