#!/usr/bin/env python3
"""Two engine groups of different real-size models on ONE MI355X behind one LLM service
(``llm.server --serve smart=gemma-2b@0:mem=A --serve summary=llama-3-8b@0:mem=B``), under
concurrent load of both features.

Each group runs in its own engine process (WorkerPool) with an explicit HBM budget; the
answer / suggest features share the summary group here.  Closed-loop gRPC clients issue smart replies (5 recent messages,
48 new tokens) and summaries (20 messages, 128 new tokens) at once; the JSON line reports per
feature requests, tok/s, p50 / p99 latency against the reference's node -> LLM deadlines (20 s
smart reply, 10 s summarize: ref server/raft_node.py:2018, :2084) and each group's KV split
(blocks, cached tokens, GB, budget) from its replica heartbeats.

  python scripts/colocate_bench.py --smart-mem 0.3 --summary-mem 0.6
"""
import argparse
import json
import os
import random
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import grpc  # noqa: E402

from drtc_amd.llm import server as S  # noqa: E402
from drtc_amd.llm.service import FeatureParams  # noqa: E402
from drtc_amd.protos import LLM_SERVICE, llm_pb, make_stub  # noqa: E402
from drtc_amd.utils.cluster import free_port  # noqa: E402
from drtc_amd.utils.synthetic import channel_history  # noqa: E402


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(q * (len(xs) - 1))))] if xs else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--smart-model", default="gemma-2b")
    ap.add_argument("--summary-model", default="llama-3-8b")
    ap.add_argument("--smart-mem", type=float, default=0.3)
    ap.add_argument("--summary-mem", type=float, default=0.6)
    ap.add_argument("--smart-batch", type=int, default=1024)
    ap.add_argument("--summary-batch", type=int, default=256)
    ap.add_argument("--smart-clients", type=int, default=512)
    ap.add_argument("--summary-clients", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=40.0, help="load duration")
    a = ap.parse_args()

    args = argparse.Namespace(backend="engine", model=a.summary_model, tp=1, gpus=1,
                              max_batch=0, max_model_len=2048, no_graphs=False,
                              custom_allreduce=False, in_process=False, hbm_budget=None)
    specs = [f"smart={a.smart_model}@0:mem={a.smart_mem}",
             f"summary={a.summary_model}@0:mem={a.summary_mem}",
             f"answer={a.summary_model}@0:mem={a.summary_mem}",
             f"suggest={a.summary_model}@0:mem={a.summary_mem}"]
    # per-group batches: the smart group at its knee, the summary group sized for 10 s
    bat = {a.smart_model: a.smart_batch, a.summary_model: a.summary_batch}
    orig = S.default_max_batch
    S.default_max_batch = lambda m, tp=1: bat.get(m, orig(m, tp))
    t0 = time.time()
    router = S.build_feature_backends(args, specs)
    S.default_max_batch = orig
    print(f"[colocate] groups up in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    fp = FeatureParams(ignore_eos=True)  # full token budgets (random weights never stop)
    port = free_port()
    srv = S.serve(router, port=port, bind="127.0.0.1", params=fp,
                  workers=a.smart_clients + a.summary_clients + 16)
    target = f"127.0.0.1:{port}"
    stop = threading.Event()
    res = {"smart": [], "summary": []}
    errs = {"smart": 0, "summary": 0}
    lock = threading.Lock()

    def client(feature, k):
        stub = make_stub(grpc.insecure_channel(target), LLM_SERVICE)
        rng = random.Random(k * 7 + (1 if feature == "summary" else 0))
        i = 0
        while not stop.is_set():
            i += 1
            hist = channel_history(rng, 20 if feature == "summary" else 5)
            msgs = [llm_pb.Message(sender=m.sender, content=m.content) for m in hist]
            t = time.perf_counter()
            try:
                if feature == "smart":
                    r = stub.GetSmartReply(llm_pb.SmartReplyRequest(
                        request_id=f"s{k}.{i}", recent_messages=msgs), timeout=60)
                    ok = len(r.suggestions) > 0
                else:
                    r = stub.SummarizeConversation(llm_pb.SummarizeRequest(
                        request_id=f"m{k}.{i}", messages=msgs, max_length=200), timeout=60)
                    ok = bool(r.summary)
            except grpc.RpcError:
                ok = False
            dt = time.perf_counter() - t
            with lock:
                if ok and not stop.is_set():
                    res[feature].append(dt)
                elif not ok:
                    errs[feature] += 1

    threads = [threading.Thread(target=client, args=("smart", k), daemon=True)
               for k in range(a.smart_clients)]
    threads += [threading.Thread(target=client, args=("summary", k), daemon=True)
                for k in range(a.summary_clients)]
    for t in threads:
        t.start()
    time.sleep(a.seconds)
    stop.set()
    t_end = a.seconds
    for t in threads:
        t.join(timeout=70)
    tokens = {"smart": fp.smart.max_new_tokens, "summary": fp.summary.max_new_tokens}
    deadline = {"smart": 20.0, "summary": 10.0}
    out = {"metric": "co-located engine groups on one MI355X", "features": {}, "groups": {}}
    for f, lat in res.items():
        out["features"][f] = dict(
            model=a.smart_model if f == "smart" else a.summary_model, requests=len(lat),
            errors=errs[f], tok_s=round(len(lat) * tokens[f] / t_end, 1),
            p50_s=round(pct(lat, 0.5), 3) if lat else None,
            p99_s=round(pct(lat, 0.99), 3) if lat else None, deadline_s=deadline[f],
            within_deadline=bool(lat) and pct(lat, 0.99) < deadline[f])
    for f in ("smart", "summary"):
        be = router.route(f)
        pool = getattr(be, "pool", None)
        if pool is not None:
            h = pool.health()[0]
            out["groups"][f] = {k: h.get(k) for k in ("device", "kv_blocks", "kv_tokens",
                                                      "kv_gb", "hbm_budget", "healthy")}
    print(json.dumps(out), flush=True)
    srv.stop(0)
    router.close()


if __name__ == "__main__":
    main()
