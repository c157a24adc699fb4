#!/usr/bin/env python3
"""Write-path benchmark of the Raft chat cluster (CPU plane, no GPU).

The reference's most important request path is `send hello`: the client's
SendMessage goes to the leader, which appends a SEND_MESSAGE entry and (here) answers once a
majority has it.  This drives that path end to end:

  * 3 node processes (`python -m drtc_amd.server.node`) on ephemeral localhost ports, each
    with its own data directory (native CRC log, fsync group commit unless --no-fsync);
  * --clients client threads in --client-procs processes, each logged in as one of the seeded
    users, sending SendMessage RPCs to the leader back to back for --seconds;
  * reports committed writes/s and the p50 / p99 / max client-observed commit latency,
    then checks that every follower applied every acknowledged message.

usage: raft_write_bench.py [--clients 32] [--client-procs 4] [--seconds 10] [--no-fsync]
       [--local-commit]
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _spawn(i, port, peers, root, a):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    cmd = [sys.executable, "-m", "drtc_amd.server.node", "--node-id", str(i), "--port", str(port),
           "--peers", peers, "--data-root", root, "--llm", "", "--election-timeout", "0.4,0.8",
           "--heartbeat", "0.04", "--bcrypt-rounds", "4", "--log-level", "WARNING"]
    if not a.fsync:
        cmd.append("--no-fsync")
    if a.local_commit:
        cmd.append("--local-commit")
    return subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                            start_new_session=True)


def _leader(addrs, timeout=30.0):
    import grpc

    from drtc_amd.protos import RAFT_SERVICE, make_stub, raft_pb
    t_end = time.time() + timeout
    while time.time() < t_end:
        for i, ad in addrs.items():
            try:
                r = make_stub(grpc.insecure_channel(ad), RAFT_SERVICE).GetLeaderInfo(
                    raft_pb.GetLeaderRequest(), timeout=0.5)
                if r.is_leader:
                    return i
            except grpc.RpcError:
                pass
        time.sleep(0.1)
    raise TimeoutError("no leader")


def _client_proc(addr, token, n_threads, seconds, start_at, tag, out_q):
    import grpc

    from drtc_amd.protos import RAFT_SERVICE, make_stub, raft_pb
    lat, acked, errors = [], [], [0]
    lock = threading.Lock()

    def worker(t):
        stub = make_stub(grpc.insecure_channel(addr), RAFT_SERVICE)
        k = 0
        while time.time() < start_at:
            time.sleep(0.001)
        t_end = start_at + seconds
        while time.time() < t_end:
            rid = f"{tag}-{t}-{k}"
            k += 1
            t0 = time.perf_counter()
            try:
                r = stub.SendMessage(raft_pb.SendMessageRequest(
                    token=token, channel_id="general", content=rid, request_id=rid), timeout=10)
                ok = r.success
            except grpc.RpcError:
                ok = False
            dt = time.perf_counter() - t0
            with lock:
                if ok:
                    lat.append(dt)
                    acked.append(rid)
                else:
                    errors[0] += 1

    ts = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    out_q.put((lat, acked, errors[0]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--client-procs", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--no-fsync", dest="fsync", action="store_false", default=True)
    ap.add_argument("--local-commit", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import grpc

    from drtc_amd.protos import RAFT_SERVICE, make_stub, raft_pb
    from drtc_amd.utils.cluster import free_port

    root = tempfile.mkdtemp(prefix="raftbench_")
    ports = {i: free_port() for i in (1, 2, 3)}
    addrs = {i: f"127.0.0.1:{p}" for i, p in ports.items()}
    peers = ",".join(f"{i}={ad}" for i, ad in addrs.items())
    procs = {i: _spawn(i, ports[i], peers, root, a) for i in ports}
    try:
        L = _leader(addrs)
        stub = make_stub(grpc.insecure_channel(addrs[L]), RAFT_SERVICE)
        t_end = time.time() + 30
        while True:  # the default users arrive through the log right after the election
            r = stub.Login(raft_pb.LoginRequest(username="alice", password="alice123"), timeout=10)
            if r.success or time.time() > t_end:
                break
            time.sleep(0.1)
        assert r.success, "login failed"
        token = r.token
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        per = [a.clients // a.client_procs + (1 if p < a.clients % a.client_procs else 0)
               for p in range(a.client_procs)]
        start_at = time.time() + 3.0
        cps = [ctx.Process(target=_client_proc, args=(addrs[L], token, n, a.seconds, start_at,
                                                       f"p{p}", q))
               for p, n in enumerate(per) if n]
        for p in cps:
            p.start()
        res = [q.get(timeout=a.seconds + 120) for _ in cps]
        for p in cps:
            p.join(timeout=30)
        lat = sorted(x for r in res for x in r[0])
        acked = [x for r in res for x in r[1]]
        errors = sum(r[2] for r in res)

        def pct(v):
            return round(1000 * lat[min(len(lat) - 1, int(round(v * (len(lat) - 1))))], 2) if lat else None

        # every follower applied every acknowledged write (reads are served locally)
        want = set(acked)
        caught_up = {}
        for i, ad in addrs.items():
            st = make_stub(grpc.insecure_channel(ad), RAFT_SERVICE)
            t_end = time.time() + 30
            while True:
                m = st.GetMessages(raft_pb.GetMessagesRequest(token=token, channel_id="general",
                                                              limit=len(want) + 100), timeout=10)
                have = {x.content for x in m.messages}
                if want <= have or time.time() > t_end:
                    break
                time.sleep(0.2)
            caught_up[i] = want <= have
        out = {"metric": "raft SendMessage commits/s (3 nodes, localhost)",
               "writes_per_s": round(len(lat) / a.seconds, 1), "acked": len(acked),
               "errors": errors, "clients": a.clients, "client_procs": len(cps),
               "p50_ms": pct(0.5), "p99_ms": pct(0.99), "max_ms": pct(1.0),
               "fsync": a.fsync, "commit": "local (reference Q1)" if a.local_commit else "majority",
               "all_replicas_applied_every_ack": all(caught_up.values()), "leader": L,
               "cpus": os.cpu_count()}
        print(json.dumps(out), flush=True)
        if a.out:
            with open(a.out, "w") as f:
                json.dump(out, f, indent=1)
    finally:
        for p in procs.values():
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        for p in procs.values():
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
