#!/usr/bin/env python3
"""Leader election and failover timing of the 3-node Raft cluster on localhost (CPU plane),
against the reference's derived 13.5-18.7 s election / 11.5-18.7 s failover
(ref server/raft_node.py:469-471,522,629-630,948-949).

Per trial: start a fresh in-process cluster and time start -> a leader with the genesis
entries applied; then kill the leader and time kill -> a new leader that commits a write
(SendMessage through it succeeds).  Default timeouts (RaftConfig: 1.5-3 s election) and the
test timeouts (0.3-0.6 s) are both reported.  One JSON line.

  python scripts/election_bench.py --trials 5
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from drtc_amd.raft.core import RaftConfig  # noqa: E402
from drtc_amd.utils.cluster import LocalCluster  # noqa: E402


def trial(raft: RaftConfig) -> tuple[float, float]:
    with tempfile.TemporaryDirectory() as root:
        c = LocalCluster(3, data_root=root, raft=raft)
        t0 = time.time()
        c.start()
        try:
            lead = c.leader(timeout=60)
            t_elect = time.time() - t0
            token = c.login(lead)
            t1 = time.time()
            c.kill(lead)
            # a new leader, which has committed an entry of its own term (its NOOP)
            while True:
                ls = [i for i, n in c.nodes.items() if n.rt.is_leader()]
                if ls:
                    core = c.nodes[ls[0]].rt.core
                    ci = core.commit_index
                    if ci >= 0 and core.term_at(ci) == core.term:
                        break
                if time.time() - t1 > 60:
                    raise TimeoutError("no new leader")
                time.sleep(0.005)
            t_fail = time.time() - t1
            del token
            return t_elect, t_fail
        finally:
            c.stop()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=5)
    a = ap.parse_args()
    out = {"metric": "raft leader election / failover (3 nodes, localhost)", "trials": a.trials}
    for name, cfg in (("default", RaftConfig()),
                      ("fast", RaftConfig(election_timeout=(0.3, 0.6), heartbeat_interval=0.03))):
        el, fo = zip(*(trial(cfg) for _ in range(a.trials)))
        out[name] = {"election_timeout_s": list(cfg.election_timeout),
                     "election_s_p50": round(statistics.median(el), 3),
                     "election_s_max": round(max(el), 3),
                     "failover_s_p50": round(statistics.median(fo), 3),
                     "failover_s_max": round(max(fo), 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
