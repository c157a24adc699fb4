"""Raft safety/liveness under fault injection (deterministic simulator)."""
import pytest

from drtc_amd.raft.core import (AppendReq, AppendResp, Entry, NotLeaderError, RaftConfig, RaftCore,
                                Role, VoteReq)
from drtc_amd.raft.sim import SimCluster


def _check_log_matching(c: SimCluster):
    """Absolute-index log matching over the entries both nodes still hold
    (compaction drops committed prefixes)."""
    nodes = list(c.nodes.values())
    for a in nodes:
        for b in nodes:
            lo = max(a.first_index, b.first_index)
            hi = min(a.last_index, b.last_index)
            for i in range(hi, lo - 1, -1):
                if a.term_at(i) == b.term_at(i):
                    assert all(a.entry(j) == b.entry(j) for j in range(lo, i + 1)), \
                        "log matching violated"
                    break


def _check_state_machine_safety(c: SimCluster):
    seqs = [[(i, e) for i, e in c.applied[n]] for n in c.nodes]
    for s1 in seqs:
        for s2 in seqs:
            n = min(len(s1), len(s2))
            assert s1[:n] == s2[:n], "two nodes applied different entries at the same index"


def test_single_leader_elected():
    c = SimCluster(3, seed=1)
    l = c.wait_leader()
    c.run(1.0)
    assert c.leader() == l
    for t, ls in c.leaders_by_term.items():
        assert len(ls) == 1, f"two leaders in term {t}"


def test_single_node_cluster_commits_immediately():
    core = RaftCore(1, [], config=RaftConfig(election_timeout=(0.1, 0.2)))
    core.tick(1.0)
    assert core.is_leader()
    idx, _ = core.propose("SEND_MESSAGE", b"{}")
    assert core.commit_index == idx and core.last_applied == idx


def test_replication_and_commit():
    c = SimCluster(3, seed=2)
    c.wait_leader()
    for k in range(20):
        c.propose("SEND_MESSAGE", str(k).encode())
    c.run(1.0)
    for i in c.nodes:
        assert len(c.committed_commands(i)) == 20
    _check_log_matching(c)
    _check_state_machine_safety(c)


def test_leader_crash_failover_keeps_committed_entries():
    c = SimCluster(5, seed=3)
    l = c.wait_leader()
    for k in range(10):
        c.propose("SEND_DM", str(k).encode())
    c.run(0.5)
    c.crash(l)
    l2 = c.wait_leader()
    assert l2 != l
    c.propose("SEND_DM", b"after")
    c.run(1.0)
    for i in c.nodes:
        if i != l:
            cmds = c.committed_commands(i)
            assert len(cmds) == 11
    c.restart(l)
    c.run(2.0)
    assert len(c.committed_commands(l)) == 11
    _check_log_matching(c)
    _check_state_machine_safety(c)


@pytest.mark.parametrize("seed", range(8))
def test_safety_under_loss_dup_and_partitions(seed):
    c = SimCluster(5, seed=seed, drop=0.15, dup=0.1, delay=(0.001, 0.04))
    c.wait_leader(30)
    proposed = 0
    for rnd in range(12):
        if rnd % 4 == 1:
            ids = sorted(c.nodes)
            c.partition = [set(ids[:2]), set(ids[2:])]
        if rnd % 4 == 3:
            c.partition = None
        for _ in range(3):
            try:
                c.propose("SEND_MESSAGE", f"{rnd}".encode())
                proposed += 1
            except (RuntimeError, NotLeaderError):
                pass
        c.run(0.4)
    c.partition = None
    c.drop = 0.0
    c.run(5.0)
    for t, ls in c.leaders_by_term.items():
        assert len(ls) == 1, f"two leaders in term {t}"
    _check_log_matching(c)
    _check_state_machine_safety(c)
    commits = {len(c.applied[i]) for i in c.nodes}
    assert len(commits) == 1  # converged after healing


def test_stale_append_does_not_truncate_newer_entries():
    """Quirk Q4 regression: an old AppendEntries that overlaps entries the
    follower already has must not delete the suffix."""
    f = RaftCore(2, [1, 3])
    e = [Entry(1, "A", b""), Entry(1, "B", b""), Entry(1, "C", b"")]
    assert f.on_append_entries(AppendReq(1, 1, -1, 0, e, -1)).success
    assert len(f.log) == 3
    stale = AppendReq(1, 1, -1, 0, e[:1], -1)  # reordered, older RPC
    assert f.on_append_entries(stale).success
    assert [x.command for x in f.log] == ["A", "B", "C"]
    # a real conflict still truncates
    assert f.on_append_entries(AppendReq(2, 1, 0, 1, [Entry(2, "X", b"")], -1)).success
    assert [x.command for x in f.log] == ["A", "X"]


def test_vote_rules():
    n = RaftCore(1, [2, 3])
    n.log = [Entry(1, "A", b""), Entry(2, "B", b"")]
    # candidate with an older last term is refused
    assert not n.on_request_vote(VoteReq(3, 2, 5, 1)).vote_granted
    assert n.term == 3
    # up-to-date candidate is granted, then a second candidate in the same term refused
    assert n.on_request_vote(VoteReq(3, 2, 1, 2)).vote_granted
    assert not n.on_request_vote(VoteReq(3, 3, 1, 2)).vote_granted
    # stale term refused
    assert not n.on_request_vote(VoteReq(2, 3, 9, 9)).vote_granted


def test_commit_requires_current_term_entry():
    """A leader never counts replicas to commit an entry from an older term."""
    l = RaftCore(1, [2, 3, 4, 5], config=RaftConfig(leader_noop=False))
    l.log = [Entry(1, "OLD", b"")]
    l.term = 2
    l.role = Role.LEADER
    l.leader_id = 1
    for p in l.peers:
        l.next_index[p] = 1
        l.match_index[p] = -1
    req = AppendReq(2, 1, -1, 0, [l.log[0]], -1)
    l.on_append_reply(2, req, AppendResp(2, True))
    l.on_append_reply(3, req, AppendResp(2, True))
    assert l.commit_index == -1
    l.propose("NEW", b"")
    req2 = AppendReq(2, 1, 0, 1, [l.log[1]], -1)
    l.on_append_reply(2, req2, AppendResp(2, True))
    l.on_append_reply(3, req2, AppendResp(2, True))
    assert l.commit_index == 1


def test_local_commit_mode_reference_behaviour():
    c = SimCluster(3, seed=4, config=RaftConfig(election_timeout=(0.15, 0.3), heartbeat_interval=0.02,
                                                 local_commit=True, rpc_timeout_append=0.1))
    l = c.wait_leader()
    c.partition = [{l}, set(c.nodes) - {l}]
    idx, _ = c.propose("SEND_MESSAGE", b"x")
    assert c.nodes[l].commit_index >= idx  # acknowledged without a majority (quirk Q1)


def test_follower_catch_up_after_long_partition():
    c = SimCluster(3, seed=6)
    l = c.wait_leader()
    lagger = next(i for i in c.nodes if i != l)
    c.partition = [set(c.nodes) - {lagger}, {lagger}]
    for k in range(300):
        c.propose("SEND_MESSAGE", str(k).encode())
    c.run(0.5)
    c.partition = None
    c.run(3.0)
    assert len(c.committed_commands(lagger)) == 300


# ------------------------------------------------------------ compaction
def test_compaction_and_install_snapshot_to_lagging_follower():
    c = SimCluster(3, seed=11)
    l = c.wait_leader()
    lag = next(i for i in c.nodes if i != l)
    c.crash(lag)
    for k in range(60):
        c.propose("SEND_MESSAGE", str(k).encode())
    c.run(1.0)
    for i in c.nodes:
        if i != lag:
            assert c.compact(i)
            assert c.nodes[i].snap_index >= 60 and len(c.nodes[i].log) == 0
    for k in range(60, 70):
        c.propose("SEND_MESSAGE", str(k).encode())
    c.restart(lag)
    c.run(2.0)
    ref = c.committed_commands(l)
    assert len(ref) == 70
    assert c.committed_commands(lag) == ref  # caught up through InstallSnapshot
    assert c.nodes[lag].snap_index >= 60
    _check_log_matching(c)
    _check_state_machine_safety(c)


def test_restart_after_compaction_restores_snapshot_then_replays():
    c = SimCluster(3, seed=12)
    c.wait_leader()
    for k in range(30):
        c.propose("SEND_MESSAGE", str(k).encode())
    c.run(1.0)
    node = next(iter(c.nodes))
    assert c.compact(node)
    for k in range(30, 40):
        c.propose("SEND_MESSAGE", str(k).encode())
    c.run(1.0)
    before = c.committed_commands(node)
    c.crash(node)
    c.restart(node)
    c.run(1.0)
    assert c.committed_commands(node)[:len(before)] == before
    assert len(c.committed_commands(node)) == 40


@pytest.mark.parametrize("seed", [21, 22, 23])
def test_safety_with_periodic_compaction_under_faults(seed):
    c = SimCluster(5, seed=seed, drop=0.1, dup=0.05)
    c.wait_leader()
    sent = 0
    for rnd in range(12):
        for _ in range(8):
            try:
                c.propose("SEND_MESSAGE", str(sent).encode())
                sent += 1
            except (RuntimeError, NotLeaderError):
                pass
        if rnd % 3 == 1:
            victim = 1 + rnd % 5
            c.crash(victim)
        if rnd % 3 == 2:
            for i in list(c.down):
                c.restart(i)
        for i in c.nodes:
            if i not in c.down and c.nodes[i].last_applied - c.nodes[i].snap_index > 10:
                c.compact(i)
        c.run(0.5)
    for i in list(c.down):
        c.restart(i)
    c.run(3.0)
    _check_log_matching(c)
    _check_state_machine_safety(c)
    for t, ls in c.leaders_by_term.items():
        assert len(ls) == 1
    lens = {len(c.committed_commands(i)) for i in c.nodes}
    assert len(lens) == 1  # everyone converged
