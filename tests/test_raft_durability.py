"""Raft wire/disk interoperability and crash safety.

* The exported reference-format pair (raft_log_port_*.pkl + raft_state_port_*.pkl)
  replays, with the reference's apply semantics (ref server/raft_node.py:1196-1397,
  re-implemented here as an oracle: json-decode every entry, dispatch on the
  command, skip unknown commands), to the same chat state the node holds - the
  leader NOOP and REVOKE_TOKEN entries included.
* The pair on disk never claims a commit beyond the log it holds.
* Default users/channels come from genesis log entries: channels.pkl / users.pkl
  are byte-identical on every replica.
* Logout is replicated; a write retried with the same request_id is applied once.
* Three node PROCESSES: SIGKILL the leader in the middle of a write stream,
  restart it from disk; no acknowledged write is lost anywhere.
"""
import json
import os
import signal
import subprocess
import sys
import time

import grpc
import pytest

from drtc_amd.protos import RAFT_SERVICE, make_stub, raft_pb
from drtc_amd.raft.core import Entry
from drtc_amd.raft.state_machine import ChatState
from drtc_amd.raft.storage import NativeStorage
from drtc_amd.server.raft_service import ChatNode
from drtc_amd.utils import pickle_compat
from drtc_amd.utils.cluster import LocalCluster, free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- reference oracle
def reference_replay(log_entries, commit_index):
    """Apply entries 0..commit_index with the reference's semantics."""
    users, users_by_id, channels, msgs, dms, files = {}, {}, {}, {}, [], {}
    for i in range(commit_index + 1):
        e = log_entries[i]
        data = json.loads(e["data"].decode("utf-8"))  # the reference decodes EVERY entry
        cmd = e["command"]
        if cmd == "CREATE_USER":
            if data["username"] not in users:
                users[data["username"]] = {"id": data["user_id"],
                                           "password": data["password"].encode("latin1")}
                users_by_id[data["user_id"]] = data["username"]
        elif cmd == "CREATE_CHANNEL":
            if data["channel_id"] not in channels:
                channels[data["channel_id"]] = {"name": data["name"], "members": set(data["members"]),
                                                "admins": set(data["admins"])}
                msgs.setdefault(data["channel_id"], [])
        elif cmd == "JOIN_CHANNEL":
            if data["channel_id"] in channels:
                channels[data["channel_id"]]["members"].add(data["user_id"])
        elif cmd == "LEAVE_CHANNEL":
            if data["channel_id"] in channels:
                channels[data["channel_id"]]["members"].discard(data["user_id"])
        elif cmd == "SEND_MESSAGE":
            lst = msgs.setdefault(data["channel_id"], [])
            if all(m.get("id") != data.get("id") for m in lst):
                lst.append(data)
        elif cmd == "SEND_DM":
            if all(d.get("id") != data.get("id") for d in dms):
                dms.append(data)
        elif cmd == "UPLOAD_FILE":
            files.setdefault(data["file_id"], bytes.fromhex(data["data"]))
        # anything else (NOOP, REVOKE_TOKEN, LOGIN_USER...) is logged and skipped
    return users, channels, msgs, dms, files


def _node_view(st):
    users = {n: {"id": u["id"], "password": u["password"]} for n, u in st.users.items()}
    chans = {cid: {"name": c["name"], "members": set(c["members"]), "admins": set(c["admins"])}
             for cid, c in st.channels.items()}
    files = {fid: f["data"] for fid, f in st.files.items()}
    return users, chans, st.channel_messages, st.direct_messages, files


@pytest.fixture
def cluster(tmp_path):
    c = LocalCluster(3, data_root=str(tmp_path)).start()
    yield c
    c.stop()


def _workload(cluster):
    L = cluster.leader()
    s = cluster.stub(L)
    assert s.Signup(raft_pb.SignupRequest(username="dave", password="pw12345", email="d@x.io")).success
    tok = cluster.login(L)
    cid = s.CreateChannel(raft_pb.CreateChannelRequest(token=tok, channel_name="proj")).channel_id
    assert s.AddUserToChannel(raft_pb.ChannelAdminRequest(token=tok, channel_id=cid,
                                                          target_username="bob")).success
    for k in range(5):
        assert s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id=cid, content=f"m{k}")).success
    assert s.SendDirectMessage(raft_pb.DirectMessageRequest(token=tok, recipient_username="bob",
                                                            content="hi")).success
    assert s.UploadFile(raft_pb.FileUploadRequest(token=tok, file_name="f.bin", file_data=b"\x00\x01" * 64,
                                                  channel_id=cid)).success
    assert s.RemoveUserFromChannel(raft_pb.ChannelAdminRequest(token=tok, channel_id=cid,
                                                               target_username="bob")).success
    assert s.Logout(raft_pb.LogoutRequest(token=tok)).success
    return L, cid


def test_exported_log_replays_under_reference_semantics(cluster, tmp_path):
    L, cid = _workload(cluster)
    assert cluster.wait_applied(lambda n: n.rt.core.last_applied == cluster.nodes[L].rt.core.commit_index)
    views = {i: _node_view(n.st) for i, n in cluster.nodes.items()}
    ports = {i: cluster.ports[i - 1] for i in cluster.nodes}
    cluster.stop()  # clean shutdown exports the reference-format log pickle
    for i, view in views.items():
        d = os.path.join(str(tmp_path), f"raft_node_{i}_data")
        log = pickle_compat.safe_load(os.path.join(d, f"raft_log_port_{ports[i]}.pkl"))
        st = pickle_compat.safe_load(os.path.join(d, f"raft_state_port_{ports[i]}.pkl"))
        assert set(st) == {"current_term", "voted_for", "commit_index", "last_applied"}
        assert st["commit_index"] <= len(log) - 1
        assert any(e["command"] == "NOOP" and e["data"] == b"{}" for e in log)
        assert any(e["command"] == "REVOKE_TOKEN" for e in log)
        ref = reference_replay(log, st["commit_index"])
        assert ref[0] == view[0]          # users (incl. genesis bcrypt hashes)
        assert ref[1] == view[1]          # channels: names, members, admins
        assert ref[2] == view[2]          # messages per channel
        assert ref[3] == view[3]          # DMs
        assert ref[4] == view[4]          # files


def test_genesis_pickles_byte_identical_across_replicas(cluster, tmp_path):
    L = cluster.leader()
    s = cluster.stub(L)
    tok = cluster.login(L)
    s.CreateChannel(raft_pb.CreateChannelRequest(token=tok, channel_name="team"))
    assert cluster.wait_applied(lambda n: len(n.st.channels) == 4)
    for n in cluster.nodes.values():
        n.rt.persist(all_files=True)
    blobs = {}
    for i in cluster.nodes:
        d = os.path.join(str(tmp_path), f"raft_node_{i}_data")
        blobs[i] = {f: open(os.path.join(d, f), "rb").read()
                    for f in ("channels.pkl", "messages.pkl", "direct_messages.pkl")}
    assert blobs[1] == blobs[2] == blobs[3]
    # default records are replicated (same hash bytes everywhere), not per-node seeds
    hashes = {n.st.users["alice"]["password"] for n in cluster.nodes.values()}
    assert len(hashes) == 1


def test_logout_revocation_is_replicated_and_survives_failover(cluster):
    L = cluster.leader()
    tok = cluster.login(L)
    F = next(i for i in cluster.nodes if i != L)
    ok = cluster.stub(F).GetChannels(raft_pb.GetChannelsRequest(token=tok))
    assert ok.success
    assert cluster.stub(L).Logout(raft_pb.LogoutRequest(token=tok)).success
    assert cluster.wait_applied(lambda n: len(n.st.revoked_tokens) == 1)
    assert not cluster.stub(F).GetChannels(raft_pb.GetChannelsRequest(token=tok)).success
    cluster.kill(L)
    L2 = cluster.leader()
    assert not cluster.stub(L2).GetChannels(raft_pb.GetChannelsRequest(token=tok)).success
    tok2 = cluster.login(L2)  # a fresh login still works, even within the same second
    assert tok2 != tok  # random jti: never the revoked token again
    assert cluster.stub(L2).GetChannels(raft_pb.GetChannelsRequest(token=tok2)).success


def test_request_id_makes_writes_idempotent(cluster):
    L = cluster.leader()
    s = cluster.stub(L)
    tok = cluster.login(L)
    for _ in range(3):  # a client retrying the same write (e.g. after DEADLINE_EXCEEDED)
        assert s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general", content="once",
                                                        request_id="req-42")).success
        assert s.SendDirectMessage(raft_pb.DirectMessageRequest(token=tok, recipient_username="bob",
                                                                content="dm", request_id="req-43")).success
    msgs = s.GetMessages(raft_pb.GetMessagesRequest(token=tok, channel_id="general")).messages
    assert [m.content for m in msgs].count("once") == 1
    assert msgs[-1].message_id == ChatNode._write_id(
        raft_pb.SendMessageRequest(request_id="req-42"), "alice")
    dms = s.GetDirectMessages(raft_pb.GetDirectMessagesRequest(token=tok, other_username="bob")).messages
    assert len(dms) == 1


def test_same_request_id_from_two_users_stores_both(cluster):
    """request_id de-duplicates one user's retries only: another user's write
    that carries the same request_id (a counter, or an id read back from
    GetMessages) is a different record, and an upload returns its own file_id."""
    L = cluster.leader()
    s = cluster.stub(L)
    ta, tb = cluster.login(L, "alice"), cluster.login(L, "bob")
    for tok, text in ((ta, "from alice"), (tb, "from bob")):
        assert s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general", content=text,
                                                        request_id="7")).success
    msgs = s.GetMessages(raft_pb.GetMessagesRequest(token=ta, channel_id="general")).messages
    got = [m.content for m in msgs]
    assert got.count("from alice") == 1 and got.count("from bob") == 1
    assert len({m.message_id for m in msgs}) == len(msgs)
    # alice re-uses an id she can see (bob's message id) as her request_id: still her own record
    bob_id = next(m.message_id for m in msgs if m.content == "from bob")
    assert s.SendMessage(raft_pb.SendMessageRequest(token=ta, channel_id="general", content="copycat",
                                                    request_id=bob_id[:64])).success
    got = [m.content for m in s.GetMessages(raft_pb.GetMessagesRequest(token=ta, channel_id="general")).messages]
    assert "copycat" in got and got.count("from bob") == 1
    fa = s.UploadFile(raft_pb.FileUploadRequest(token=ta, file_name="a.txt", file_data=b"A",
                                                channel_id="general", request_id="f1"))
    fb = s.UploadFile(raft_pb.FileUploadRequest(token=tb, file_name="b.txt", file_data=b"B",
                                                channel_id="general", request_id="f1"))
    assert fa.success and fb.success and fa.file_id != fb.file_id
    da = s.DownloadFile(raft_pb.FileDownloadRequest(token=ta, file_id=fa.file_id))
    db = s.DownloadFile(raft_pb.FileDownloadRequest(token=tb, file_id=fb.file_id))
    assert da.file_data == b"A" and db.file_data == b"B"


def test_native_storage_reference_pair_never_ahead_of_log(tmp_path):
    d = str(tmp_path)
    st = NativeStorage(d, 5000, fsync=True)
    st.load()
    state_p = os.path.join(d, "raft_state_port_5000.pkl")
    log_p = os.path.join(d, "raft_log_port_5000.pkl")

    def pair():
        s = pickle_compat.safe_load(state_p)
        n = len(pickle_compat.safe_load(log_p)) if os.path.exists(log_p) else 0
        return s, n

    st.append([Entry(1, "NOOP", b"{}"), Entry(1, "SEND_MESSAGE", b'{"id": "a"}')])
    st.save_state({"current_term": 1, "voted_for": 1, "commit_index": 1, "last_applied": 1})
    s, n = pair()
    assert s["current_term"] == 1 and s["commit_index"] <= n - 1 and s["last_applied"] <= n - 1
    st.export()
    s, n = pair()
    assert n == 2 and s["commit_index"] == 1
    st.append([Entry(2, "SEND_MESSAGE", b'{"id": "b"}')])
    st.save_state({"commit_index": 2, "last_applied": 2})
    s, n = pair()
    assert n == 2 and s["commit_index"] == 1  # clamped to the exported log
    # a follower truncation past the export point re-clamps
    st.truncate_from(1)
    st.append([Entry(3, "SEND_MESSAGE", b'{"id": "c"}')])
    st.save_state({"current_term": 3, "commit_index": 1, "last_applied": 1})
    s, n = pair()
    assert s["commit_index"] <= 0  # exported entry 1 was replaced: not claimable any more
    st.export()
    s, n = pair()
    assert n == 2 and s["commit_index"] == 1
    st.close()
    # restart: the native log is authoritative, the clamped indices only replay more
    st2 = NativeStorage(d, 5000, fsync=True)
    state, entries = st2.load()
    assert [e.data for e in entries] == [b"{}", b'{"id": "c"}'] and state["current_term"] == 3
    st2.close()


# ---------------------------------------------------------------- process crash test
def _spawn(i, port, peers, root):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    cmd = [sys.executable, "-m", "drtc_amd.server.node", "--node-id", str(i), "--port", str(port),
           "--peers", peers, "--data-root", root, "--llm", "", "--election-timeout", "0.4,0.8",
           "--heartbeat", "0.04", "--bcrypt-rounds", "4", "--log-level", "WARNING"]
    return subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                            start_new_session=True)


def _leader(addrs, timeout=30.0):
    t_end = time.time() + timeout
    while time.time() < t_end:
        for i, a in addrs.items():
            try:
                r = make_stub(grpc.insecure_channel(a), RAFT_SERVICE).GetLeaderInfo(
                    raft_pb.GetLeaderRequest(), timeout=0.5)
                if r.is_leader:
                    return i
            except grpc.RpcError:
                pass
        time.sleep(0.1)
    raise TimeoutError("no leader")


def test_sigkill_leader_mid_write_then_restart_from_disk(tmp_path):
    ports = {i: free_port() for i in (1, 2, 3)}
    addrs = {i: f"127.0.0.1:{p}" for i, p in ports.items()}
    peers = ",".join(f"{i}={a}" for i, a in addrs.items())
    procs = {i: _spawn(i, ports[i], peers, str(tmp_path)) for i in ports}
    acked = []
    try:
        L = _leader(addrs)
        stub = make_stub(grpc.insecure_channel(addrs[L]), RAFT_SERVICE)
        t_end = time.time() + 30
        while True:  # defaults arrive through the log right after the first election
            r = stub.Login(raft_pb.LoginRequest(username="alice", password="alice123"), timeout=10)
            if r.success or time.time() > t_end:
                break
            time.sleep(0.1)
        assert r.success
        tok = r.token

        def send(stub, k):
            rid = f"w{k}"
            try:
                rr = stub.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general",
                                                                 content=rid, request_id=rid), timeout=3)
                if rr.success:
                    acked.append(rid)
                return rr.success
            except grpc.RpcError:
                return False

        for k in range(40):
            send(stub, k)
        # SIGKILL the leader while a burst of writes is in flight
        import threading
        burst = threading.Thread(target=lambda: [send(stub, k) for k in range(40, 80)])
        burst.start()
        time.sleep(0.05)
        os.killpg(procs[L].pid, signal.SIGKILL)
        procs[L].wait(timeout=10)
        burst.join(timeout=60)
        rest = {i: a for i, a in addrs.items() if i != L}
        L2 = _leader(rest)
        stub2 = make_stub(grpc.insecure_channel(addrs[L2]), RAFT_SERVICE)
        for k in range(80, 100):
            send(stub2, k)
        # restart the killed node from its data directory
        procs[L] = _spawn(L, ports[L], peers, str(tmp_path))
        want = set(acked)
        assert len(want) >= 60
        t_end = time.time() + 40
        ok = False
        while time.time() < t_end and not ok:
            ok = True
            for i, a in addrs.items():
                try:
                    ms = make_stub(grpc.insecure_channel(a), RAFT_SERVICE).GetMessages(
                        raft_pb.GetMessagesRequest(token=tok, channel_id="general", limit=1000),
                        timeout=2).messages
                except grpc.RpcError:
                    ok = False
                    break
                ids = [m.content for m in ms]  # content = the write's request_id
                if not want <= set(ids) or len(ids) != len(set(ids)):
                    ok = False
            time.sleep(0.2)
        assert ok, "an acknowledged write is missing (or duplicated) on some node after the crash"
    finally:
        for p in procs.values():
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait(timeout=10)


def test_persist_writes_app_state_outside_the_state_lock(cluster, monkeypatch):
    """App-state pickles are taken under the state lock and written after it is
    released: applies never wait for file I/O (a large messages.pkl rewrite used to
    block every apply for its whole duration).  The files still match the state."""
    L, cid = _workload(cluster)
    rt = cluster.nodes[L].rt
    writes = []
    real = pickle_compat.write_bytes

    def probe(data, path, fsync=False):
        if rt.state_lock._is_owned():  # only the leader's own state lock is of interest
            writes.append(path)
        return real(data, path, fsync)

    monkeypatch.setattr(pickle_compat, "write_bytes", probe)
    held = rt.persist(all_files=True)
    monkeypatch.undo()
    assert writes == [] and held >= 0.0, writes
    st = ChatState()
    st.load(rt.dir)
    assert [m["content"] for m in st.channel_messages[cid]] == [f"m{k}" for k in range(5)]


def test_failed_persist_keeps_files_dirty(cluster, monkeypatch):
    """encode() marks the files clean before they are written (outside the lock):
    a write that fails (disk full, I/O error) must put its file - and every file
    not written yet - back on the dirty list so the next persist retries it."""
    L, cid = _workload(cluster)
    rt = cluster.nodes[L].rt
    rt.persist(all_files=True)
    with rt.state_lock:
        rt.state.dirty.update({"users", "messages"})
    real = pickle_compat.write_bytes

    def broken(data, path, fsync=False):
        raise OSError(28, "No space left on device")

    monkeypatch.setattr(pickle_compat, "write_bytes", broken)
    with pytest.raises(OSError):
        rt.persist()
    with rt.state_lock:
        assert {"users", "messages"} <= rt.state.dirty
    monkeypatch.setattr(pickle_compat, "write_bytes", real)
    rt.persist()
    with rt.state_lock:
        assert not ({"users", "messages"} & rt.state.dirty)


def test_native_storage_vote_survives_torn_reference_state_file(tmp_path):
    """term / vote live in their own fsynced hard-state file: the reference-format
    state pickle (rewritten unsynced on every commit_index change) coming back
    empty or stale after a power loss must not undo a vote."""
    d = str(tmp_path)
    st = NativeStorage(d, 5001, fsync=True)
    st.load()
    st.save_state({"current_term": 3, "voted_for": 2, "commit_index": -1, "last_applied": -1})
    st.append([Entry(3, "NOOP", b"{}")])
    for c in range(5):  # commit progress: no hard-state change, no sync
        st.save_state({"commit_index": 0, "last_applied": 0})
    st.close()
    state_p = os.path.join(d, "raft_state_port_5001.pkl")
    with open(state_p, "wb"):
        pass  # torn: empty file
    st2 = NativeStorage(d, 5001, fsync=True)
    s, log = st2.load()
    assert s["current_term"] == 3 and s["voted_for"] == 2 and len(log) == 1
    st2.close()
    # stale: an older term in the reference pickle, the newer vote in the hard state
    pickle_compat.dump({"current_term": 1, "voted_for": None, "commit_index": -1,
                        "last_applied": -1}, state_p)
    st3 = NativeStorage(d, 5001, fsync=True)
    s, _ = st3.load()
    assert s["current_term"] == 3 and s["voted_for"] == 2
    st3.save_state({"current_term": 4, "voted_for": None})
    st3.close()
    s, _ = NativeStorage(d, 5001, fsync=True).load()
    assert s["current_term"] == 4 and s["voted_for"] is None


def test_native_storage_upgrades_old_dir_without_hard_state(tmp_path):
    """A data directory written before the hard-state file existed holds term / vote only in
    the reference state pickle.  The first save_state after the upgrade must write and fsync
    the hard state (even with term / vote unchanged) before the unsynced pickle rewrite, so a
    torn pickle afterwards cannot bring back term 0 with no vote."""
    d = str(tmp_path)
    state_p = os.path.join(d, "raft_state_port_5002.pkl")
    hard_p = os.path.join(d, "raft_hardstate_port_5002.pkl")
    pickle_compat.dump({"current_term": 7, "voted_for": 3, "commit_index": -1,
                        "last_applied": -1}, state_p)
    st = NativeStorage(d, 5002, fsync=True)
    s, _ = st.load()
    assert s["current_term"] == 7 and s["voted_for"] == 3
    assert not os.path.exists(hard_p)
    st.save_state({"commit_index": -1, "last_applied": -1})  # term / vote unchanged
    assert os.path.exists(hard_p)
    st.close()
    with open(state_p, "wb"):
        pass  # power loss tears the unsynced reference pickle
    s, _ = NativeStorage(d, 5002, fsync=True).load()
    assert s["current_term"] == 7 and s["voted_for"] == 3
