"""Multi-node integration over real gRPC on localhost (in-process nodes)."""
import io
import time

import pytest

from drtc_amd.client.cli import ChatShell
from drtc_amd.client.connection import ClusterConnection
from drtc_amd.llm.backends import ScriptedBackend
from drtc_amd.llm.server import serve as serve_llm
from drtc_amd.protos import raft_pb
from drtc_amd.utils.cluster import LocalCluster, free_port


@pytest.fixture
def cluster(tmp_path):
    c = LocalCluster(3, data_root=str(tmp_path)).start()
    yield c
    c.stop()


def test_writes_replicate_and_reads_from_followers(cluster):
    L = cluster.leader()
    s = cluster.stub(L)
    tok = cluster.login(L)
    assert s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general", content="hello")).success
    r = s.CreateChannel(raft_pb.CreateChannelRequest(token=tok, channel_name="proj", description="d"))
    assert r.success and r.channel_id
    assert not s.CreateChannel(raft_pb.CreateChannelRequest(token=tok, channel_name="PROJ")).success
    assert s.SendDirectMessage(raft_pb.DirectMessageRequest(token=tok, recipient_username="bob",
                                                            content="hey")).success
    up = s.UploadFile(raft_pb.FileUploadRequest(token=tok, file_name="a.txt", file_data=b"x" * 1000,
                                                channel_id="general"))
    assert up.success and up.file_url == f"file://{up.file_id}"
    # majority commit: every node applies (followers shortly after)
    assert cluster.wait_applied(lambda n: len(n.st.channel_messages.get("general", [])) == 1
                                and up.file_id in n.st.files)
    for i in cluster.nodes:
        fs = cluster.stub(i)
        msgs = fs.GetMessages(raft_pb.GetMessagesRequest(token=tok, channel_id="general")).messages
        assert [m.content for m in msgs] == ["hello"]
        d = fs.DownloadFile(raft_pb.FileDownloadRequest(token=tok, file_id=up.file_id))
        assert d.success and d.file_data == b"x" * 1000
    # follower rejects writes
    F = next(i for i in cluster.nodes if i != L)
    r = cluster.stub(F).SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general", content="x"))
    assert not r.success and r.message == "Not the leader"
    info = cluster.stub(F).GetLeaderInfo(raft_pb.GetLeaderRequest())
    assert not info.is_leader and info.leader_id == L and info.leader_address == cluster.peers[L]


def test_channel_admin_rules(cluster):
    L = cluster.leader()
    s = cluster.stub(L)
    a, b = cluster.login(L, "alice"), cluster.login(L, "bob")
    cid = s.CreateChannel(raft_pb.CreateChannelRequest(token=a, channel_name="secret", is_private=True)).channel_id
    r = s.JoinChannel(raft_pb.JoinChannelRequest(token=b, channel_id=cid))
    assert not r.success and "add_user bob" in r.message
    r = s.AddUserToChannel(raft_pb.ChannelAdminRequest(token=b, channel_id=cid, target_username="charlie"))
    assert not r.success and "Only admins" in r.message
    assert s.AddUserToChannel(raft_pb.ChannelAdminRequest(token=a, channel_id=cid, target_username="bob")).success
    r = s.AddUserToChannel(raft_pb.ChannelAdminRequest(token=a, channel_id=cid, target_username="bob"))
    assert "already a member" in r.message
    r = s.RemoveUserFromChannel(raft_pb.ChannelAdminRequest(token=a, channel_id=cid, target_username="alice"))
    assert not r.success and "only admin" in r.message
    assert s.RemoveUserFromChannel(raft_pb.ChannelAdminRequest(token=a, channel_id=cid,
                                                               target_username="bob")).success
    mem = s.GetChannelMembers(raft_pb.GetChannelMembersRequest(token=a, channel_id=cid))
    assert [m.username for m in mem.members] == ["alice"] and mem.members[0].is_admin


def test_signup_login_logout_and_paging(cluster):
    L = cluster.leader()
    s = cluster.stub(L)
    r = s.Signup(raft_pb.SignupRequest(username="dave", password="pw12345", email="d@x.io"))
    assert r.success and r.user_info.username == "dave"
    assert s.Signup(raft_pb.SignupRequest(username="dave", password="x")).message == "Username already exists"
    assert not s.Login(raft_pb.LoginRequest(username="dave", password="bad")).success
    tok = cluster.login(L, "dave", "pw12345")
    for k in range(30):
        s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="random", content=str(k)))
    page = s.GetMessages(raft_pb.GetMessagesRequest(token=tok, channel_id="random", limit=10, offset=5))
    assert [m.content for m in page.messages] == [str(k) for k in range(15, 25)]  # Q9: offset honoured
    users = s.GetOnlineUsers(raft_pb.GetOnlineUsersRequest(token=tok)).users
    assert {u.username for u in users} >= {"alice", "bob", "charlie", "dave"}
    assert s.Logout(raft_pb.LogoutRequest(token=tok)).success
    assert not s.GetChannels(raft_pb.GetChannelsRequest(token=tok)).success


def test_failover_preserves_data_and_tokens(cluster):
    L = cluster.leader()
    tok = cluster.login(L)
    s = cluster.stub(L)
    for k in range(5):
        assert s.SendDirectMessage(raft_pb.DirectMessageRequest(token=tok, recipient_username="bob",
                                                                content=f"dm{k}")).success
    t0 = time.time()
    cluster.kill(L)
    L2 = cluster.leader()
    failover = time.time() - t0
    assert L2 != L and failover < 5.0
    s2 = cluster.stub(L2)
    # Q6: the token issued by the dead leader is valid on the new leader
    assert s2.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general", content="after")).success
    dms = s2.GetDirectMessages(raft_pb.GetDirectMessagesRequest(token=tok, other_username="bob"))
    assert [m.content for m in dms.messages] == [f"dm{k}" for k in range(5)]
    # restart the old leader from disk: it catches up
    cluster.start_node(L)
    assert cluster.wait_applied(lambda n: any(m["content"] == "after"
                                              for m in n.st.channel_messages.get("general", [])), 10)
    assert len(cluster.nodes[L].st.direct_messages) == 5


def test_conversations_unread(cluster):
    L = cluster.leader()
    s = cluster.stub(L)
    a, b = cluster.login(L, "alice"), cluster.login(L, "bob")
    for k in range(3):
        s.SendDirectMessage(raft_pb.DirectMessageRequest(token=a, recipient_username="bob", content=str(k)))
    conv = s.ListConversations(raft_pb.ListConversationsRequest(token=b)).conversations
    assert [(c.username, c.unread_count) for c in conv] == [("alice", 3)]


def test_ai_proxy_with_llm_service_and_fallbacks(tmp_path):
    port = free_port()
    llm_server = serve_llm(ScriptedBackend(), port=port, bind="127.0.0.1")
    try:
        with LocalCluster(3, data_root=str(tmp_path), llm_address=f"127.0.0.1:{port}") as c:
            L = c.leader()
            s = c.stub(L)
            tok = c.login(L)
            s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general", content="lunch?"))
            r = s.GetSmartReply(raft_pb.SmartReplyRequest(token=tok, channel_id="general"))
            assert list(r.suggestions) == ["Sounds good to me", "Let's do it tomorrow", "Thanks for the update"]
            r = s.SummarizeConversation(raft_pb.SummarizeRequest(token=tok, channel_id="general"))
            assert r.summary.startswith("The team") and len(r.key_points) == 3
            r = s.GetContextSuggestions(raft_pb.ContextSuggestionsRequest(token=tok, channel_id="general",
                                                                          current_input="I think"))
            assert list(r.suggestions)[:1] == ["sounds like a plan"] and list(r.topics) == ["deadlines", "code review"]
            r = s.GetLLMAnswer(raft_pb.LLMRequest(token=tok, query="what is raft?"))
            assert r.success and r.answer
    finally:
        llm_server.stop(0)
    # LLM down -> the reference's canned fallbacks
    with LocalCluster(1, data_root=str(tmp_path / "solo"), llm_address=f"127.0.0.1:{free_port()}") as c:
        L = c.leader()
        tok = c.login(L)
        s = c.stub(L)
        r = s.GetSmartReply(raft_pb.SmartReplyRequest(token=tok, channel_id="general"))
        assert list(r.suggestions) in (["Sounds good", "I understand", "Interesting"],
                                       ["I agree", "That's interesting", "Tell me more"])
        r = s.SummarizeConversation(raft_pb.SummarizeRequest(token=tok, channel_id="general"))
        assert r.summary == "No messages to summarize"


def test_cli_session(cluster, tmp_path):
    cluster.leader()
    conn = ClusterConnection(cluster.addresses(), round_sleep=0.1, discovery_rounds=30)
    conn.discover()
    out = io.StringIO()
    sh = ChatShell(conn, stdout=out, password_fn=lambda p: "alice123", download_dir=str(tmp_path / "dl"))
    f = tmp_path / "notes.txt"
    f.write_text("hello file")
    for line in ["login alice", "send hi team", "channels", "create_channel proj project room",
                 "send in proj", "members", "add_user bob", "switch general", "history 5", "users",
                 f"upload {f}", "files", "smart_reply", "summarize 3", "suggest lets", "ask what?",
                 "dm bob", "send hi bob", "back", "conversations", "status", "switch general",
                 "help_all", "help", "help send"]:
        sh.onecmd(line)
    text = out.getvalue()
    assert "Direct messages:" in text and "smart_reply [k]" in text
    assert "You -> #general: hi team" in text and "#proj" in text
    assert "Added bob to #proj" in text
    assert "Uploaded notes.txt" in text and "notes.txt" in text
    fid = text.split("Uploaded notes.txt (id ")[1].split(")")[0]
    sh.onecmd(f"download {fid}")
    assert open(tmp_path / "dl" / "alice" / "notes.txt").read() == "hello file"
    assert "Smart replies" in text and "Summary:" in text
    assert sh.onecmd("exit") is True
    # leader failover: the shell follows the new leader (Q25)
    cluster.kill(cluster.leader())
    cluster.leader()
    sh.onecmd("send after failover")
    assert "You -> #general: after failover" in out.getvalue()


def test_log_compaction_and_install_snapshot_over_grpc(tmp_path):
    """Nodes compact their logs; a follower that missed the compacted prefix
    catches up through raft.RaftSnapshot/InstallSnapshot (chunked), files
    included; a full-cluster restart recovers from snapshot + log suffix."""
    c = LocalCluster(3, data_root=str(tmp_path), snapshot_every=16).start()
    try:
        for rt in (n.rt for n in c.nodes.values()):
            rt.snapshot_chunk = 1024  # force a multi-chunk transfer
        L = c.leader()
        s = c.stub(L)
        tok = c.login(L)
        F = next(i for i in c.nodes if i != L)
        c.kill(F)
        for k in range(60):
            assert s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general",
                                                            content=f"m{k}")).success
        up = s.UploadFile(raft_pb.FileUploadRequest(token=tok, file_name="f.bin",
                                                    file_data=bytes(range(256)) * 40,
                                                    channel_id="general"))
        assert up.success
        for k in range(60, 64):
            assert s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general",
                                                            content=f"m{k}")).success
        t0 = time.time()
        while c.nodes[L].rt.core.snap_index < 40 and time.time() - t0 < 5:
            time.sleep(0.05)
        lead_core = c.nodes[L].rt.core
        assert lead_core.snap_index >= 40 and lead_core.first_index > 10
        c.start_node(F)
        for rt in (n.rt for n in c.nodes.values()):
            rt.snapshot_chunk = 1024
        assert c.wait_applied(lambda n: len(n.st.channel_messages.get("general", [])) == 64
                              and up.file_id in n.st.files, timeout=15)
        assert c.nodes[F].rt.core.snap_index >= 40  # state arrived as a snapshot
        from drtc_amd.utils.metrics import METRICS
        calls = METRICS.snapshot()["counters"].get("rpc.raft.RaftSnapshot/InstallSnapshot.calls", 0)
        assert calls > 1  # chunked transfer
        d = c.stub(F).DownloadFile(raft_pb.FileDownloadRequest(token=tok, file_id=up.file_id))
        assert d.success and d.file_data == bytes(range(256)) * 40
        # whole-cluster restart: snapshot + log suffix replay
        for i in list(c.nodes):
            c.kill(i)
        for i in c.peers:
            c.start_node(i)
        L2 = c.leader()
        tok2 = c.login(L2)
        msgs = c.stub(L2).GetMessages(raft_pb.GetMessagesRequest(token=tok2, channel_id="general",
                                                                 limit=100)).messages
        assert [m.content for m in msgs] == [f"m{k}" for k in range(64)]
    finally:
        c.stop()


def test_cli_failover_session_recovery(tmp_path):
    """Reconnect recovery (ref client/chat_client.py:147-228): on a new leader the
    shell re-validates its token and restores the channel; with node-local tokens
    (token_mode="reference") the new leader rejects it and the shell logs out.
    Plus the send-time channel check and history's auto-logout."""
    for mode, survives in (("replicated", True), ("reference", False)):
        c = LocalCluster(3, data_root=str(tmp_path / mode), token_mode=mode).start()
        try:
            c.leader()
            conn = ClusterConnection(c.addresses(), round_sleep=0.1, discovery_rounds=30)
            conn.discover()
            out = io.StringIO()
            sh = ChatShell(conn, stdout=out, password_fn=lambda p: "alice123")
            sh.onecmd("login alice")
            sh.onecmd("join random")
            c.kill(c.leader())
            c.leader()
            sh.onecmd("send after failover")
            text = out.getvalue()
            assert "Reconnected to new leader" in text
            if survives:
                assert "Restored channel #random" in text
                assert "You -> #random: after failover" in text
            else:
                assert "Session expired on new leader" in text and "Please re-login: login alice" in text
                assert sh.token is None
        finally:
            c.stop()


def test_cli_send_checks_channel_and_history_auto_logout(cluster):
    cluster.leader()
    conn = ClusterConnection(cluster.addresses(), round_sleep=0.1, discovery_rounds=30)
    conn.discover()
    out = io.StringIO()
    sh = ChatShell(conn, stdout=out, password_fn=lambda p: "alice123")
    sh.onecmd("login alice")
    sh.channel_id, sh.channel_name = "gone-channel-id", "gone"
    sh.onecmd("send hello?")
    assert "Channel #gone no longer exists" in out.getvalue() and sh.channel_name == "general"
    sh.token = sh.token[:-4] + "AAAA"  # a token the server rejects
    sh.onecmd("history 5")
    assert "Your session is invalid on this server" in out.getvalue() and sh.token is None


def test_per_feature_llm_routing(tmp_path):
    """Each AI RPC goes to its feature's LLM service (NodeConfig.llm_smart / llm_summary /
    llm_ask / llm_suggest): one node serving the per-feature model matrix of BASELINE.json."""
    backends = {f: ScriptedBackend() for f in ("smart", "summary", "ask", "suggest")}
    ports = {f: free_port() for f in backends}
    servers = [serve_llm(b, port=ports[f], bind="127.0.0.1") for f, b in backends.items()]
    try:
        kw = {f"llm_{f}": f"127.0.0.1:{p}" for f, p in ports.items()}
        with LocalCluster(3, data_root=str(tmp_path), llm_address=f"127.0.0.1:{free_port()}",
                          **kw) as c:
            L = c.leader()
            s = c.stub(L)
            tok = c.login(L)
            s.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general", content="lunch?"))
            calls = []
            r = s.GetSmartReply(raft_pb.SmartReplyRequest(token=tok, channel_id="general"))
            assert list(r.suggestions)[0] == "Sounds good to me"
            calls.append({f: b.calls for f, b in backends.items()})
            r = s.SummarizeConversation(raft_pb.SummarizeRequest(token=tok, channel_id="general"))
            assert r.summary.startswith("The team")
            calls.append({f: b.calls for f, b in backends.items()})
            r = s.GetLLMAnswer(raft_pb.LLMRequest(token=tok, query="what is raft?"))
            assert r.success
            calls.append({f: b.calls for f, b in backends.items()})
            r = s.GetContextSuggestions(raft_pb.ContextSuggestionsRequest(
                token=tok, channel_id="general", current_input="I think"))
            assert list(r.topics) == ["deadlines", "code review"]
            calls.append({f: b.calls for f, b in backends.items()})
            order = ["smart", "summary", "ask", "suggest"]
            for i, snap in enumerate(calls):  # after RPC i exactly features 0..i were called once
                assert snap == {f: int(order.index(f) <= i) for f in order}, (i, snap)
            # the routing holds on every node (a follower serves AI RPCs too)
            F = next(i for i in c.peers if i != L)
            deadline = time.time() + 5
            while time.time() < deadline and not c.stub(F).GetMessages(
                    raft_pb.GetMessagesRequest(token=tok, channel_id="general")).messages:
                time.sleep(0.02)  # the follower applies the message
            r = c.stub(F).GetSmartReply(raft_pb.SmartReplyRequest(token=tok, channel_id="general"))
            assert r.success and backends["smart"].calls == 2 and backends["ask"].calls == 1
    finally:
        for sv in servers:
            sv.stop(0)


def test_logout_on_follower_is_forwarded_to_leader(cluster):
    """The reference logs out on any node (server/raft_node.py:1751): a follower relays the
    logout to the leader, whose replicated revocation invalidates the token everywhere."""
    L = cluster.leader()
    tok = cluster.login(L)
    F = next(i for i in cluster.peers if i != L)
    r = cluster.stub(F).Logout(raft_pb.LogoutRequest(token=tok))
    assert r.success, r.message
    deadline = time.time() + 5
    while time.time() < deadline:
        ok = [cluster.stub(i).GetOnlineUsers(raft_pb.GetOnlineUsersRequest(token=tok)).success
              for i in cluster.peers]
        if not any(ok):
            break
        time.sleep(0.05)
    assert not any(ok)


def test_process_cluster_one_interpreter_per_node(tmp_path):
    """utils.cluster.ProcessCluster: three Raft nodes in three processes elect a leader that
    serves logins and a replicated write over RPC, then shut down together."""
    from drtc_amd.protos import raft_pb
    from drtc_amd.utils.cluster import ProcessCluster

    c = ProcessCluster(3, data_root=str(tmp_path)).start()
    try:
        L = c.leader()
        tok = c.login(L)
        r = c.stub(L).SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general",
                                                             content="from another process"))
        assert r.success
        got = c.stub(L).GetMessages(raft_pb.GetMessagesRequest(token=tok, channel_id="general",
                                                               limit=50))
        assert any(m.content == "from another process" for m in got.messages)
    finally:
        c.stop()
    assert all(not p.is_alive() for p in c.procs.values())
