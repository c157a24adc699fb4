"""LLM service contract (prompts/parsers, engine backend over gRPC, TP over
gloo) and the legacy single-node chat.ChatService with streaming."""
import os
import sys
import threading
import time

import grpc
import pytest

from drtc_amd.engine import ChatTokenizer, LLMEngine
from drtc_amd.llm import prompts as P
from drtc_amd.llm.backends import EngineBackend
from drtc_amd.llm.server import serve as serve_llm
from drtc_amd.models import TINY_LLAMA, TransformerLM
from drtc_amd.protos import CHAT_SERVICE, LLM_SERVICE, chat_pb, llm_pb, make_stub
from drtc_amd.server.legacy import serve as serve_legacy
from drtc_amd.utils.cluster import free_port

M = P.ChatLine


def test_prompt_templates():
    msgs = [M("alice", f"m{i}") for i in range(8)]
    p = P.smart_reply_prompt(msgs)
    assert p.startswith("Based on this conversation:\nalice: m3\n") and "alice: m7\n\nGenerate exactly 3" in p
    assert "alice: m2" not in p
    s = P.summarize_prompt(msgs, 200)
    assert s.startswith("Summarize this conversation concisely in under 200 characters:\n\nalice: m0")
    assert P.answer_prompt("q?", []) == "q?\n\nProvide a short, helpful answer in 2 sentences or less."
    a = P.answer_prompt("q?", [f"c{i}" for i in range(7)])
    assert "c1" not in a and "c2\nc3" in a and "User's question: q?" in a
    assert 'User started typing: "hel"' in P.suggestions_prompt(msgs, "hel")
    assert "No previous context" in P.suggestions_prompt([], "")


def test_parsers():
    assert P.parse_smart_replies("1. Sure thing\n- Sounds good\n* OK!\nextra") == ["Sure thing", "Sounds good", "OK!"]
    assert P.parse_smart_replies("only one") == ["only one", "I agree", "Interesting point"]
    msgs = [M("a", "x"), M("b", "y")]
    s, k = P.parse_summary("Summary: hello\nworld\n\nKey Points:\n- one\n• two\n- three\n- four", msgs, 200)
    assert s == "hello world" and k == ["one", "two", "three"]
    s, k = P.parse_summary("Summary: " + "z" * 300, msgs, 200)
    assert len(s) == 200 and s.endswith("...") and k[0] == "2 messages exchanged"
    s, k = P.parse_summary("no structure", msgs, 200)
    assert s == "no structure"
    sug, top = P.parse_suggestions("COMPLETIONS:\n- a\n- b\nTOPICS:\n- t1", "")
    assert sug == ["a", "b"] and top == ["t1"]
    sug, top = P.parse_suggestions("garbage", "I think")
    assert sug[0] == "I think be the best option" and top == ["current discussion", "related ideas"]


def _llm_stub(port):
    return make_stub(grpc.insecure_channel(f"127.0.0.1:{port}"), LLM_SERVICE)


def test_llm_service_all_four_rpcs_with_engine_backend():
    m = TransformerLM(TINY_LLAMA, "cpu", seed=1)
    eng = LLMEngine(m, max_batch=8, max_model_len=1024, num_blocks=256, use_graphs=False)
    backend = EngineBackend(eng, ChatTokenizer(TINY_LLAMA.vocab_size))
    from drtc_amd.llm.service import FeatureParams

    fp = FeatureParams(ignore_eos=True)
    for f in (fp.answer, fp.smart, fp.summary, fp.suggest):
        f.max_new_tokens = 6
    port = free_port()
    srv = serve_llm(backend, port=port, bind="127.0.0.1", params=fp)
    try:
        s = _llm_stub(port)
        msgs = [llm_pb.Message(sender="alice", content="lunch at noon?"),
                llm_pb.Message(sender="bob", content="sure")]
        r = s.GetSmartReply(llm_pb.SmartReplyRequest(request_id="r1", recent_messages=msgs), timeout=60)
        assert r.request_id == "r1" and len(r.suggestions) == 3
        r = s.SummarizeConversation(llm_pb.SummarizeRequest(request_id="r2", messages=msgs, max_length=50),
                                    timeout=60)
        assert len(r.summary) <= 50 and 1 <= len(r.key_points) <= 3
        r = s.GetContextSuggestions(llm_pb.ContextRequest(request_id="r3", context=msgs, current_input="ok"),
                                    timeout=60)
        assert 1 <= len(r.suggestions) <= 5 and 1 <= len(r.topics) <= 3
        r = s.GetLLMAnswer(llm_pb.LLMRequest(request_id="r4", query="why?"), timeout=60)
        assert r.request_id == "r4" and r.confidence == pytest.approx(0.95)
        # concurrent requests share the continuous batch
        out = []
        ths = [threading.Thread(target=lambda: out.append(s.GetSmartReply(
            llm_pb.SmartReplyRequest(recent_messages=msgs), timeout=60))) for _ in range(6)]
        [t.start() for t in ths]
        [t.join() for t in ths]
        assert len(out) == 6 and eng.stats["decode_steps"] > 0
        e = s.GetSmartReply(llm_pb.SmartReplyRequest(recent_messages=[]), timeout=10)
        assert list(e.suggestions) == P.SMART_REPLY_EMPTY
    finally:
        srv.stop(0)
        backend.close()


def test_llm_service_fallbacks_on_backend_error():
    class Boom:
        def generate(self, *a, **k):
            raise RuntimeError("gpu on fire")

    port = free_port()
    srv = serve_llm(Boom(), port=port, bind="127.0.0.1")
    try:
        s = _llm_stub(port)
        msgs = [llm_pb.Message(sender="a", content="x")]
        assert list(s.GetSmartReply(llm_pb.SmartReplyRequest(recent_messages=msgs)).suggestions) == P.SMART_REPLY_FALLBACK
        assert s.SummarizeConversation(llm_pb.SummarizeRequest(messages=msgs)).summary == P.SUMMARY_ERROR
        assert s.GetLLMAnswer(llm_pb.LLMRequest(query="q")).confidence == 0.0
        assert list(s.GetContextSuggestions(llm_pb.ContextRequest(context=msgs)).suggestions) == P.SUGGEST_ERROR
    finally:
        srv.stop(0)


def test_llm_service_takes_a_burst_of_concurrent_calls():
    """1,200 smart-reply RPCs started together (a client wave over a 1,024-slot engine) all
    complete: the server's pending-call queue is sized above grpc-core's default of 1,000,
    which CANCELs the excess of such a burst (protos.SERVER_QUEUE_OPTS)."""
    from drtc_amd.llm.backends import ScriptedBackend

    n = 1200
    port = free_port()
    srv = serve_llm(ScriptedBackend(delay=0.05), port=port, bind="127.0.0.1", workers=n + 8)
    chans = [grpc.insecure_channel(f"127.0.0.1:{port}", options=[("grpc.use_local_subchannel_pool", 1)])
             for _ in range(16)]
    try:
        for ch in chans:
            grpc.channel_ready_future(ch).result(timeout=30)
        stubs = [make_stub(ch, LLM_SERVICE) for ch in chans]
        msgs = [llm_pb.Message(sender="a", content="x")]
        go, errors, ok = threading.Event(), [], []

        def one(k):
            go.wait()
            try:
                r = stubs[k % len(stubs)].GetSmartReply(
                    llm_pb.SmartReplyRequest(recent_messages=msgs), timeout=60)
                ok.append(len(r.suggestions))
            except grpc.RpcError as e:
                errors.append(e.code())

        ths = [threading.Thread(target=one, args=(k,)) for k in range(n)]
        [t.start() for t in ths]
        go.set()
        [t.join() for t in ths]
        assert not errors, set(errors)
        assert len(ok) == n and set(ok) == {3}
    finally:
        [ch.close() for ch in chans]
        srv.stop(0)


def test_ask_ai_retries_with_backoff():
    """GetLLMAnswer retries failures and empty answers with exponential backoff
    (ref llm_server.py:164-208) and stops retrying when the deadline is near."""
    from drtc_amd.llm.service import LLMServicer

    class Flaky:
        def __init__(self, script):
            self.script, self.calls = list(script), 0

        def generate(self, prompts, params, timeout=None):
            self.calls += 1
            item = self.script.pop(0)
            if isinstance(item, Exception):
                raise item
            return [item]

    class Ctx:
        def __init__(self, left):
            self.left = left

        def time_remaining(self):
            return self.left

    req = llm_pb.LLMRequest(request_id="q1", query="what is raft?")
    b = Flaky([RuntimeError("busy"), "", "Raft is a consensus protocol."])
    r = LLMServicer(b, answer_backoff=0.01).GetLLMAnswer(req, Ctx(None))
    assert b.calls == 3 and r.answer == "Raft is a consensus protocol." and r.confidence > 0.9
    b = Flaky(["", "", ""])
    r = LLMServicer(b, answer_backoff=0.01).GetLLMAnswer(req, Ctx(None))
    assert b.calls == 3 and r.answer == P.ANSWER_EMPTY and r.confidence == 0.0
    b = Flaky([RuntimeError("down")] * 3)
    r = LLMServicer(b, answer_backoff=0.01).GetLLMAnswer(req, Ctx(None))
    assert r.answer == P.ANSWER_ERROR and r.request_id == "q1"
    b = Flaky([RuntimeError("down")] * 3)  # 0.5 s left: no retry fits
    r = LLMServicer(b, answer_backoff=1.0).GetLLMAnswer(req, Ctx(0.5))
    assert b.calls == 1 and r.answer == P.ANSWER_ERROR


@pytest.mark.slow
def test_tp2_engine_group_over_gloo():
    """Two lockstep TP ranks (gloo, CPU) produce the same greedy text as TP=1."""
    code = r"""
import sys
sys.path.insert(0, %r)
from drtc_amd.parallel.tp_engine import TPEngineGroup
from drtc_amd.engine import ChatTokenizer, SamplingParams, LLMEngine
from drtc_amd.models import TINY_LLAMA, TransformerLM
if __name__ == '__main__':
    tok = ChatTokenizer(TINY_LLAMA.vocab_size)
    kw = dict(max_batch=8, max_model_len=512, num_blocks=64, use_graphs=False)
    g = TPEngineGroup('tiny-llama', 2, kw, tok)
    a = g.generate(['hello world', 'lunch tomorrow?'], SamplingParams.greedy(8, ignore_eos=True), timeout=120)
    try:  # a caller that gives up: the abort is broadcast and applied by both ranks
        g.generate(['hello ' * 30], SamplingParams.greedy(400, ignore_eos=True), timeout=0.3)
        raise AssertionError('expected a timeout')
    except TimeoutError:
        pass
    c = g.generate(['hello world'], SamplingParams.greedy(8, ignore_eos=True), timeout=120)
    assert c[0] == a[0], (c, a)  # the group is still in lockstep and serving
    g.close()
    eng = LLMEngine(TransformerLM(TINY_LLAMA, 'cpu', seed=1234), seed=0, **kw)
    b = [tok.decode(r.output_ids) for r in eng.generate([tok.encode('hello world'), tok.encode('lunch tomorrow?')],
                                                        SamplingParams.greedy(8, ignore_eos=True))]
    assert a == b, (a, b)
    print('TP-OK')
""" % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    import subprocess
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
    assert "TP-OK" in r.stdout, r.stderr[-2000:]


def test_legacy_chat_service(tmp_path):
    port = free_port()
    srv, server = serve_legacy(port, str(tmp_path / "server_data"), block=False, bcrypt_rounds=4)
    try:
        s = make_stub(grpc.insecure_channel(f"127.0.0.1:{port}"), CHAT_SERVICE)
        r = s.Signup(chat_pb.SignupRequest(username="x", password="pw", email="bad"))
        assert r.code == 400 and "3-20" in r.message
        r = s.Signup(chat_pb.SignupRequest(username="dave", password="nodigits", email="d@x.io"))
        assert "number or special" in r.message
        assert s.Signup(chat_pb.SignupRequest(username="dave", password="pw1234", email="d@x.io")).code == 201
        ta = s.Login(chat_pb.LoginRequest(username="admin", password="admin123")).token
        td = s.Login(chat_pb.LoginRequest(username="dave", password="pw1234")).token
        chans = {c.name: c.channel_id for c in s.GetChannels(chat_pb.GetChannelsRequest(token=ta)).channels}
        assert set(chans) == {"general", "random", "development"}
        events = []
        stream = s.StreamMessages(chat_pb.StreamRequest(token=td))

        def consume():
            try:
                for ev in stream:
                    events.append(ev)
            except grpc.RpcError:
                pass

        th = threading.Thread(target=consume, daemon=True)
        th.start()
        time.sleep(0.3)
        assert s.PostMessage(chat_pb.PostRequest(token=ta, channel_id=chans["general"], content="hi all",
                                                 type="text")).success
        assert s.SendDirectMessage(chat_pb.DirectMessageRequest(token=ta, recipient_username="dave",
                                                                content="psst")).success
        t_end = time.time() + 5
        while len(events) < 2 and time.time() < t_end:
            time.sleep(0.05)
        stream.cancel()
        assert [e.event_type for e in events[:2]] == ["message", "dm"]
        assert events[0].message.content == "hi all" and events[1].direct_message.content == "psst"
        for k in range(5):
            s.PostMessage(chat_pb.PostRequest(token=ta, channel_id=chans["general"], content=str(k)))
        page = s.GetMessages(chat_pb.GetRequest(token=ta, channel_id=chans["general"], limit=2, offset=1))
        assert [m.content for m in page.messages] == ["0", "1"] and page.next_cursor == "3"
        cid_r = s.CreateChannel(chat_pb.CreateChannelRequest(token=td, channel_name="ops"))
        assert cid_r.success
        ops_id = next(c.channel_id for c in s.GetChannels(chat_pb.GetChannelsRequest(token=td)).channels
                      if c.name == "ops")
        r = s.ManageChannel(chat_pb.ManageChannelRequest(token=td, channel_id=ops_id, action="add_user",
                                                         parameters={"username": "user1"}))
        assert r.success
        assert not s.ManageChannel(chat_pb.ManageChannelRequest(token=ta, channel_id=ops_id,
                                                                action="add_user")).success
        # the reference's UNIMPLEMENTED four
        assert s.UpdatePresence(chat_pb.UpdatePresenceRequest(token=td, status="away")).success
        assert s.LeaveChannel(chat_pb.LeaveChannelRequest(token=ta, channel_id=chans["general"])).success
        info = s.GetServerInfo(chat_pb.ServerInfoRequest())
        assert info.is_leader and info.node_id == 1
        uid = next(u.user_id for u in s.GetOnlineUsers(chat_pb.GetOnlineUsersRequest(token=ta)).users
                   if u.username == "user2")
        assert s.ManageUser(chat_pb.ManageUserRequest(token=ta, target_user_id=uid, action="disable")).success
        assert not s.Login(chat_pb.LoginRequest(username="user2", password="user123")).success
        up = s.UploadFile(chat_pb.FileUploadRequest(token=ta, channel_id=chans["general"], file_name="f.bin",
                                                    file_data=b"\x00\x01"))
        assert s.DownloadFile(chat_pb.FileDownloadRequest(token=ta, file_id=up.file_id)).file_data == b"\x00\x01"
        conv = s.ListConversations(chat_pb.ListConversationsRequest(token=td)).conversations
        assert conv[0].username == "admin" and conv[0].last_message.content == "psst"
    finally:
        server.stop(0)
    # persistence in the reference layout
    from drtc_amd.utils.pickle_compat import safe_load
    d = safe_load(str(tmp_path / "server_data" / "users.pkl"))
    assert {"users", "users_by_email", "users_by_id"} <= set(d) and "dave" in d["users"]


def test_replica_pool_evicts_dead_replica_and_respawns():
    """DP failure detection: a killed engine process is evicted, its in-flight
    requests are re-dispatched to a healthy replica, and it is respawned."""
    import time

    from drtc_amd.engine import ChatTokenizer, SamplingParams
    from drtc_amd.llm.backends import ReplicaRouter, WorkerPool
    from drtc_amd.models import TINY_LLAMA

    kw = dict(max_batch=4, max_model_len=256, num_blocks=64, use_graphs=False)
    pool = WorkerPool("tiny-llama", ["cpu", "cpu"], kw, hb_interval=0.2, hb_timeout=20,
                      max_restarts=1)
    try:
        router = ReplicaRouter(pool, ChatTokenizer(TINY_LLAMA.vocab_size), 256)
        prm = SamplingParams.greedy(4, ignore_eos=True)
        assert len(router.generate(["hello there"] * 4, prm, timeout=60)) == 4
        pool.procs[0].kill()
        outs = router.generate(["after the crash"] * 4, prm, timeout=60)
        assert len(outs) == 4
        assert pool.evictions and pool.evictions[0][0] == 0
        t0 = time.monotonic()
        while not pool.healthy[0] and time.monotonic() - t0 < 60:
            time.sleep(0.2)
        assert pool.healthy[0] and pool.restarts[0] == 1
        h = pool.health()
        assert h[1]["healthy"] and "running" in h[1]
        assert len(router.generate(["back again"] * 4, prm, timeout=60)) == 4
    finally:
        pool.close()


def test_fit_prompt_keeps_instruction_head_and_tail():
    """Over-long prompts lose their oldest conversation lines, never the
    summarize instruction."""
    from drtc_amd.engine import ChatTokenizer
    from drtc_amd.llm.prompts import ChatLine, fit_prompt, summarize_prompt

    tok = ChatTokenizer(4096)
    msgs = [ChatLine("alice", f"message number {i} about the release plan") for i in range(400)]
    text = summarize_prompt(msgs, 200)
    full = tok.encode(text)
    ids = fit_prompt(tok, text, 300)
    assert len(full) > 300 and len(ids) == 300
    out = tok.decode(ids)
    assert out.startswith("Summarize this conversation concisely in under 200 characters")
    assert "Key Points:" in out and "message number 399" in out and "message number 0 " not in out
    assert fit_prompt(tok, "short prompt", 300) == tok.encode("short prompt")


def test_pool_workers_exit_when_parent_dies():
    """A parent that dies without closing its WorkerPool (os._exit, SIGKILL)
    must not leave engine workers behind holding the device and its KV cache."""
    import subprocess
    import sys as _sys

    code = r"""
import os, sys
sys.path.insert(0, %r)
from drtc_amd.llm.backends import WorkerPool
pool = WorkerPool("tiny-llama", ["cpu"], dict(max_batch=2, max_model_len=128, num_blocks=16,
                  use_graphs=False), hb_interval=0.2)
print(pool.procs[0].pid, flush=True)
os._exit(0)
""" % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([_sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    pid = int(p.stdout.strip().splitlines()[-1])
    deadline = time.time() + 30
    while time.time() < deadline:
        try:
            os.kill(pid, 0)
        except ProcessLookupError:
            return
        with open(f"/proc/{pid}/stat") as f:  # reaped zombie counts as gone
            if f.read().split()[2] == "Z":
                return
        time.sleep(0.2)
    raise AssertionError(f"engine worker {pid} outlived its parent")


def test_pool_router_timeout_aborts_on_the_replica():
    """A request whose caller times out is aborted on its replica (the engine
    frees its slot and KV blocks) and the replica's load count comes back to
    zero (it used to leak one per released-before-done request)."""
    from drtc_amd.engine import SamplingParams
    from drtc_amd.llm.backends import GenerationError, ReplicaRouter, WorkerPool

    kw = dict(max_batch=4, max_model_len=1024, num_blocks=64, use_graphs=False)
    pool = WorkerPool("tiny-llama", ["cpu"], kw, hb_interval=0.1)
    try:
        router = ReplicaRouter(pool, ChatTokenizer(TINY_LLAMA.vocab_size), 1024)
        with pytest.raises(GenerationError):
            router.generate(["hello " * 20], SamplingParams.greedy(900, ignore_eos=True),
                            timeout=0.2)
        assert pool.load == [0]
        deadline = time.time() + 30
        while time.time() < deadline:
            h = pool.health()[0]
            if h.get("aborted", 0) == 1 and h.get("running", 1) == 0:
                break
            time.sleep(0.1)
        assert h.get("aborted") == 1 and h.get("running") == 0, h
        out = router.generate(["hi"], SamplingParams.greedy(3, ignore_eos=True), timeout=60)
        assert len(out) == 1 and pool.load == [0]
    finally:
        pool.close()


def test_default_engine_batch_per_model():
    """Without --max-batch the LLM server sizes the engine batch per model from the
    BASELINE measurements that stay inside the reference's deadlines."""
    from drtc_amd.llm.server import default_max_batch

    assert default_max_batch("llama-3-8b") == 1024
    assert default_max_batch("mixtral-8x7b") == 1024
    assert default_max_batch("gemma-2b") == 2048
    assert default_max_batch("llama-3-70b") == 224      # p50 9.15 s < 10 s ask-AI deadline
    assert default_max_batch("llama-3-70b", tp=8) == 256
    assert default_max_batch("tiny-llama") == 256


def test_aio_frontend_serves_all_rpcs_over_a_replica_pool():
    """--frontend aio: grpc.aio handlers await ReplicaRouter.agenerate (no thread per
    request); every RPC answers through a tiny-llama replica process, a timed-out
    coroutine aborts its request on the replica, and the pool's load returns to zero."""
    import asyncio

    from drtc_amd.engine import SamplingParams
    from drtc_amd.llm.backends import GenerationError, ReplicaRouter, WorkerPool
    from drtc_amd.llm.server import serve_aio
    from drtc_amd.llm.service import FeatureParams
    from drtc_amd.protos import llm_pb

    kw = dict(max_batch=8, max_model_len=1024, num_blocks=128, use_graphs=False)
    pool = WorkerPool("tiny-llama", ["cpu"], kw, hb_interval=0.1)
    srv = None
    try:
        router = ReplicaRouter(pool, ChatTokenizer(TINY_LLAMA.vocab_size), 1024)
        fp = FeatureParams(ignore_eos=True)
        for f in ("answer", "smart", "summary", "suggest"):
            setattr(fp, f, SamplingParams(max_new_tokens=6, temperature=1.0, top_k=8,
                                          top_p=0.95, ignore_eos=True))
        port = free_port()
        srv = serve_aio(router, port=port, bind="127.0.0.1", params=fp)
        stub = _llm_stub(port)
        msgs = [llm_pb.Message(sender="alice", content="are we shipping today?"),
                llm_pb.Message(sender="bob", content="after the review")]
        r = stub.GetSmartReply(llm_pb.SmartReplyRequest(request_id="a", recent_messages=msgs),
                               timeout=60)
        assert len(r.suggestions) == 3
        r = stub.GetLLMAnswer(llm_pb.LLMRequest(request_id="b", query="when is the release?"),
                              timeout=60)
        assert r.request_id == "b" and r.answer
        r = stub.SummarizeConversation(llm_pb.SummarizeRequest(request_id="c", messages=msgs,
                                                               max_length=80), timeout=60)
        assert r.summary and r.request_id == "c"
        r = stub.GetContextSuggestions(llm_pb.ContextRequest(request_id="d", context=msgs,
                                                             current_input="ok"), timeout=60)
        assert r.request_id == "d" and len(r.suggestions) >= 1
        # concurrent RPCs meet in the replica's batch
        futs = [stub.GetSmartReply.future(llm_pb.SmartReplyRequest(request_id=str(i),
                                                                   recent_messages=msgs))
                for i in range(16)]
        assert all(len(f.result(timeout=120).suggestions) == 3 for f in futs)
        # a coroutine that times out aborts its request on the replica
        loop = asyncio.new_event_loop()
        try:
            with pytest.raises(GenerationError):
                loop.run_until_complete(router.agenerate(
                    "hello " * 20, SamplingParams.greedy(900, ignore_eos=True), timeout=0.2))
        finally:
            loop.close()
        deadline = time.time() + 30
        while time.time() < deadline and pool.load != [0]:
            time.sleep(0.1)
        assert pool.load == [0]
    finally:
        if srv is not None:
            srv.stop(0)
        pool.close()


def test_serve_placement_needs_budgets_on_shared_gpus():
    """Engine groups may share a GPU only with an explicit HBM budget each, adding up to at
    most 0.95 per GPU; the module docstring's five-config 8-GPU layout is valid."""
    import argparse
    import re

    from drtc_amd.llm import server as S

    def groups(specs):
        return [(f, S._group_devices(d, tp, 1 if tp > 1 else (len(d) if d else 1)), mem)
                for f, _, d, tp, mem in map(S.parse_serve, specs)]
    # the round-4 docstring example: the 70B TP8 group over every GPU beside unbudgeted groups
    with pytest.raises(ValueError, match="GPU 0 is shared"):
        S.check_placement(groups(["smart=gemma-2b@0", "summary=llama-3-8b@1",
                                  "answer=llama-3-70b@0-7:tp8", "suggest=mixtral-8x7b@2,3"]))
    with pytest.raises(ValueError, match="add up to"):
        S.check_placement(groups(["smart=gemma-2b@0:mem=0.5", "summary=llama-3-8b@0:mem=0.5"]))
    doc = re.findall(r"--serve ([a-z]+=\S+@\S+)", S.__doc__)
    assert len(doc) == 4, doc
    used = S.check_placement(groups(doc))
    assert sorted(used) == list(range(8)) and max(used.values()) <= 0.95
    # build_feature_backends checks before building anything (default group included)
    args = argparse.Namespace(backend="engine", model="llama-3-8b", tp=1, gpus=1, max_batch=4,
                              max_model_len=512, no_graphs=True, custom_allreduce=False,
                              in_process=True, hbm_budget=None)
    with pytest.raises(ValueError, match="GPU 0 is shared"):
        S.build_feature_backends(args, ["smart=gemma-2b@0:mem=0.3"])


def test_serve_group_without_gpus_is_placed_where_it_is_built(monkeypatch):
    """A tp1 --serve group without @GPUS runs on GPU 0 (one replica): the placement check and
    the build use that same rule, so it does not collide with groups on the other GPUs of a
    --gpus 8 server."""
    import argparse

    from drtc_amd.llm import server as S

    built = []
    monkeypatch.setattr(S, "build_backend",
                        lambda sub, devices=None: built.append((sub.model, sub.gpus, devices))
                        or object())
    args = argparse.Namespace(backend="engine", model="llama-3-8b", tp=1, gpus=8, max_batch=0,
                              max_model_len=512, no_graphs=True, custom_allreduce=False,
                              in_process=True, hbm_budget=None)
    S.build_feature_backends(args, ["smart=gemma-2b", "summary=llama-3-8b@1",
                                    "answer=llama-3-8b@2", "suggest=mixtral-8x7b@3"])
    assert ("gemma-2b", 1, [0]) in built and ("llama-3-8b", 1, [1]) in built
    with pytest.raises(ValueError, match="GPU 0 is shared"):  # and still checked
        S.build_feature_backends(args, ["smart=gemma-2b", "summary=llama-3-8b@0"])


def test_llm_server_serves_features_from_separate_backends():
    """``llm.server --serve FEATURE=MODEL...``: one service address, one engine group per
    feature (scripted stand-ins here); the feature spec grammar and its errors."""
    import argparse

    import grpc

    from drtc_amd.llm import server as S
    from drtc_amd.llm.service import FeatureRouter
    from drtc_amd.protos import LLM_SERVICE, llm_pb, make_stub
    from drtc_amd.utils.cluster import free_port

    assert S.parse_serve("smart=gemma-2b@0") == ("smart", "gemma-2b", [0], 1, None)
    assert S.parse_serve("ask=llama-3-70b@0-7:tp8") == ("answer", "llama-3-70b", list(range(8)),
                                                        8, None)
    assert S.parse_serve("suggest=mixtral-8x7b@2,3:mem=0.6") == ("suggest", "mixtral-8x7b",
                                                                 [2, 3], 1, 0.6)
    assert S.parse_serve("ask=llama-3-70b@0-7:tp8:mem=0.35")[3:] == (8, 0.35)
    for bad in ("smart", "chat=llama-3-8b", "smart=x@0,0", "answer=llama-3-70b@0-3:tp8",
                "smart=gemma-2b@0:mem=1.2", "smart=gemma-2b@0:mem=x", "smart=gemma-2b@0:foo"):
        with pytest.raises(ValueError):
            S.parse_serve(bad)
    args = argparse.Namespace(backend="engine", model="scripted", tp=1, gpus=1, max_batch=4,
                              max_model_len=512, no_graphs=True, custom_allreduce=False,
                              in_process=True)
    router = S.build_feature_backends(args, ["smart=scripted@0", "summary=scripted@1"])
    assert isinstance(router, FeatureRouter)
    assert router.route("smart") is not router.route("summary")
    assert router.route("answer") is router.route("suggest") is router.default
    port = free_port()
    srv = S.serve(router, port=port, bind="127.0.0.1")
    try:
        stub = make_stub(grpc.insecure_channel(f"127.0.0.1:{port}"), LLM_SERVICE)
        msgs = [llm_pb.Message(sender="a", content="lunch?")]
        stub.GetSmartReply(llm_pb.SmartReplyRequest(request_id="1", recent_messages=msgs), timeout=10)
        stub.SummarizeConversation(llm_pb.SummarizeRequest(request_id="2", messages=msgs,
                                                           max_length=200), timeout=10)
        stub.SummarizeConversation(llm_pb.SummarizeRequest(request_id="3", messages=msgs,
                                                           max_length=200), timeout=10)
        stub.GetLLMAnswer(llm_pb.LLMRequest(request_id="4", query="q?"), timeout=10)
        assert (router.route("smart").calls, router.route("summary").calls,
                router.default.calls) == (1, 2, 1)
    finally:
        srv.stop(0)
