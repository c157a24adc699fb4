"""The LLM service end to end on the GPU: gRPC -> engine loop (continuous
batching, hipGraph decode, HIP kernels) -> parsers, and the Raft cluster's
AI proxy in front of it."""
import threading

import grpc
import pytest

from drtc_amd.engine import ChatTokenizer, LLMEngine
from drtc_amd.llm.backends import EngineBackend
from drtc_amd.llm.server import serve as serve_llm
from drtc_amd.llm.service import FeatureParams
from drtc_amd.models import TINY_LLAMA, TransformerLM
from drtc_amd.protos import LLM_SERVICE, llm_pb, make_stub, raft_pb
from drtc_amd.utils.cluster import LocalCluster, free_port

pytestmark = pytest.mark.gpu


def test_llm_service_on_gpu_through_raft_cluster(hipk, tmp_path):
    m = TransformerLM(TINY_LLAMA, "cuda", seed=1)
    eng = LLMEngine(m, max_batch=16, max_model_len=1024, num_blocks=512, use_graphs=True)
    eng.warmup()
    backend = EngineBackend(eng, ChatTokenizer(TINY_LLAMA.vocab_size))
    fp = FeatureParams(ignore_eos=True)
    for f in (fp.answer, fp.smart, fp.summary, fp.suggest):
        f.max_new_tokens = 8
    port = free_port()
    srv = serve_llm(backend, port=port, bind="127.0.0.1", params=fp)
    ch = grpc.insecure_channel(f"127.0.0.1:{port}")
    try:
        s = make_stub(ch, LLM_SERVICE)
        msgs = [llm_pb.Message(sender="alice", content="ship it friday?"),
                llm_pb.Message(sender="bob", content="after review")]
        outs = []
        ths = [threading.Thread(target=lambda: outs.append(
            s.GetSmartReply(llm_pb.SmartReplyRequest(recent_messages=msgs), timeout=60)))
               for _ in range(12)]
        [t.start() for t in ths]
        [t.join() for t in ths]
        assert len(outs) == 12 and all(len(o.suggestions) == 3 for o in outs)
        assert eng.stats["decode_steps"] > 0
        with LocalCluster(3, data_root=str(tmp_path), llm_address=f"127.0.0.1:{port}") as c:
            L = c.leader()
            tok = c.login(L)
            st = c.stub(L)
            st.SendMessage(raft_pb.SendMessageRequest(token=tok, channel_id="general", content="hi"))
            r = st.SummarizeConversation(raft_pb.SummarizeRequest(token=tok, channel_id="general"))
            assert r.success and 1 <= len(r.key_points) <= 3
            r = st.GetLLMAnswer(raft_pb.LLMRequest(token=tok, query="status?"))
            assert r.success
    finally:
        ch.close()
        srv.stop(0).wait(10)
        backend.close()


def test_llm_server_serves_two_models_side_by_side_on_one_gpu(hipk):
    """``llm.server --serve smart=tiny-llama@0:mem=0.1 --serve summary=tiny-gemma@0:mem=0.1``:
    two engine groups (different model families) share one MI355X behind one service address,
    each inside its HBM budget; each RPC runs on its feature's engine (its engine's step
    counters move, the other's do not)."""
    import argparse

    from drtc_amd.llm import server as S
    from drtc_amd.utils.cluster import free_port

    args = argparse.Namespace(backend="engine", model="tiny-llama", tp=1, gpus=1, max_batch=8,
                              max_model_len=512, no_graphs=False, custom_allreduce=False,
                              in_process=True, hbm_budget=0.1)
    router = S.build_feature_backends(args, ["smart=tiny-llama@0:mem=0.1",
                                             "summary=tiny-gemma@0:mem=0.1"])
    smart, summ = router.route("smart"), router.route("summary")
    assert smart is not summ
    assert smart.engine.model.cfg.name == "tiny-llama"
    assert summ.engine.model.cfg.name == "tiny-gemma"
    fp = FeatureParams(ignore_eos=True)
    for f in (fp.answer, fp.smart, fp.summary, fp.suggest):
        f.max_new_tokens = 6
    port = free_port()
    srv = S.serve(router, port=port, bind="127.0.0.1", params=fp)
    ch = grpc.insecure_channel(f"127.0.0.1:{port}")
    try:
        stub = make_stub(ch, LLM_SERVICE)
        msgs = [llm_pb.Message(sender="a", content="lunch tomorrow?")]
        s0 = dict(smart.engine.stats), dict(summ.engine.stats)
        r = stub.GetSmartReply(llm_pb.SmartReplyRequest(request_id="1", recent_messages=msgs),
                               timeout=60)
        assert len(r.suggestions) == 3
        s1 = dict(smart.engine.stats), dict(summ.engine.stats)
        assert s1[0].get("prefill_steps", 0) > s0[0].get("prefill_steps", 0)
        assert s1[1].get("prefill_steps", 0) == s0[1].get("prefill_steps", 0)
        stub.SummarizeConversation(llm_pb.SummarizeRequest(request_id="2", messages=msgs,
                                                           max_length=200), timeout=60)
        s2 = dict(smart.engine.stats), dict(summ.engine.stats)
        assert s2[1].get("prefill_steps", 0) > s1[1].get("prefill_steps", 0)
        assert s2[0].get("prefill_steps", 0) == s1[0].get("prefill_steps", 0)
    finally:
        ch.close()
        srv.stop(0).wait(10)
        router.close()
