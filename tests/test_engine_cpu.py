"""Engine, model and op references on CPU (tiny configs)."""
import math

import pytest
import torch

from drtc_amd import ops
from drtc_amd.engine import ChatTokenizer, LLMEngine, SamplingParams
from drtc_amd.engine.block_allocator import BlockAllocator, PyBlockAllocator
from drtc_amd.models import (GEMMA_2B, LLAMA3_8B, LLAMA3_70B, MIXTRAL_8X7B, TINY_GEMMA, TINY_LLAMA,
                             TINY_MIXTRAL, TransformerLM)


@pytest.mark.parametrize("cfg", [TINY_LLAMA, TINY_GEMMA, TINY_MIXTRAL], ids=lambda c: c.name)
def test_engine_greedy_matches_full_forward(cfg):
    m = TransformerLM(cfg, "cpu", seed=3)
    eng = LLMEngine(m, max_batch=8, max_model_len=256, num_blocks=64, use_graphs=False)
    prompts = [[1, 5, 9], [1, 5, 9, 13, 22, 40, 41, 42], list(range(1, 70)), [7] * 33]
    reqs = eng.generate(prompts, SamplingParams.greedy(6, ignore_eos=True))
    for p, r in zip(prompts, reqs):
        ref = m.forward_reference([p + r.output_ids[:-1]])[0].float()
        got = ref[len(p) - 1:]
        for j, tok in enumerate(r.output_ids):
            assert got[j, tok] >= got[j].max() - 1e-3 * max(1.0, got[j].abs().max().item())
    assert eng.alloc.num_used == 0


@pytest.mark.parametrize("cfg", [TINY_LLAMA, TINY_MIXTRAL], ids=lambda c: c.name)
def test_packed_prefill_last_layer_pruning(cfg):
    """forward_prefill runs the last layer's o-projection / MLP / final norm
    on each sequence's last token only: the packed logits equal the last rows
    of the unpruned per-sequence forward (last_idx = every position)."""
    from drtc_amd.models.transformer import PrefillMeta

    m = TransformerLM(cfg, "cpu", seed=7)
    seqs = [list(range(1, 12)), [3, 4], list(range(5, 45))]
    cu = [0]
    for s in seqs:
        cu.append(cu[-1] + len(s))
    ids = torch.tensor(sum(seqs, []), dtype=torch.long)
    pos = torch.cat([torch.arange(len(s), dtype=torch.int32) for s in seqs])
    meta = PrefillMeta(positions=pos, slots=torch.full((cu[-1],), -1, dtype=torch.int64),
                       cu_seqlens=torch.tensor(cu, dtype=torch.int32), cu_host=cu, tiles=None,
                       last_idx=torch.tensor(cu[1:], dtype=torch.int64) - 1)
    got = m.forward_prefill(ids, meta, None).float()
    assert got.shape[0] == len(seqs)
    for j, s in enumerate(seqs):
        ref = m.forward_reference([s])[0][-1].float()
        assert (got[j] - ref).abs().max() <= 2e-2 * max(1.0, ref.abs().max().item())


def test_engine_preemption_and_recompute():
    m = TransformerLM(TINY_LLAMA, "cpu", seed=3)
    eng = LLMEngine(m, max_batch=8, max_model_len=512, num_blocks=12, use_graphs=False)
    reqs = eng.generate([list(range(1, 50))] * 6, SamplingParams(max_new_tokens=40, temperature=0.8,
                                                                 top_k=20, top_p=0.9, ignore_eos=True))
    assert all(len(r.output_ids) == 40 for r in reqs)
    assert eng.stats["preemptions"] > 0 and eng.alloc.num_used == 0
    assert eng._waiting_tokens == 0 and not eng.waiting  # incremental backlog count


def test_engine_stop_conditions():
    m = TransformerLM(TINY_LLAMA, "cpu", seed=4)
    eng = LLMEngine(m, max_batch=4, max_model_len=64, num_blocks=32, use_graphs=False)
    r = eng.generate([list(range(1, 60))], SamplingParams.greedy(100, ignore_eos=True))[0]
    assert r.finish_reason == "length" and r.num_tokens == 64
    first = eng.generate([[1, 2, 3]], SamplingParams.greedy(1, ignore_eos=True))[0].output_ids[0]
    r = eng.generate([[1, 2, 3]], SamplingParams(max_new_tokens=10, temperature=0.0, top_k=0, top_p=1.0,
                                                 stop_token_ids=(first,)))[0]
    assert r.finish_reason == "stop" and r.output_ids == [first]
    with pytest.raises(ValueError):
        eng.add_request(__import__("drtc_amd.engine", fromlist=["Request"]).Request([1] * 100))


def test_pipelined_decode_matches_synchronous():
    """Pipelined decode (step t+1 enqueued before step t is read, tokens fed
    back on the device) produces exactly the synchronous engine's outputs,
    including EOS/stop finishes discovered one step late (zombie slots),
    length finishes, block growth and mid-run admissions."""
    from drtc_amd.engine import Request

    m = TransformerLM(TINY_LLAMA, "cpu", seed=5)
    prompts = [list(range(1, 10 + 7 * i)) for i in range(6)]

    def run(pipeline: bool):
        eng = LLMEngine(m, max_batch=8, max_model_len=256, num_blocks=64, use_graphs=False)
        eng.pipeline = pipeline
        probe = eng.generate([prompts[0]], SamplingParams.greedy(5, ignore_eos=True))[0]
        stop_tok = probe.output_ids[3]  # request 0 stops on its 4th token
        params = [SamplingParams(max_new_tokens=12 + 5 * i, temperature=0.0, top_k=0, top_p=1.0,
                                 stop_token_ids=(stop_tok,) if i == 0 else ())
                  for i in range(6)]
        reqs = [eng.add_request(Request(list(p), prm)) for p, prm in zip(prompts[:4], params[:4])]
        for _ in range(6):  # a few decode steps, then two late arrivals
            eng.step()
        reqs += [eng.add_request(Request(list(p), prm)) for p, prm in zip(prompts[4:], params[4:])]
        while eng.has_work():
            eng.step()
        assert eng.alloc.num_used == 0 and not eng.running
        return [(r.output_ids, r.finish_reason) for r in reqs], eng.stats, stop_tok

    sync, st_sync, stop_tok = run(False)
    pipe, st_pipe, _ = run(True)
    assert pipe == sync
    assert sync[0][1] == "stop" and sync[0][0][-1] == stop_tok and stop_tok not in sync[0][0][:-1]
    assert all(reason == "length" for _, reason in sync[1:])
    assert st_pipe["decode_steps_pipelined"] > 0 and st_sync["decode_steps_pipelined"] == 0


def test_sorted_slots_match_unsorted(monkeypatch):
    """Slots reordered by context length before non-pipelined decode launches
    (LLMEngine._sort_slots, for the balanced attention item order) leave every greedy output
    unchanged - with stop-token finishes, staggered lengths, block growth, pipelined steps and
    mid-run admissions - and the order holds: longest context first."""
    from drtc_amd.engine import Request

    m = TransformerLM(TINY_LLAMA, "cpu", seed=6)
    prompts = [list(range(1, 5 + 11 * ((3 * i) % 7))) for i in range(7)]

    def run(sort_min: int):
        monkeypatch.setattr(LLMEngine, "SORT_SLOTS_MIN", sort_min)
        eng = LLMEngine(m, max_batch=8, max_model_len=256, num_blocks=96, use_graphs=False)
        probe = eng.generate([prompts[1]], SamplingParams.greedy(5, ignore_eos=True))[0]
        stop_tok = probe.output_ids[2]
        params = [SamplingParams(max_new_tokens=10 + 4 * i, temperature=0.0, top_k=0, top_p=1.0,
                                 stop_token_ids=(stop_tok,) if i == 1 else ())
                  for i in range(7)]
        reqs = [eng.add_request(Request(list(p), prm)) for p, prm in zip(prompts[:5], params[:5])]
        orders = []
        for _ in range(5):
            eng.step()
            n = len(eng.running)
            orders.append(list(eng.ctx[:n]))
        reqs += [eng.add_request(Request(list(p), prm)) for p, prm in zip(prompts[5:], params[5:])]
        while eng.has_work():
            eng.step()
        assert eng.alloc.num_used == 0 and not eng.running
        return [(r.output_ids, r.finish_reason) for r in reqs], eng.stats, orders

    plain, st_plain, _ = run(0)
    srt, st_srt, orders = run(1)
    assert srt == plain
    assert st_srt["slot_sorts"] > 0 and st_plain.get("slot_sorts", 0) == 0
    assert any(o == sorted(o, reverse=True) and len(set(o)) > 1 for o in orders)


@pytest.mark.parametrize("cfg", [TINY_LLAMA, TINY_MIXTRAL], ids=lambda c: c.name)
def test_mixed_steps_match_prefill_first(cfg):
    """Mixed scheduling (late prompts prefilled inside decode steps under a
    token budget, decode rows attended against the paged cache in the same
    forward) produces the prefill-first engine's tokens, with finishes, block
    growth and a budget that splits one arrival wave over several steps."""
    from drtc_amd.engine import Request

    m = TransformerLM(cfg, "cpu", seed=5)
    prompts = [list(range(1, 10 + 7 * i)) for i in range(7)]

    def run(mixed: bool):
        eng = LLMEngine(m, max_batch=8, max_model_len=256, num_blocks=64, use_graphs=False)
        eng.mixed, eng.mixed_tokens = mixed, 40
        params = [SamplingParams.greedy(10 + 4 * i, ignore_eos=True) for i in range(7)]
        reqs = [eng.add_request(Request(list(p), prm)) for p, prm in zip(prompts[:2], params[:2])]
        for _ in range(3):
            eng.step()
        reqs += [eng.add_request(Request(list(p), prm)) for p, prm in zip(prompts[2:], params[2:])]
        while eng.has_work():
            eng.step()
        assert eng.alloc.num_used == 0 and not eng.running
        return [r.output_ids for r in reqs], eng.stats

    ref, st_ref = run(False)
    got, st = run(True)
    assert st["mixed_steps"] >= 2 and st_ref["mixed_steps"] == 0
    assert got == ref


def test_tp2_matches_tp1_logits():
    """TP sharding math (head/column split + reductions) on one process by
    summing the shards' partial outputs by hand."""
    from drtc_amd.parallel.comm import ParallelContext

    cfg = TINY_LLAMA
    full = TransformerLM(cfg, "cpu", seed=9)

    class FakeTP(ParallelContext):
        pass

    shards = [TransformerLM(cfg, "cpu", pc=FakeTP(tp_size=2, tp_rank=r), seed=9) for r in range(2)]
    H = cfg.hidden_size
    x = torch.randn(5, H).to(torch.bfloat16)
    L0 = full.layers[0]
    y_full = torch.nn.functional.linear(ops.act_glu(torch.nn.functional.linear(x, L0["gate_up"])), L0["down"])
    y_tp = sum(torch.nn.functional.linear(ops.act_glu(torch.nn.functional.linear(x, s.layers[0]["gate_up"])),
                                          s.layers[0]["down"]).float() for s in shards)
    assert (y_full.float() - y_tp).abs().max() < 0.02
    q_full = torch.nn.functional.linear(x, L0["qkv"])
    q_cat = torch.cat([torch.nn.functional.linear(x, s.layers[0]["qkv"])[:, :s.sh.hq * cfg.head_dim]
                       for s in shards], -1)
    assert torch.equal(q_full[:, :cfg.num_heads * cfg.head_dim], q_cat)


def test_block_allocators_agree():
    for cls in (PyBlockAllocator, BlockAllocator):
        a = cls(10, 1)
        b = a.allocate(4)
        assert a.num_free == 5 and len(set(b)) == 4 and 0 not in b
        a.incref(b[:1])
        a.free(b)
        assert a.num_free == 8 and a.refcount(b[0]) == 1
        a.free(b[:1])
        assert a.num_free == 9
        with pytest.raises(Exception):
            a.free(b[:1])
        with pytest.raises(Exception):
            a.allocate(10)


def test_reference_ops_consistency():
    """The paged-decode reference equals the last row of the prefill
    reference when the KV cache holds the same sequence."""
    torch.manual_seed(0)
    Hq, Hkv, D, n = 4, 2, 64, 45
    qkv = torch.randn(n, (Hq + 2 * Hkv) * D).to(torch.bfloat16)
    pre = ops.prefill_attention_ref(qkv, [0, n], Hq, Hkv, D, D ** -0.5)
    bs = ops.KV_BLOCK
    nb = math.ceil(n / bs)
    kc = torch.zeros(nb + 1, Hkv, bs, D, dtype=torch.bfloat16)
    vc = torch.zeros(nb + 1, Hkv, D, bs, dtype=torch.bfloat16)
    slots = torch.arange(n) + bs  # blocks 1..nb
    cs = ops.build_rope_cache(64, D, 1e4)
    pos = torch.zeros(n, dtype=torch.int32)  # identity rotation
    ops.rope_kv_ref(qkv.clone(), pos, slots, cs, Hq, Hkv, D, kc, vc, bs)
    q = qkv[-1:, :Hq * D].reshape(1, Hq, D)
    bt = torch.arange(1, nb + 1, dtype=torch.int32)[None]
    dec = ops.paged_decode_ref(q, kc, vc, bt, torch.tensor([n], dtype=torch.int32), D ** -0.5)
    assert (dec.reshape(1, -1).float() - pre[-1:].float()).abs().max() < 0.02


def test_v_cache_block_layout():
    """V blocks are 8 groups of 4 tokens, dim-major inside a group: the
    per-token (decode) write and the whole-block (prefill) write agree, and
    the storage <-> token-major helpers are inverse."""
    from drtc_amd.ops.rope import v_block_storage, v_block_tokens

    torch.manual_seed(1)
    Hq, Hkv, D, bs = 2, 2, 64, ops.KV_BLOCK
    n = 45
    qkv = torch.randn(n, (Hq + 2 * Hkv) * D).to(torch.bfloat16)
    v = qkv[:, (Hq + Hkv) * D:].reshape(n, Hkv, D)
    vc_tok = torch.zeros(3, Hkv, D, bs, dtype=torch.bfloat16)
    kc = torch.zeros(3, Hkv, bs, D, dtype=torch.bfloat16)
    ops.rope_kv_ref(qkv.clone(), torch.zeros(n, dtype=torch.int32), torch.arange(n) + bs,
                    ops.build_rope_cache(8, D, 1e4), Hq, Hkv, D, kc, vc_tok, bs)
    vc_blk = torch.zeros_like(vc_tok)
    segs = (torch.tensor([0, bs]), torch.tensor([bs, n - bs]), torch.tensor([1, 2]))
    ops.kv_write_v_ref(vc_blk, qkv, *segs, Hq, Hkv, D)
    assert torch.equal(vc_tok, vc_blk)
    tok = v_block_tokens(vc_blk[1:])                      # [2, Hkv, bs, D]
    assert torch.equal(tok.permute(1, 0, 2, 3).reshape(Hkv, 2 * bs, D)[:, :n], v.transpose(0, 1))
    assert torch.equal(v_block_storage(tok), vc_blk[1:])
    # raw storage order: token t of dim d sits at (t // 4) * 4D + 4d + t % 4
    flat = vc_blk[1, 0].reshape(-1)
    for t, d in [(0, 0), (5, 3), (31, 63), (17, 40)]:
        assert flat[(t // 4) * 4 * D + 4 * d + t % 4] == v[t, 0, d]


def test_rope_llama3_scaling_and_sampler_ref():
    t = ops.build_rope_cache(16, 128, 5e5, {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                           "high_freq_factor": 4.0, "original_max_position_embeddings": 8192})
    assert t.shape == (16, 128) and torch.allclose(t[0, :64], torch.ones(64))
    logits = torch.randn(4, 50).to(torch.bfloat16)
    assert torch.equal(ops.sample_ref(logits).long(), logits.float().argmax(-1))
    out = ops.sample_ref(logits, torch.ones(4), torch.full((4,), 3, dtype=torch.int32), torch.ones(4))
    top3 = logits.float().topk(3, -1).indices
    assert (top3 == out.long()[:, None]).any(-1).all()


def test_model_configs_param_counts():
    assert abs(LLAMA3_8B.num_params() / 1e9 - 8.03) < 0.05
    assert abs(LLAMA3_70B.num_params() / 1e9 - 70.6) < 0.3
    assert abs(GEMMA_2B.num_params() / 1e9 - 2.51) < 0.05
    assert abs(MIXTRAL_8X7B.num_params() / 1e9 - 46.7) < 0.3
    assert LLAMA3_8B.kv_bytes_per_token() == 131072


def test_tokenizer_roundtrip_and_density():
    tok = ChatTokenizer(128256, 128000, 128001)
    for text in ["Hello team, lunch tomorrow?", "naïve café — ünïcode ✓", "line1\nline2\n\n- bullet"]:
        ids = tok.encode(text)
        assert ids[0] == 128000 and tok.decode(ids) == text
        assert all(0 <= i < 128256 for i in ids)
    words = "should we review the project plan tomorrow after the meeting".split()
    assert len(tok.encode(" ".join(words), add_bos=False)) == len(words)
    assert len(tok.id_to_tok) == 128256


def test_tracing_spans_and_serving_metrics(tmp_path):
    import json

    from drtc_amd.utils import tracing
    from drtc_amd.utils.metrics import METRICS

    METRICS.reset()
    tracing.clear()
    tracing.enable(True)
    try:
        eng = LLMEngine(TransformerLM(TINY_LLAMA, "cpu", seed=3), max_batch=4, max_model_len=256,
                        num_blocks=64, use_graphs=False)
        eng.generate([[1, 5, 6, 7], [1, 9]], SamplingParams.greedy(5, ignore_eos=True))
    finally:
        tracing.enable(False)
    names = {e["name"] for e in tracing.events()}
    assert {"engine.prefill", "engine.decode", "decode.eager"} <= names
    n = tracing.dump_chrome_trace(str(tmp_path / "trace.json"))
    data = json.load(open(tmp_path / "trace.json"))
    assert n == len(data["traceEvents"]) > 0 and all(e["ph"] == "X" for e in data["traceEvents"])
    snap = METRICS.snapshot()
    h = snap["histograms"]
    assert h["engine.ttft_s"]["count"] == 2 and h["engine.tpot_s"]["count"] == 2
    assert snap["counters"]["engine.generated_tokens"] == 10
    assert 0.0 <= snap["gauges"]["engine.kv_used_frac"] <= 1.0


def test_engine_abort_waiting_running_and_inflight():
    """abort(): a queued request leaves the queue, running ones (one of them in
    a pipelined in-flight step) finish with reason "abort" and free their slot
    and KV blocks; the other requests produce exactly the tokens they produce
    without the aborts."""
    from drtc_amd.engine import Request

    m = TransformerLM(TINY_LLAMA, "cpu", seed=6)
    prompts = [list(range(1, 12 + 5 * i)) for i in range(6)]

    def run(abort: bool):
        eng = LLMEngine(m, max_batch=4, max_model_len=256, num_blocks=64, use_graphs=False)
        prm = SamplingParams.greedy(24, ignore_eos=True)
        reqs = [eng.add_request(Request(list(p), prm)) for p in prompts]  # 2 wait (max_batch 4)
        for _ in range(4):
            eng.step()
        if abort:
            assert eng._inflight is not None and len(eng.waiting) == 2
            for i in (1, 3, 5):  # two running, one waiting
                eng.abort(reqs[i])
        while eng.has_work():
            eng.step()
        assert eng.alloc.num_used == 0 and not eng.running and eng._waiting_tokens == 0
        return reqs, eng.stats

    base, _ = run(False)
    got, st = run(True)
    assert st["aborted"] == 3
    for i in (1, 3, 5):
        assert got[i].finish_reason == "abort" and len(got[i].output_ids) < 24
    for i in (0, 2, 4):
        assert got[i].output_ids == base[i].output_ids
    assert len(got[5].output_ids) == 0  # aborted while queued


def test_backend_timeout_aborts_request():
    import time

    from drtc_amd.llm.backends import EngineBackend, GenerationError

    m = TransformerLM(TINY_LLAMA, "cpu", seed=6)
    eng = LLMEngine(m, max_batch=4, max_model_len=1024, num_blocks=64, use_graphs=False)
    be = EngineBackend(eng, ChatTokenizer(TINY_LLAMA.vocab_size))
    try:
        with pytest.raises(GenerationError):
            be.generate(["hello " * 20], SamplingParams.greedy(900, ignore_eos=True), timeout=0.05)
        deadline = time.time() + 20
        # (the request may be mid-prefill - neither queued nor running - when
        # the wait gives up; the abort lands at the engine's next step)
        while (eng.running or eng.waiting or eng.stats["aborted"] == 0) and time.time() < deadline:
            time.sleep(0.01)
        assert not eng.running and not eng.waiting and eng.stats["aborted"] == 1
        assert eng.alloc.num_used == 0
    finally:
        be.close()


def test_decode_kernel_choice_per_geometry():
    """The measured decode-attention variant table (profiles/r2g, r2l) at the
    engine's decode buckets: static per graph, chosen from (batch, kv heads, D)
    with the block-table width the runner passes (max_model_len / 32)."""
    from drtc_amd.ops.attention import decode_partitioning, decode_variant

    mb = 2048 // ops.KV_BLOCK
    assert decode_variant(1024, 8, 128, mb) == 3      # Llama-3-8B headline
    assert decode_variant(256, 8, 128, mb) == 3       # Mixtral / Llama-3-70B at batch 256
    assert decode_variant(1024, 1, 256, mb) == 2      # Gemma-2B headline batch
    assert decode_variant(256, 1, 256, mb) == 1
    assert decode_variant(16, 8, 128, mb) == 2        # small batch: context split over waves
    assert decode_variant(64, 8, 128, 4) == 1
    # one partition whenever the batch fills the chip; split contexts never on variant 1
    for B, hkv, D in ((1024, 8, 128), (256, 8, 128), (1024, 1, 256)):
        assert decode_partitioning(B, hkv, mb, D=D) == (mb, 1)
    bpp, parts = decode_partitioning(8, 8, mb)
    assert parts > 1 and decode_variant(8, 8, 128, mb) == 2


@pytest.mark.parametrize("mixed", [True, False], ids=["mixed", "prefill_first"])
def test_slot_bound_admission_in_groups(mixed):
    """With more queued requests than free batch slots, admission waits for
    ``admit_group`` free slots and takes them in one step (the in-between
    steps are pure decodes); tokens equal the trickle-admission engine's."""
    from drtc_amd.engine import Request

    m = TransformerLM(TINY_LLAMA, "cpu", seed=7)
    prompts = [list(range(1, 8 + 3 * i)) for i in range(20)]

    def run(group: int):
        eng = LLMEngine(m, max_batch=8, max_model_len=256, num_blocks=96, use_graphs=False)
        eng.mixed, eng.mixed_tokens, eng.admit_group = mixed, 4096, group
        sizes = []
        real = eng._admit

        def spy(*a, **k):
            b = real(*a, **k)
            if b:
                sizes.append((len(b), len(eng.running), len(eng.waiting)))
            return b

        eng._admit = spy
        reqs = [eng.add_request(Request(list(p), SamplingParams.greedy(3 + (5 * i) % 11,
                                                                       ignore_eos=True)))
                for i, p in enumerate(prompts)]
        while eng.has_work():
            eng.step()
        assert eng.alloc.num_used == 0 and not eng.running
        return [r.output_ids for r in reqs], sizes

    ref, trickle = run(1)
    got, grouped = run(4)
    assert got == ref
    # first admission fills the batch; later ones are groups of >= 4 (or the whole queue)
    assert grouped[0][0] == 8
    for n, running, waiting in grouped[1:]:
        assert n >= 4 or waiting == 0, grouped
    assert len(grouped) < len(trickle)


def test_pipelined_decode_continues_across_staggered_finishes():
    """Requests finishing one or two per step (continuous traffic) no longer
    drain the decode pipeline each time: they ride along as zombies (row
    computed, token discarded) up to ``admit_group``; tokens equal the
    synchronous engine's and every KV block comes back."""
    from drtc_amd.engine import Request

    m = TransformerLM(TINY_LLAMA, "cpu", seed=3)
    prompts = [list(range(2, 9 + 2 * i)) for i in range(10)]

    def run(pipeline: bool):
        eng = LLMEngine(m, max_batch=16, max_model_len=256, num_blocks=96, use_graphs=False)
        eng.pipeline, eng.admit_group = pipeline, 4
        reqs = [eng.add_request(Request(list(p), SamplingParams.greedy(6 + 2 * i, ignore_eos=True)))
                for i, p in enumerate(prompts)]
        while eng.has_work():
            eng.step()
        assert eng.alloc.num_used == 0 and not eng.running and not eng._zombies
        return [r.output_ids for r in reqs], eng.stats

    sync, st_sync = run(False)
    pipe, st_pipe = run(True)
    assert pipe == sync
    assert all(len(o) == 6 + 2 * i for i, o in enumerate(pipe))
    # a finish every other step: most decode steps stay pipelined
    assert st_pipe["decode_steps_pipelined"] >= st_pipe["decode_steps"] // 2, st_pipe


def test_request_wait_races_finish():
    """The completion Event is created by the first wait(): a finish that happens before,
    during or after that creation always wakes (or short-circuits) the waiter."""
    import threading

    from drtc_amd.engine.request import Request

    for trial in range(500):
        r = Request([1])
        res = []
        th = threading.Thread(target=lambda: res.append(r.wait(10)))
        if trial % 2:
            th.start()
            r.mark_finished("stop")
        else:
            r.mark_finished("stop")
            th.start()
        th.join(20)
        assert res == [True] and r.finish_reason == "stop"
    r = Request([1])
    assert r.wait(0.01) is False  # not finished: times out


def test_engine_loop_burst_gathering():
    """EngineLoop burst gathering (DRTC_BURST_GAP_MS): while requests keep arriving less than
    the gap apart, the loop lets them gather (bounded by burst_max_s) instead of stepping on
    the first one; a lone request waits at most the gap."""
    import collections
    import time

    from drtc_amd.engine.engine import EngineLoop

    class Stub:
        def __init__(self):
            self.waiting, self.running, self._inflight, self._aborts = [], [], None, []
            self._waiting_tokens, self.prefill_chunk_tokens, self.max_batch = 0, 16384, 1024
            self.stats, self.steps, self.batches = collections.Counter(), 0, []

        def add_request(self, r):
            self.waiting.append(r)
            self._waiting_tokens += 100

        def has_work(self):
            return bool(self.waiting)

        def step(self):
            self.steps += 1
            self.batches.append(len(self.waiting))
            self.waiting.clear()
            self._waiting_tokens = 0

    assert EngineLoop(Stub(), burst_gap_s=0.0).burst_gap_s == 0.0  # 0 disables it
    e = Stub()
    loop = EngineLoop(e, burst_gap_s=0.02, burst_max_s=0.5).start()
    try:
        for _ in range(20):  # a burst: 20 arrivals 1 ms apart -> gathered into few steps
            loop.submit(object())
            time.sleep(0.001)
        time.sleep(0.15)
        assert sum(e.batches) == 20 and e.steps <= 3, e.batches
        assert e.stats["burst_hold_us"] > 0
        t0 = time.perf_counter()
        loop.submit(object())  # a lone request: stepped once the gap has passed
        while e.waiting:
            time.sleep(0.001)
        assert time.perf_counter() - t0 < 0.2
    finally:
        loop.stop()


def test_mixed_admission_gathers_arrivals():
    """Arrival gathering for mixed steps (DRTC_ADMIT_MIN_TOKENS): while prompts keep arriving
    the engine decodes and holds them until a chunk's worth is queued, then admits them in ONE
    mixed step; the tokens equal the prefill-first engine's; off by default."""
    from drtc_amd.engine import Request

    m = TransformerLM(TINY_LLAMA, "cpu", seed=5)
    prompts = [list(range(1, 12 + 3 * i)) for i in range(6)]
    params = [SamplingParams.greedy(12, ignore_eos=True) for _ in prompts]

    def run(min_tokens: int, mixed: bool = True):
        eng = LLMEngine(m, max_batch=8, max_model_len=256, num_blocks=64, use_graphs=False)
        eng.mixed = mixed
        assert eng.admit_min_tokens == 0
        eng.admit_min_tokens, eng.admit_gap_s, eng.admit_max_delay_s = min_tokens, 10.0, 10.0
        reqs = [eng.add_request(Request(list(prompts[0]), params[0]))]
        eng.step()  # prefill of the first request
        for p, prm in zip(prompts[1:], params[1:]):  # a burst trickles in between steps
            reqs.append(eng.add_request(Request(list(p), prm)))
            eng.step()
        while eng.has_work():
            eng.step()
        return [r.output_ids for r in reqs], eng.stats

    ref, _ = run(0, mixed=False)
    got, st = run(sum(len(p) for p in prompts[1:]))
    assert got == ref
    assert st["mixed_steps"] == 1, dict(st)  # the whole burst admitted together
    _, st0 = run(0)
    assert st0["mixed_steps"] > 1


def test_prefill_step_comes_from_the_model_config(monkeypatch):
    """LLMEngine's prefill step is the model's ``prefill_chunk`` (Mixtral 32k, Llama-3-70B 36k,
    others 16k; profiles/r6t) unless DRTC_PREFILL_CHUNK overrides it; a small step splits a
    batch into several prefill launches with the same greedy outputs."""
    import dataclasses

    assert (LLAMA3_8B.prefill_chunk, MIXTRAL_8X7B.prefill_chunk, LLAMA3_70B.prefill_chunk) == \
        (16384, 32768, 36864)
    monkeypatch.delenv("DRTC_PREFILL_CHUNK", raising=False)
    prompts = [list(range(1, 30 + 7 * i)) for i in range(4)]
    outs = {}
    for chunk in (16384, 40):
        cfg = dataclasses.replace(TINY_LLAMA, prefill_chunk=chunk)
        m = TransformerLM(cfg, "cpu", seed=3)
        eng = LLMEngine(m, max_batch=4, max_model_len=256, num_blocks=64, use_graphs=False)
        assert eng.prefill_chunk_tokens == chunk
        reqs = eng.generate(prompts, SamplingParams.greedy(6, ignore_eos=True))
        outs[chunk] = [r.output_ids for r in reqs]
        assert eng.stats["prefill_steps"] == (1 if chunk > 1000 else 4)
    assert outs[16384] == outs[40]
    monkeypatch.setenv("DRTC_PREFILL_CHUNK", "96")
    eng = LLMEngine(TransformerLM(TINY_LLAMA, "cpu", seed=3), max_batch=4, max_model_len=256,
                    num_blocks=64, use_graphs=False)
    assert eng.prefill_chunk_tokens == 96
