"""Multi-process parallelism on CPU (gloo): EP all-to-all dispatch/combine and
TP forward equivalence with world_size 2 (the same code runs on RCCL)."""
import pytest
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ep_worker(rank, world, port, q):
    """Exact-split and static-capacity expert all-to-all on each rank's token
    shard vs the single-process MoE over all experts."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drtc_amd.parallel.expert_parallel import ep_moe_forward, moe_reference

    g = torch.Generator().manual_seed(0)
    E, H, I, k = 4, 64, 32, 2
    router = (torch.randn(E, H, generator=g) * 0.3).to(torch.bfloat16)
    gu = (torch.randn(E, 2 * I, H, generator=g) * 0.1).to(torch.bfloat16)
    dn = (torch.randn(E, H, I, generator=g) * 0.1).to(torch.bfloat16)
    x_all = torch.randn(world * 13, H, generator=g).to(torch.bfloat16)
    x = x_all[rank * 13:(rank + 1) * 13]
    el = E // world
    ref = moe_reference(x_all, router, gu, dn, k)[rank * 13:(rank + 1) * 13]
    from drtc_amd.parallel.expert_parallel import EpOverflow, worst_case_capacity

    errs = []
    gl, dl = gu[rank * el:(rank + 1) * el], dn[rank * el:(rank + 1) * el]
    for form in ("exact", "static", "cap"):
        ovf = EpOverflow("cpu")
        y = ep_moe_forward(x, router, gl, dl, k, form=form, overflow=ovf)
        errs.append((y.float() - ref.float()).abs().max().item())
        assert int(ovf.count) == 0, form  # cf 2 over 2 ranks = worst case here
    # a capacity factor too small for the routing: pairs are dropped and counted,
    # and the redo at worst-case capacity is exact again
    ovf = EpOverflow("cpu")
    y_small = ep_moe_forward(x, router, gl, dl, k, form="cap", overflow=ovf, cf=0.3)
    ovf.reduce(None)
    with worst_case_capacity():
        y_redo = ep_moe_forward(x, router, gl, dl, k, form="cap", cf=0.3)
    errs.append((y_redo.float() - ref.float()).abs().max().item())
    q.put((rank, errs, int(ovf.count), (y_small.float() - ref.float()).abs().max().item()))
    dist.destroy_process_group()


def test_ep_plan_semantics():
    """ep_plan: slots in (token, pick) order per owner, inverse maps, drops."""
    from drtc_amd.parallel.expert_parallel import ep_combine, ep_gather, ep_plan

    g = torch.Generator().manual_seed(3)
    T, k, world, e_local = 37, 2, 4, 2
    topi = torch.stack([torch.randperm(world * e_local, generator=g)[:k] for _ in range(T)])
    for cap in (T * k, 24, 8, 3):
        ovf = torch.zeros(1, dtype=torch.int32)
        dst, sp, se = ep_plan(topi, e_local, world, cap, ovf)
        owner = topi.reshape(-1) // e_local
        dropped = 0
        for d in range(world):
            pairs = torch.nonzero(owner == d).flatten()  # ascending = (token, pick) order
            for s, p in enumerate(pairs.tolist()):
                if s < cap:
                    assert dst[p] == d * cap + s and sp[d * cap + s] == p
                    assert se[d * cap + s] == topi.reshape(-1)[p]
                else:
                    assert dst[p] == -1
                    dropped += 1
            n_real = min(cap, pairs.numel())
            assert (sp[d * cap + n_real:(d + 1) * cap] == -1).all()
            assert (se[d * cap + n_real:(d + 1) * cap] == -1).all()
        assert int(ovf) == dropped
        x = torch.randn(T, 16, generator=g).to(torch.bfloat16)
        sx = ep_gather(x, sp, k)
        real = sp >= 0
        assert torch.equal(sx[real], x[sp[real].long() // k])
        w = torch.rand(T, k, generator=g)
        out = ep_combine(sx, dst, w, T, k)  # back == send rows: sum_j w_j x_t over kept picks
        keep = (dst >= 0).view(T, k).float()
        want = (x.float().unsqueeze(1) * (w * keep).unsqueeze(-1)).sum(1).to(torch.bfloat16)
        assert torch.equal(out, want)


def _tp_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drtc_amd.models import TINY_GEMMA, TINY_LLAMA, TINY_MIXTRAL, TransformerLM
    from drtc_amd.parallel.comm import ParallelContext

    res = {}
    for cfg in (TINY_LLAMA, TINY_GEMMA, TINY_MIXTRAL.replace(experts_per_token=4),
                TINY_MIXTRAL):
        full_m = TransformerLM(cfg, "cpu", seed=21)
        # 37 tokens: replicated TP path; 38 tokens: sequence-parallel prefill
        # (+ expert all-to-all for the MoE model)
        for ids, tag in ((list(range(3, 40)), "tp"), (list(range(3, 41)), "sp")):
            for ep_mode in (("a2a", "allreduce") if cfg.is_moe else ("a2a",)):
                pc = ParallelContext.from_world(tp=True, ep=cfg.is_moe)
                pc.ep_combine = ep_mode
                m = TransformerLM(cfg, "cpu", pc=pc, seed=21)
                out = m.forward_reference([ids])[0]
                full = full_m.forward_reference([ids])[0]
                key = f"{cfg.name}/k{cfg.experts_per_token}/{tag}/{ep_mode}"
                res[key] = ((out.float() - full.float()).abs().max().item()
                            / full.float().abs().max().item())
        assert pc.sp_ok(38) and not pc.sp_ok(37)
        if cfg.is_moe:
            # decode form: static-capacity (graph-capturable) all-to-all on
            # replicated tokens == the replicated + all-reduce form
            import drtc_amd.models.transformer as tr
            x = torch.randn(6, cfg.hidden_size, generator=torch.Generator().manual_seed(1)).to(
                torch.bfloat16)
            L = m.layers[0]
            tr._EP_DECODE_A2A = False
            y_ar = m._moe(L, x, decode=True)
            tr._EP_DECODE_A2A = True
            y_a2a = m._moe(L, x, decode=True)
            tr._EP_DECODE_A2A = False
            res[f"{cfg.name}/k{cfg.experts_per_token}/decode_a2a"] = (
                (y_a2a.float() - y_ar.float()).abs().max().item()
                / y_ar.float().abs().max().item())
    q.put((rank, res))
    dist.destroy_process_group()


def _tp_engine_worker(rank, world, port, q):
    """TP=2 engines whose ranks see different free memory: the block count is
    agreed (MIN over the group), so the lockstep schedulers admit and preempt
    identically and produce the same tokens (engine.py:71)."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drtc_amd.engine import LLMEngine, SamplingParams
    from drtc_amd.engine.kv_cache import PagedKVCache
    from drtc_amd.models import TINY_LLAMA, TransformerLM
    from drtc_amd.parallel.comm import ParallelContext

    # rank-dependent "free HBM": 12 blocks on rank 0, 40 on rank 1
    PagedKVCache.auto_num_blocks = staticmethod(lambda *a, **k: 12 + 28 * rank)
    pc = ParallelContext.from_world(tp=True)
    m = TransformerLM(TINY_LLAMA, "cpu", pc=pc, seed=5)
    eng = LLMEngine(m, max_batch=8, max_model_len=256, use_graphs=False)
    prompts = [list(range(1 + i, 40 + 3 * i)) for i in range(6)]
    reqs = eng.generate(prompts, SamplingParams.greedy(48, ignore_eos=True))
    q.put((rank, {"blocks": eng.kv.num_blocks, "preempt": eng.stats["preemptions"],
                  "out": [r.output_ids for r in reqs]}))
    dist.destroy_process_group()


def _tp_mixed_worker(rank, world, port, q):
    """TP=2 (and TP=2 x EP=2 for the MoE model) engines driven in lockstep with
    late arrivals: prompts that arrive while others decode are prefilled in
    mixed prefill+decode steps (all-reduced partial sums over both row kinds).
    Both ranks must agree, and the tokens must equal the same TP group run
    prefill-first (and, for the dense model, a TP=1 engine; under EP a
    near-tied top-2 routing can flip between TP=1 and TP=2 sums whatever the
    scheduler)."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drtc_amd.engine import LLMEngine, Request, SamplingParams
    from drtc_amd.models import TINY_LLAMA, TINY_MIXTRAL, TransformerLM
    from drtc_amd.parallel.comm import ParallelContext

    res = {}
    for cfg in (TINY_LLAMA, TINY_MIXTRAL):
        prompts = [list(range(2 + i, 30 + 5 * i)) for i in range(6)]

        def drive(eng, mixed=True):
            eng.mixed, eng.mixed_tokens = mixed, 48
            prm = SamplingParams.greedy(16, ignore_eos=True)
            reqs = [eng.add_request(Request(list(p), prm)) for p in prompts[:2]]
            for _ in range(3):
                eng.step()
            reqs += [eng.add_request(Request(list(p), prm)) for p in prompts[2:]]
            while eng.has_work():
                eng.step()
            return [r.output_ids for r in reqs], eng.stats["mixed_steps"]

        pc = ParallelContext.from_world(tp=True, ep=cfg.is_moe)
        model = TransformerLM(cfg, "cpu", pc=pc, seed=8)
        kw = dict(max_batch=8, max_model_len=256, num_blocks=64, use_graphs=False)
        tp_out, mixed = drive(LLMEngine(model, **kw))
        tp_pf, _ = drive(LLMEngine(model, **kw), mixed=False)
        ref_out, _ = drive(LLMEngine(TransformerLM(cfg, "cpu", seed=8), **kw))
        res[cfg.name] = {"tp": tp_out, "tp_prefill_first": tp_pf, "ref": ref_out,
                         "mixed": mixed, "dense": not cfg.is_moe}
    q.put((rank, res))
    dist.destroy_process_group()


def _ep_redo_worker(rank, world, port, q):
    """EP=2 Mixtral engines with a capacity factor far too small for the
    routing: every overflowing prefill chunk and (pipelined) decode step is
    redone at worst-case capacity, so the tokens equal a run that never
    overflows; both ranks agree."""
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import drtc_amd.parallel.expert_parallel as ep
    from drtc_amd.engine import LLMEngine, Request, SamplingParams
    from drtc_amd.models import TINY_MIXTRAL, TransformerLM
    from drtc_amd.parallel.comm import ParallelContext

    pc = ParallelContext.from_world(tp=True, ep=True)
    model = TransformerLM(TINY_MIXTRAL, "cpu", pc=pc, seed=4)
    prompts = [list(range(5 + i, 29 + 3 * i)) for i in range(6)]
    res = {}
    # greedy, and sampled (t > 0: a redo must reuse the RNG counter of the step's first run)
    for mode, prm in (("greedy", SamplingParams.greedy(12, ignore_eos=True)),
                      ("sampled", SamplingParams(max_new_tokens=12, temperature=0.9, top_k=8,
                                                 top_p=0.95, ignore_eos=True))):
        for cf in (8.0, 0.2):
            ep.EP_CF = cf
            eng = LLMEngine(model, max_batch=8, max_model_len=256, num_blocks=64,
                            use_graphs=False)
            reqs = [eng.add_request(Request(list(p), prm)) for p in prompts]
            while eng.has_work():
                eng.step()
            res[(mode, cf)] = {"out": [r.output_ids for r in reqs],
                               "prefill_redo": eng.stats.get("ep_redo_steps", 0),
                               "decode_redo": eng.runner.redo_steps,
                               "pipelined": eng.stats["decode_steps_pipelined"]}
    q.put((rank, res))
    dist.destroy_process_group()


def _capped(fn, rank, world, port, q):
    # each rank gets its share of the CPUs: 2 ranks x all cores oversubscribe
    # the machine (and more so under pytest -n), which made the mixed-step test
    # miss its queue deadline
    torch.set_num_threads(max(1, (os.cpu_count() or 2) // (2 * world)))
    fn(rank, world, port, q)


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_capped, args=(fn, r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=480) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_ep_all_to_all_matches_reference():
    res = _run(_ep_worker)
    for rank, errs, dropped, err_small in res:
        assert max(errs) == 0.0, (rank, errs)  # same bf16 roundings, fp32 combine
        assert dropped > 0 and err_small > 0, (rank, dropped)
    assert res[0][2] == res[1][2]  # the EP-group sum: the same redo decision everywhere


def test_tp_and_ep_model_forward_matches_single_process():
    for rank, res in _run(_tp_worker):
        for name, rel in res.items():
            assert rel < 0.03, (rank, name, rel)


def test_tp_engines_agree_on_kv_blocks_under_preemption():
    res = dict(_run(_tp_engine_worker))
    assert res[0]["blocks"] == res[1]["blocks"] == 12
    assert res[0]["preempt"] == res[1]["preempt"] > 0
    assert res[0]["out"] == res[1]["out"]


def test_tp_mixed_prefill_decode_steps_match_tp1():
    res = dict(_run(_tp_mixed_worker))
    for name in res[0]:
        a, b = res[0][name], res[1][name]
        assert a["mixed"] == b["mixed"] >= 2, name
        assert a["tp"] == b["tp"], name
        assert a["tp"] == a["tp_prefill_first"], name
        if a["dense"]:
            assert a["tp"] == a["ref"], name


def test_ep_capacity_overflow_redo_is_exact():
    res = dict(_run(_ep_redo_worker))
    for mode in ("greedy", "sampled"):
        for rank in (0, 1):
            big, small = res[rank][(mode, 8.0)], res[rank][(mode, 0.2)]
            assert big["prefill_redo"] == big["decode_redo"] == 0
            assert small["prefill_redo"] > 0 and small["decode_redo"] > 0, small
            assert small["pipelined"] > 0
            assert small["out"] == big["out"], mode
        assert res[0][(mode, 0.2)]["out"] == res[1][(mode, 0.2)]["out"]
    # the sampled run really samples (not the greedy tokens)
    assert res[0][("sampled", 8.0)]["out"] != res[0][("greedy", 8.0)]["out"]


def test_tp_device_checks():
    """A TP group on real GPUs: distinct devices, in range, every pair peer-accessible."""
    from drtc_amd.parallel.tp_engine import check_devices

    check_devices([0, 1, 2, 3], 8, lambda a, b: True)
    with pytest.raises(RuntimeError, match="share a device"):
        check_devices([0, 0], 8, lambda a, b: True)
    with pytest.raises(RuntimeError, match="out of range"):
        check_devices([6, 8], 8, lambda a, b: True)
    with pytest.raises(RuntimeError, match="peer access"):
        check_devices([0, 1, 2], 8, lambda a, b: {a, b} != {1, 2})
