"""Hand-written CDNA4 GEMM (csrc/kernels/gemm.hip) vs a PyTorch fp32 reference of the
same op, including the fused epilogues (residual add in place, SiLU / tanh-GELU
gating of a [gate; up] weight), split-K with the in-launch last-arriver combine,
row tails (M not a multiple of the 256-row tile), every pipeline variant, and
hipGraph replay (split-K counters re-arm themselves between replays)."""
import pytest
import torch
import torch.nn.functional as F

from drtc_amd.ops import gemm as G

pytestmark = pytest.mark.gpu


def _ref(x, w, epi, res):
    y = x.float() @ w.float().t()
    if epi == "residual":
        return y + res.float()
    if epi in ("silu", "gelu_tanh"):
        i = w.shape[0] // 2
        g, u = y[:, :i], y[:, i:]
        return (F.silu(g) if epi == "silu" else F.gelu(g, approximate="tanh")) * u
    return y


def _check(out, ref, tol=1.5e-2):
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= tol * max(scale, 1e-3), (err, scale)


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 7])
@pytest.mark.parametrize("epi", ["store", "residual", "silu", "gelu_tanh"])
@pytest.mark.parametrize("M,N,K,splitk", [(256, 256, 256, 1), (300, 512, 512, 2), (1, 768, 1024, 4),
                                          (1024, 1024, 2048, 2), (515, 256, 384, 3)])
def test_mfma_gemm_matches_fp32(hipk, variant, epi, M, N, K, splitk):
    g = torch.Generator(device="cuda").manual_seed(M * 31 + N + K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    nout = N // 2 if epi in ("silu", "gelu_tanh") else N
    res = torch.randn(M, nout, device="cuda", dtype=torch.bfloat16, generator=g) if epi == "residual" else None
    ref = _ref(x, w, epi, res)
    out = G.mfma_gemm(x, w, epi, residual=res, variant=variant, splitk=splitk)
    _check(out, ref)


@pytest.mark.parametrize("variant", [1, 5, 7])
def test_mfma_gemm_residual_in_place_and_strided(hipk, variant):
    """o / down projection adding into the residual stream in place; x is a
    column slice of a wider buffer (row stride > K)."""
    g = torch.Generator(device="cuda").manual_seed(7)
    big = torch.randn(640, 1024 + 256, device="cuda", dtype=torch.bfloat16, generator=g)
    x = big[:, :1024]
    w = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    h = torch.randn(640, 512, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = _ref(x, w, "residual", h)
    out = G.mfma_gemm(x, w, "residual", residual=h, out=h, variant=variant, splitk=2)
    assert out.data_ptr() == h.data_ptr()
    _check(h, ref)


@pytest.mark.parametrize("variant", [5, 7])
def test_mfma_gemm_graph_replay_splitk(hipk, variant):
    """Split-K inside a hipGraph: counters are re-armed by each tile's last
    arriver, so replays with new inputs stay exact."""
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(768, 1024, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    out = torch.empty(512, 768, device="cuda", dtype=torch.bfloat16)
    G.mfma_gemm(x, w, out=out, variant=variant, splitk=4)  # eager warm-up (workspace exists)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        G.mfma_gemm(x, w, out=out, variant=variant, splitk=4)
    for i in range(3):
        x.copy_(torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16, generator=g))
        gr.replay()
        torch.cuda.synchronize()
        _check(out, _ref(x, w, "store", None))


def test_mfma_gemm_rejects_bad_shapes(hipk):
    x = torch.randn(64, 100, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(256, 100, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        G.mfma_gemm(x, w)  # K % 64 != 0
    x = torch.randn(64, 128, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(200, 128, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        G.mfma_gemm(x, w)  # N % 256 != 0


# ---------------------------------------------------------------- medium-M decode GEMM
def _rel(out, ref):
    return (out.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)


@pytest.mark.parametrize("M", [17, 24, 33, 64, 100, 128, 150, 192, 256])
@pytest.mark.parametrize("N,K,S", [(4096, 4096, 8), (6144, 4096, 4), (2560, 2048, 8),
                                   (4096, 14336, 7), (4096, 14336, 14), (1024, 1024, 1)])
def test_midm_store_and_residual(hipk, M, N, K, S):
    """gemm_midm.hip vs fp32: plain store and residual-add epilogues, ragged M
    (column groups padded with zero rows), K splits summed by the reduce kernel."""
    g = torch.Generator(device="cuda").manual_seed(M + N + S)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    y = G.midm_gemm(x, w, splits=S)
    assert _rel(y, ref) < 1e-2
    res = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    ref_r = ref + res.float()
    out = G.midm_gemm(x, w, "residual", residual=res, splits=S)  # in place
    assert out.data_ptr() == res.data_ptr() and _rel(out, ref_r) < 1e-2


@pytest.mark.parametrize("act", ["silu", "gelu_tanh"])
@pytest.mark.parametrize("M", [24, 64, 128, 200, 256])
def test_midm_glu_epilogue(hipk, act, M):
    I, K = 2048, 2048
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(2 * I, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    y = (x.float() @ w.float().t()).to(torch.bfloat16).float()
    gte, up = y[:, :I], y[:, I:]
    a = F.silu(gte) if act == "silu" else F.gelu(gte, approximate="tanh")
    out = G.midm_gemm(x, w, act, splits=2)
    assert out.shape == (M, I) and _rel(out, a * up) < 1e-2


def test_midm_strided_input_and_graph_replay(hipk):
    """x as a row-strided view (decode attention output / norm slices), the
    kernel pair captured in a hipGraph and replayed bitwise."""
    g = torch.Generator(device="cuda").manual_seed(3)
    big = torch.randn(64, 6144, device="cuda", generator=g).to(torch.bfloat16)
    x = big[:, :4096]
    w = (torch.randn(4096, 4096, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    eager = G.midm_gemm(x, w, splits=8)
    assert _rel(eager, x.float() @ w.float().t()) < 1e-2
    out = torch.empty_like(eager)
    G.gemm_workspace(x.device)
    G.midm_gemm(x, w, out=out, splits=8)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        G.midm_gemm(x, w, out=out, splits=8)
    for _ in range(3):
        out.zero_()
        gr.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)


def test_linear_dispatches_midm_from_table(hipk):
    """ops.linear takes the medium-M kernel for a shape the tuning table marks
    (Llama-3-8B down at M = 64) and matches the library within bf16 rounding."""
    G.reset()
    ent = G._activate().get((64, 4096, 14336, 14336))
    if ent is None or not ent[2]:
        pytest.skip("no medium-M entry for this hipBLASLt version")
    g = torch.Generator(device="cuda").manual_seed(4)
    x = torch.randn(64, 14336, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(4096, 14336, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
    got = G.linear(x, w)
    assert _rel(got, x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("epi", ["store", "residual", "silu"])
@pytest.mark.parametrize("M,N,K,splitk", [(1024, 1024, 1024, 4), (300, 512, 2048, 2), (1024, 2048, 4096, 4),
                                          (700, 768, 1536, 4)])
def test_w4_reduce_scatter_splitk(hipk, epi, M, N, K, splitk):
    """gemm_w4's reduce-scatter split-K (variant 11): every slice finishes part of the tile
    from the others' write-through partials; counters re-arm for the next call (run twice)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + splitk)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    nout = N // 2 if epi == "silu" else N
    res = torch.randn(M, nout, device="cuda", dtype=torch.bfloat16, generator=g) if epi == "residual" else None
    ref = _ref(x, w, epi, res)
    for _ in range(2):
        r_in = res.clone() if res is not None else None
        out = G.mfma_gemm(x, w, epi, residual=r_in, out=r_in, variant=11, splitk=splitk)
        torch.cuda.synchronize()
        _check(out, ref)


# ------------------------------------------- split-K partial planes summed by the next norm
@pytest.mark.parametrize("M,N,K,sk", [(800, 512, 1024, 4), (1024, 4096, 14336, 4),
                                      (1024, 4096, 4096, 4), (777, 256, 512, 2)])
@pytest.mark.parametrize("gemma", [False, True])
def test_linear_partials_through_pending_norm(hipk, monkeypatch, M, N, K, sk, gemma):
    """gemm_w4 W4_PARTIAL + rmsnorm_partials (decode o / down at TP = 1): the pending norm
    of the planes equals norm(x @ w.T + residual) in fp32 within bf16 rounding, the
    residual stream is updated in place to h, and the pair replays from a hipGraph."""
    from drtc_amd import ops
    from drtc_amd.ops import gemm as Gm

    monkeypatch.setattr(Gm, "W4_PARTIAL", {(N, K): sk})
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    res = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    nw = (torch.rand(N, device="cuda", generator=g) + 0.5).to(torch.bfloat16)
    h_ref = x.float() @ w.float().t() + res.float()
    hf = h_ref.to(torch.bfloat16).float()
    ww = nw.float() + (1.0 if gemma else 0.0)
    out_ref = hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5) * ww
    part = ops.linear_partials(x, w)
    assert isinstance(part, ops.Partials) and part.sk == sk and tuple(part.shape) == (M, N)
    r1 = res.clone()
    p = ops.PendingNorm(part, r1, nw, 1e-5, gemma)
    out = p.materialize()
    torch.cuda.synchronize()
    assert p.stream().data_ptr() == r1.data_ptr()
    assert _rel(r1, h_ref) < 1e-2
    assert _rel(out, out_ref) < 2e-2
    # graph capture of the producer / consumer pair, replayed on fresh inputs
    r2 = res.clone()
    o2 = torch.empty_like(out)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        pp = ops.PendingNorm(ops.linear_partials(x, w), r2, nw, 1e-5, gemma)
        o2.copy_(pp.materialize())
    r2.copy_(res)
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(o2, out) and torch.equal(r2, r1)


def test_decode_with_partials_matches_reference(hipk, monkeypatch):
    """The engine's full-batch decode with o / down as split-K partial planes (batch 800 >=
    W4_PARTIAL_MIN_M: 3 full 256-row tiles + a 32-row one, hipGraphs): every greedy token is
    a maximiser (within bf16 tolerance) of the full-sequence reference forward's logits."""
    from drtc_amd.engine import LLMEngine, SamplingParams
    from drtc_amd.models import TINY_LLAMA, TransformerLM
    from drtc_amd.ops import gemm as Gm

    monkeypatch.setattr(Gm, "W4_PARTIAL", {(256, 256): 4, (256, 512): 4})
    prompts = [[1 + (7 * i + j) % 500 for j in range(5 + i % 23)] for i in range(800)]
    m = TransformerLM(TINY_LLAMA, "cuda", seed=21)
    eng = LLMEngine(m, max_batch=800, max_model_len=256, num_blocks=2048, use_graphs=True)
    reqs = eng.generate(prompts, SamplingParams.greedy(6, ignore_eos=True))
    bad = []
    for i, (p, r) in enumerate(zip(prompts, reqs)):
        ref = m.forward_reference([p + r.output_ids[:-1]])[0].float()
        for j, tok in enumerate(r.output_ids):
            row = ref[len(p) - 1 + j]
            if row[tok] < row.max() - 0.05 * max(1.0, row.abs().max().item()):
                bad.append((i, j))
    assert not bad, bad[:10]


# --------------------------------------------------- RMSNorm folded across a prefill layer
@pytest.mark.parametrize("M,N,K", [(4096, 512, 1024), (4500, 4096, 4096), (4096, 4096, 14336)])
def test_linear_residual_rinv(hipk, monkeypatch, M, N, K):
    """residual += x @ w.T with the next norm's row statistic: from the gemm_w4 epilogue
    (partial sums of squares, W4_RESIDUAL_SQ) or, for the library's long-K shape, from one
    read of the rows; h and rinv against fp32."""
    from drtc_amd import ops
    from drtc_amd.ops import gemm as Gm

    monkeypatch.setattr(Gm, "_fold_norm", True)

    g = torch.Generator(device="cuda").manual_seed(M + K)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(torch.bfloat16)
    res = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    h_ref = x.float() @ w.float().t() + res.float()
    h, rinv = ops.linear_residual_rinv(x, w, res, 1e-5)
    assert h.data_ptr() == res.data_ptr() and rinv is not None and rinv.shape == (M,)
    assert _rel(h, h_ref) < 1e-2
    r_ref = torch.rsqrt(h.float().pow(2).mean(-1) + 1e-5)  # of the stored (bf16) stream
    assert ((rinv - r_ref).abs() / r_ref).max().item() < 1e-4


@pytest.mark.parametrize("act", [None, "silu", "gelu_tanh"])
@pytest.mark.parametrize("gemma", [False, True])
def test_rs_linear_equals_norm_then_linear(hipk, act, gemma):
    """(h @ (W diag(g)).T) * rinv[row] (gemm_w4 *_RS epilogues, the norm weight folded into
    W) equals the projection of the materialised RMSNorm within bf16 rounding."""
    from drtc_amd import ops

    M, H, N = 4352, 1024, 1536 if act is None else 2048
    g = torch.Generator(device="cuda").manual_seed(7)
    h = torch.randn(M, H, device="cuda", generator=g).to(torch.bfloat16)
    nw = (torch.rand(H, device="cuda", generator=g) * 0.5 + (0.0 if gemma else 0.75)).to(torch.bfloat16)
    w = (torch.randn(N, H, device="cuda", generator=g) / H ** 0.5).to(torch.bfloat16)
    gam = nw.float() + (1.0 if gemma else 0.0)
    w_f = (w.float() * gam[None, :]).to(torch.bfloat16)
    rinv = torch.rsqrt(h.float().pow(2).mean(-1) + 1e-6)
    xn = h.float() * rinv[:, None] * gam[None, :]
    ref = xn @ w.float().t()
    if act is not None:
        I = N // 2
        gt, up = ref[:, :I], ref[:, I:]
        ref = (torch.nn.functional.silu(gt) if act == "silu"
               else torch.nn.functional.gelu(gt, approximate="tanh")) * up
    y = ops.rs_linear(h, w_f, rinv.contiguous(), act)
    assert y is not None
    assert _rel(y, ref) < 2e-2
    # the engine's path: a PendingNorm carrying rinv
    p = ops.PendingNorm(h, None, nw, 1e-6, gemma, rinv=rinv.contiguous())
    y2 = ops.norm_linear(p, w, w_f) if act is None else ops.norm_glu(p, w, act, w_f)
    assert torch.equal(y2, y) and p._out is None and p.stream().data_ptr() == h.data_ptr()


def test_prefill_with_folded_norms_matches_reference(hipk, monkeypatch):
    """A 2-layer model with H = 512 at a 4.4k-token prefill chunk: o / down leave the norm's
    row statistic, qkv / gate_up run on the residual stream with folded (non-unit) norm
    weights; logits agree with the unfolded HIP path and with the fp32 reference path."""
    from drtc_amd import ops
    from drtc_amd.models import TINY_LLAMA, TransformerLM
    from drtc_amd.models.transformer import PrefillMeta
    from drtc_amd.ops import gemm as Gm

    cfg = TINY_LLAMA.replace(hidden_size=512, intermediate_size=1024, num_heads=8,
                             num_kv_heads=8, head_dim=64, max_position=512)
    m = TransformerLM(cfg, "cuda", seed=4)
    g = torch.Generator().manual_seed(5)
    for L in m.layers:  # non-unit norm weights: the folded copies are real copies
        L["ln_in"].copy_((torch.rand(512, generator=g) + 0.5).to(torch.bfloat16))
        L["ln_post"].copy_((torch.rand(512, generator=g) + 0.5).to(torch.bfloat16))
    m.fold_norm_weights()
    assert m.layers[0]["qkv_n"].data_ptr() != m.layers[0]["qkv"].data_ptr()
    lens = [100 + (7 * i) % 60 for i in range(34)]
    T = sum(lens)
    assert T >= 4096
    ids = torch.randint(3, 500, (T,), device="cuda", dtype=torch.int64)
    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    pos = torch.cat([torch.arange(n) for n in lens]).to(torch.int32).cuda()
    last = torch.tensor(cu[1:], dtype=torch.int64, device="cuda") - 1

    def run():
        meta = PrefillMeta(positions=pos, slots=torch.full((T,), -1, dtype=torch.int64, device="cuda"),
                           cu_seqlens=torch.tensor(cu, dtype=torch.int32, device="cuda"), cu_host=cu,
                           tiles=None, last_idx=last, max_len=max(lens))
        return m.forward_prefill(ids, meta, None).float()

    monkeypatch.setattr(Gm, "_fold_norm", True)
    folded = run()
    monkeypatch.setattr(Gm, "_fold_norm", False)
    plain = run()
    with ops.reference_mode():
        ref = run()
    scale = max(1.0, ref.abs().max().item())
    assert (folded - plain).abs().max().item() < 0.03 * scale
    assert (folded - ref).abs().max().item() < 0.05 * scale


# ------------------------------------------------------ gemm_w4 persistent form (variant 15)
@pytest.mark.parametrize("epi", ["store", "residual", "silu", "gelu_tanh"])
@pytest.mark.parametrize("M,N,K", [(8192, 8192, 128), (4500, 4096, 576), (2300, 8192, 192),
                                   (300, 512, 512), (1, 768, 1024)])
def test_w4_persistent_matches_fp32(hipk, epi, M, N, K):
    """Persistent gemm_w4: min(tiles, CUs) workgroups walk the tile order and each tile's
    last two K steps stage the next tile's first two (odd and even K-tile counts, a partial
    last row tile, several tiles per workgroup, in-place residual)."""
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + 7 * K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    nout = N // 2 if epi in ("silu", "gelu_tanh") else N
    res = torch.randn(M, nout, device="cuda", dtype=torch.bfloat16, generator=g) if epi == "residual" else None
    ref = _ref(x, w, epi, res)
    if epi == "residual":
        out = G.mfma_gemm(x, w, epi, residual=res, out=res, variant=15)
        assert out.data_ptr() == res.data_ptr()
    else:
        out = G.mfma_gemm(x, w, epi, variant=15)
    _check(out, ref)
    # the same call on the per-tile form agrees bit for bit (same MFMA order per tile)
    if epi != "residual":
        _check(out, G.mfma_gemm(x, w, epi, variant=7).float(), tol=1e-6)


def test_w4_persistent_rejects_single_k_tile_and_splitk(hipk):
    x = torch.randn(512, 64, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(256, 64, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        G.mfma_gemm(x, w, variant=15)  # one K tile: nothing to prefetch across the seam
    x = torch.randn(512, 512, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        G.mfma_gemm(x, w, variant=15, splitk=2)
