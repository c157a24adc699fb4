"""Hand-written CDNA4 GEMMs vs a PyTorch fp32 reference of the same op: gemm_w4.hip (the
4-wave MFMA GEMM) with every fused epilogue (residual add in place, SiLU / tanh-GELU gating
of a [gate; up] weight), split-K with the in-launch last-arriver combine in both tile
orders, row tails (M not a multiple of the 256-row tile), the persistent forms and hipGraph
replay (split-K counters re-arm themselves between replays); gemm_midm.hip; and the
projection router of ops.linear."""
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


@pytest.mark.parametrize("variant", [7, 9])
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


@pytest.mark.parametrize("variant", [7, 9])
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


@pytest.mark.parametrize("variant", [7, 9])
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
@pytest.mark.parametrize("M,N,K,splitk,gm", [(1024, 4096, 4096, 4, -4), (1024, 4096, 4096, 2, -2),
                                             (512, 2048, 1024, 8, -2), (1000, 1024, 2048, 4, -1)])
def test_w4_splitk_xcd_slice_order(hipk, epi, M, N, K, splitk, gm):
    """Split-K in the K-slice-by-XCD tile order (group_m < 0: the block labels b % 8 split
    into K slices x tile subsets): every (tile, slice) pair is computed exactly once whatever
    the placement; counters re-arm (run twice)."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + splitk)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    nout = N // 2 if epi == "silu" else N
    res = torch.randn(M, nout, device="cuda", dtype=torch.bfloat16, generator=g) if epi == "residual" else None
    ref = _ref(x, w, epi, res)
    for _ in range(2):
        r_in = res.clone() if res is not None else None
        out = G.mfma_gemm(x, w, epi, residual=r_in, out=r_in, variant=7, splitk=splitk,
                          group_m=gm)
        torch.cuda.synchronize()
        _check(out, ref)


@pytest.mark.parametrize("epi", ["store", "residual", "silu", "gelu_tanh"])
@pytest.mark.parametrize("M,N,K,splitk,gm", [(256, 8192, 8192, 8, -1), (192, 8192, 4096, 8, 1),
                                             (1024, 4096, 4096, 4, -4), (300, 1024, 2048, 2, 4),
                                             (1000, 2048, 1024, 4, -2)])
def test_w4_splitk_parallel_combine(hipk, epi, M, N, K, splitk, gm):
    """Split-K with the parallel combine (variants 11 / 13): every slice publishes its fp32
    tile write-through, waits for the others and finishes a row band of the tile (row tails
    past M, gated tiles, in-place residual); counters re-arm, so repeated calls and a
    hipGraph replay stay exact."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + splitk)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    nout = N // 2 if epi in ("silu", "gelu_tanh") else N
    res = torch.randn(M, nout, device="cuda", dtype=torch.bfloat16, generator=g) if epi == "residual" else None
    ref = _ref(x, w, epi, res)
    for v in (11, 13):
        r_in = res.clone() if res is not None else None
        out = G.mfma_gemm(x, w, epi, residual=r_in, out=r_in, variant=v, splitk=splitk,
                          group_m=gm)
        torch.cuda.synchronize()
        _check(out, ref)
    if epi == "store":
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            G.mfma_gemm(x, w, out=out, variant=11, splitk=splitk, group_m=gm)
        for _ in range(3):
            out.zero_()
            gr.replay()
            torch.cuda.synchronize()
            _check(out, ref)


def test_w4_splitk_parallel_combine_rejects(hipk):
    x = torch.randn(1024, 4096, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(8192, 4096, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        G.mfma_gemm(x, w, variant=11, splitk=1)  # a split-K form
    with pytest.raises(RuntimeError):
        G.mfma_gemm(x, w, variant=11, splitk=8)  # 128 tiles x 8 > the CUs: not co-resident


# ------------------------------------------------------ gemm_w4 persistent forms (15 / 31)
@pytest.mark.parametrize("variant", [15, 31, 47, 63])
@pytest.mark.parametrize("epi", ["store", "residual", "silu", "gelu_tanh"])
@pytest.mark.parametrize("M,N,K", [(8192, 8192, 128), (4500, 4096, 576), (2300, 8192, 192),
                                   (1024, 4096, 1088), (2048, 2048, 512)])
def test_w4_persistent_matches_fp32(hipk, variant, epi, M, N, K):
    """Persistent gemm_w4: min(tiles, CUs) workgroups walk the tile order and each tile's
    last two K steps stage the next tile's first two (odd and even K-tile counts, a partial
    last row tile, several tiles per workgroup, in-place residual).  Variant 31 runs each
    XCD label's K loop from its own eighth of K (wrapping), so its sums are reordered."""
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + 7 * K)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    nout = N // 2 if epi in ("silu", "gelu_tanh") else N
    res = torch.randn(M, nout, device="cuda", dtype=torch.bfloat16, generator=g) if epi == "residual" else None
    ref = _ref(x, w, epi, res)
    if epi == "residual":
        out = G.mfma_gemm(x, w, epi, residual=res, out=res, variant=variant)
        assert out.data_ptr() == res.data_ptr()
    else:
        out = G.mfma_gemm(x, w, epi, variant=variant)
    _check(out, ref)
    # the same call on the per-tile form agrees bit for bit (same MFMA order per tile)
    if epi != "residual" and variant == 15:
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
    # 2 x 1 tiles, fewer than one per XCD label: the plain persistent form runs
    y = G.mfma_gemm(x, w, variant=31)
    torch.cuda.synchronize()
    _check(y, _ref(x, w, "store", None))


# ------------------------------------------------------------------ projection router
def test_router_covers_every_served_decode_shape(hipk):
    """Every projection ops.linear serves for the TP = 1 models, at every hipGraph bucket up
    to the LLM server's default batch, the default batch itself and off-bucket batches,
    resolves to a hand kernel, a tuned library solution, or - at a bucket the tuner measured
    it fastest - the library's heuristic pick; an off-bucket M takes its bucket-above route
    (never an unmeasured path), and every prefill shape the hand GEMM covers takes it."""
    from drtc_amd.llm.server import default_max_batch
    from drtc_amd.models import get_config

    G.reset()
    for name in ("llama-3-8b", "gemma-2b", "mixtral-8x7b", "llama-3-70b"):
        cfg = get_config(name)
        H, D = cfg.hidden_size, cfg.head_dim
        shapes = {"qkv": ((cfg.num_heads + 2 * cfg.num_kv_heads) * D, H),
                  "o": (H, cfg.num_heads * D), "lm_head": (cfg.vocab_size, H)}
        if not cfg.is_moe:
            shapes["down"] = (H, cfg.intermediate_size)
            shapes["gate_up"] = (2 * cfg.intermediate_size, H)
        top = default_max_batch(name)
        ms = sorted({b for b in G.DECODE_BUCKETS if b <= top} | {top, 208, 1000, 16384})
        for proj, (N, K) in shapes.items():
            for M in ms:
                if proj == "gate_up" and M >= G.W4_GLU_MIN_M:
                    continue  # the fused-GLU hand GEMM (norm_glu), not linear
                kind, arg = G.route(M, N, K, K)
                assert kind in ("w4", "lt", "skinny", "midm", "xd", "torch"), (name, proj, M, kind)
                if G.w4_shape_ok(M, N, K):
                    assert kind == "w4", (name, proj, M, kind)
                elif M <= G.DECODE_MAX_M and M not in G.DECODE_BUCKETS:
                    Mb = next(b for b in G.DECODE_BUCKETS if b >= M)
                    kb = G.route(Mb, N, K, K)
                    # the bucket's kernel, or the heuristic where its solution rejects this M
                    assert kind == kb[0] or (kind == "torch" and kb[0] in ("lt", "skinny")), \
                        (name, proj, M, kind, Mb, kb)
                ent = G._activate().get((M, N, K, K))
                if ent is not None and (ent[0] >= 0 or ent[1] or ent[2] or ent[3]):
                    assert kind != "torch", (name, proj, M, ent)  # a measured winner is used


def test_linear_off_bucket_matches_fp32(hipk):
    """An off-bucket decode batch (M = 208, Llama-3-70B down shape scaled down to the
    8B's) runs its bucket-above route and matches fp32."""
    g = torch.Generator(device="cuda").manual_seed(9)
    for M, N, K in ((208, 4096, 14336), (1000, 6144, 4096), (200, 4096, 4096)):
        x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16)
        assert _rel(G.linear(x, w), x.float() @ w.float().t()) < 1e-2, (M, N, K)


# ---------------------------------------------------------------- gemm_xd.hip (decode tiles)
@pytest.mark.parametrize("epi", ["store", "residual"])
@pytest.mark.parametrize("form", sorted(G.XD_FORMS))
@pytest.mark.parametrize("M,N,K", [(1024, 768, 4096), (1000, 1536, 896), (77, 384, 1024),
                                   (512, 3072, 1408), (129, 1152, 2048), (300, 768, 640)])
def test_xd_gemm_matches_fp32(hipk, epi, form, M, N, K):
    if not G.xd_supported(M, N, K, form):
        pytest.skip("shape outside the form's tile grid")
    g = torch.Generator(device="cuda").manual_seed(M * 7 + N + K + form)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g) \
        if epi == "residual" else None
    ref = _ref(x, w, epi, res)
    out = G.xd_gemm(x, w, epi, residual=res, form=form)
    torch.cuda.synchronize()
    _check(out, ref)
    if form % 10 > 1:  # split-K: counters re-armed, a second call gives the same bits
        out2 = G.xd_gemm(x, w, epi, residual=res, form=form)
        torch.cuda.synchronize()
        assert torch.equal(out, out2)
        assert int(G.gemm_workspace(x.device)[1][:2 * 256 + 1].abs().sum()) == 0


@pytest.mark.parametrize("act", ["silu", "gelu_tanh"])
@pytest.mark.parametrize("form", [121, 141, 161, 241, 242, 243, 261, 264, 281, 283])
@pytest.mark.parametrize("M,I,K", [(256, 1536, 1024), (200, 768, 1600), (1024, 384, 832)])
def test_xd_gemm_glu_matches_fp32(hipk, act, form, M, I, K):
    if not G.xd_supported(M, I, K, form, glu=True):
        pytest.skip("shape outside the form's tile grid")
    g = torch.Generator(device="cuda").manual_seed(M + I + K + form)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(2 * I, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    out = G.xd_gemm(x, w, act, form=form)
    torch.cuda.synchronize()
    _check(out, _ref(x, w, act, None))


@pytest.mark.parametrize("epi", ["store", "residual", "silu"])
@pytest.mark.parametrize("form", [1141, 1161, 1241, 1244, 1261, 1281, 1282])
def test_xd_gemm_nontemporal_weights_match_fp32(hipk, epi, form):
    """Forms with non-temporal weight loads (form + 1000): same numerics as the plain form."""
    glu = epi == "silu"
    M, N, K = 256, 1536, 2048
    assert G.xd_supported(M, N, K, form, glu) and G.xd_nt(form)
    g = torch.Generator(device="cuda").manual_seed(form)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(2 * N if glu else N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g) \
        if epi == "residual" else None
    out = G.xd_gemm(x, w, epi, residual=res.clone() if res is not None else None, form=form)
    plain = G.xd_gemm(x, w, epi, residual=res.clone() if res is not None else None,
                      form=form - 1000)
    torch.cuda.synchronize()
    _check(out, _ref(x, w, epi, res))
    assert torch.equal(out, plain)


def test_xd_nontemporal_forms_rejected_outside_built_tiles():
    assert not G.xd_supported(256, 1536, 2048, 1121)  # 128 x 64 tile: no nt build
    assert not G.xd_supported(256, 1536, 2048, 2241)


@pytest.mark.parametrize("form", [143, 145, 247, 268, 285])
def test_xd_gemm_uneven_splitk(hipk, form):
    """K tiles that the slices do not divide evenly (K / 64 = 61 over 3, 5, 7, 8 slices)."""
    M, N, K = 384, 768, 61 * 64
    g = torch.Generator(device="cuda").manual_seed(form)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    out = G.xd_gemm(x, w, form=form)
    torch.cuda.synchronize()
    _check(out, _ref(x, w, "store", None))


@pytest.mark.parametrize("form", [141, 242])
def test_xd_gemm_strided_input_in_place_residual_and_graph(hipk, form):
    M, N, K = 640, 4096, 2048
    g = torch.Generator(device="cuda").manual_seed(5)
    big = torch.randn(M, K + 192, device="cuda", dtype=torch.bfloat16, generator=g)
    x = big[:, 64:64 + K]  # row stride K + 192
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    res = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, generator=g)
    ref = _ref(x, w, "residual", res)
    r = res.clone()
    G.xd_gemm(x, w, "residual", residual=r, out=r, form=form)  # in place into the residual
    torch.cuda.synchronize()
    _check(r, ref)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        G.xd_gemm(x, w, out=out, form=form)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):
            G.xd_gemm(x, w, out=out, form=form)
    for _ in range(3):
        out.zero_()
        gr.replay()
    torch.cuda.synchronize()
    _check(out, _ref(x, w, "store", None))


def test_xd_gemm_rejects_bad_shapes(hipk):
    def call(M, N, K, epi=0, mt=1, nf=4, sk=1, ws=None):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        slab, cnt = ws or (None, None)
        return hipk.gemm_xd(y.data_ptr(), x.data_ptr(), w.data_ptr(), 0, M, N, K, K, K, N, 0,
                            epi, mt, nf, sk, slab.data_ptr() if slab is not None else 0,
                            slab.numel() * 4 if slab is not None else 0,
                            cnt.data_ptr() if cnt is not None else 0,
                            cnt.numel() if cnt is not None else 0, 0)
    assert call(64, 200, 512, nf=2) == -1        # N not a multiple of the tile width
    assert call(64, 256, 512, nf=3) == -1        # no such form
    assert call(64, 256, 512, sk=9) == -1        # at most 8 slices
    assert call(64, 40, 512, epi=2, nf=2) == -1  # gated: N not a multiple of 16 nf
    assert call(64, 256, 256, nf=4) == -1        # K / 64 must exceed the ring depth (4)
    assert call(64, 256, 512, epi=1, nf=2) == -1  # residual epilogue without a residual
    assert call(256, 256, 1024, mt=2, nf=4, sk=2) == -2  # split-K without a workspace


def test_norm_glu_takes_tuned_xd_form(hipk, monkeypatch):
    """A decode batch whose table entry carries a gated gemm_xd form runs it through
    ops.norm_glu (no act_glu pass) and matches the fp32 reference of norm + GLU."""
    from drtc_amd import ops

    M, I, K = 256, 1536, 1024
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    nw = (1 + 0.1 * torch.randn(K, device="cuda", generator=g)).to(torch.bfloat16)
    w = torch.randn(2 * I, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    G.reset()
    tab = dict(G._activate())
    tab[(M, 2 * I, K, K)] = (-1, 0, 0, 0, 242)
    monkeypatch.setattr(G, "_table", tab)
    calls = []
    real = G.xd_gemm
    monkeypatch.setattr(G, "xd_gemm", lambda *a, **k: calls.append(k.get("form")) or real(*a, **k))
    out = ops.norm_glu(ops.PendingNorm(x, None, nw, 1e-5, False), w, "silu")
    torch.cuda.synchronize()
    assert calls == [242]
    xn = ops.rmsnorm_ref(x, nw, 1e-5).to(torch.bfloat16)
    _check(out, _ref(xn, w, "silu", None))
    G.reset()


# ------------------------------------------------------------ split-K fault visibility
@pytest.mark.parametrize("kind", ["xd", "w4"])
def test_splitk_timeout_is_raised_and_next_gemm_is_correct(hipk, kind):
    """A split-K combine whose poll for the other slices times out (forced here with a
    negative spin bound) records the fault in the workspace's LAST counter - outside every
    launch's ticket range - and leaves its counters un-armed; check_splitk_fault raises and
    resets them, after which the same GEMM is correct again."""
    g = torch.Generator(device="cuda").manual_seed(99)
    x = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(1024, 1024, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    ref = _ref(x, w, "store", None)

    def run():
        if kind == "xd":
            return G.xd_gemm(x, w, form=242)           # 256 x 128 tiles, 2 K slices
        return G.mfma_gemm(x, w, variant=11, splitk=2)  # parallel combine
    G.check_splitk_fault()  # a clean start
    prev = G.set_splitk_spin_limit(-1)
    try:
        run()
        torch.cuda.synchronize()
    finally:
        G.set_splitk_spin_limit(prev)
    with pytest.raises(G.SplitKFault):
        G.check_splitk_fault(torch.device("cuda"))
    G.check_splitk_fault()  # cleared by the raise
    _check(run(), ref)
    G.check_splitk_fault()
    # the fault word sits at a fixed slot: a later GEMM with more tiles (its ticket range
    # covers the old 2 * tiles slot) is unaffected
    x2 = torch.randn(1024, 1024, device="cuda", dtype=torch.bfloat16, generator=g)
    w2 = torch.randn(4096, 1024, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    _check(G.xd_gemm(x2, w2, form=242), _ref(x2, w2, "store", None))
    G.check_splitk_fault()


def test_splitk_watch_reports_a_fault_without_a_sync(hipk):
    """ops.gemm.SplitKWatch (the engine's per-step fault poll): the fault word is copied to
    pinned memory asynchronously after each step and read by a later poll once the copy has
    landed - a forced combine timeout is reported within a few polls, counters reset, and a
    clean run never reports."""
    g = torch.Generator(device="cuda").manual_seed(98)
    x = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(1024, 1024, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    ref = _ref(x, w, "store", None)
    G.check_splitk_fault()
    watch = G.SplitKWatch(torch.device("cuda"))
    for _ in range(4):  # clean steps: nothing to report
        _check(G.xd_gemm(x, w, form=242), ref)
        assert watch.poll(raise_=False) is False
        torch.cuda.synchronize()
    assert watch.poll(raise_=False) is False
    prev = G.set_splitk_spin_limit(-1)
    try:
        G.xd_gemm(x, w, form=242)
    finally:
        G.set_splitk_spin_limit(prev)
    seen = False
    for _ in range(4):  # the copy issued by one poll is read by the next
        torch.cuda.synchronize()
        if watch.poll(raise_=False):
            seen = True
            break
    assert seen
    G.check_splitk_fault()  # the watch reset the counters
    _check(G.xd_gemm(x, w, form=242), ref)
    with pytest.raises(G.SplitKFault):  # raising form
        prev = G.set_splitk_spin_limit(-1)
        try:
            G.xd_gemm(x, w, form=242)
        finally:
            G.set_splitk_spin_limit(prev)
        for _ in range(4):
            torch.cuda.synchronize()
            watch.poll()
    G.check_splitk_fault()


def test_hbm_budget_too_small_for_one_sequence_is_an_error(hipk):
    """An engine group whose HBM budget cannot hold its weights plus one max_model_len sequence
    of KV cache fails at start with the numbers, instead of starting with 2 blocks."""
    from drtc_amd.engine import LLMEngine
    from drtc_amd.models import LLAMA3_8B, TransformerLM

    m = TransformerLM(LLAMA3_8B.replace(num_layers=2), "cuda", seed=0, full_then_shard=False)
    with pytest.raises(ValueError, match="HBM budget"):
        LLMEngine(m, max_batch=8, max_model_len=4096, hbm_budget=0.01, use_graphs=False)
    eng = LLMEngine(m, max_batch=8, max_model_len=4096, hbm_budget=0.2, use_graphs=False)
    assert eng.kv.num_blocks >= eng.max_blocks


@pytest.mark.parametrize("epi", ["store", "silu", "gelu_tanh"])
@pytest.mark.parametrize("sizes,N,K,r0", [
    ((300, 0, 700, 256, 1), 512, 256, 7),   # an empty group, row tails, a one-row group
    ((1024, 1024, 513), 1024, 1024, 0),
    ((5,), 256, 128, 3),                    # one partial tile: surplus workgroups leave at once
    ((2048, 1900, 2100, 2000, 1990, 2010, 2080, 1970), 256, 512, 0),  # MoE-like, 8 experts
])
def test_w4_grouped_matches_fp32(hipk, epi, sizes, N, K, r0):
    """gemm_w4's grouped persistent form (the MoE prefill GEMM): every row group times its own
    weight, device-side row offsets, rows outside the groups untouched."""
    glu = epi != "store"
    G_ = len(sizes)
    g = torch.Generator(device="cuda").manual_seed(sum(sizes) + N)
    offs = [r0]
    for s in sizes:
        offs.append(offs[-1] + s)
    R = offs[-1] + 5
    x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(G_, 2 * N if glu else N, K, device="cuda", dtype=torch.bfloat16,
                    generator=g) * 0.05
    grp = torch.tensor(offs, dtype=torch.int32, device="cuda")
    out = torch.full((R, N), 7.0, device="cuda", dtype=torch.bfloat16)
    G.mfma_gemm_grouped(x, w, grp, epi, out=out)
    for e in range(G_):
        a, b = offs[e], offs[e + 1]
        if b > a:
            _check(out[a:b], _ref(x[a:b], w[e], epi, None))
    assert bool((out[:r0] == 7).all()) and bool((out[offs[-1]:] == 7).all())


@pytest.mark.parametrize("ksplit", [2, 4])
def test_w4_grouped_split_k_partials_sum_to_fp32(hipk, ksplit):
    """Grouped form with K cut into slices (the MoE down at few rows per expert): the bf16
    partial products of the slices sum to the fp32 product; a gated epilogue is refused."""
    g = torch.Generator(device="cuda").manual_seed(11 + ksplit)
    offs = [0, 300, 300, 812, 1000]
    R, N, K = 1000, 512, 1024
    x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(4, N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    grp = torch.tensor(offs, dtype=torch.int32, device="cuda")
    out = G.mfma_gemm_grouped(x, w, grp, "store", ksplit=ksplit)
    assert out.shape == (ksplit, R, N)
    tot = out.float().sum(0)
    for e in range(4):
        a, b = offs[e], offs[e + 1]
        if b > a:
            _check(tot[a:b], _ref(x[a:b], w[e], "store", None), tol=2e-2)
    w2 = torch.randn(4, 2 * N, K, device="cuda", dtype=torch.bfloat16, generator=g)
    with pytest.raises(RuntimeError):
        G.mfma_gemm_grouped(x, w2, grp, "silu", ksplit=2)


def test_w4_grouped_clamps_offsets_to_the_operands(hipk):
    """Device offsets past the rows the launch was sized for (or decreasing) are clamped: the
    kernel never reads or writes outside its operands."""
    g = torch.Generator(device="cuda").manual_seed(5)
    R, N, K = 600, 256, 256
    x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(3, N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    grp = torch.tensor([-5, 400, 300, 10 ** 6], dtype=torch.int32, device="cuda")
    out = torch.full((R, N), 7.0, device="cuda", dtype=torch.bfloat16)
    G.mfma_gemm_grouped(x, w, grp, "store", out=out)
    torch.cuda.synchronize()
    _check(out[:400], _ref(x[:400], w[0], "store", None))     # group 0: rows [0, 400)
    _check(out[400:], _ref(x[400:], w[2], "store", None))     # group 1 empty, group 2 [400, 600)


def test_w4_grouped_graph_replay_follows_device_offsets(hipk):
    """The group offsets are read on the device at run time: a captured launch replays with
    new offsets written into the same tensor (no host sync, no re-capture)."""
    g = torch.Generator(device="cuda").manual_seed(3)
    R, N, K = 1500, 512, 256
    x = torch.randn(R, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(3, N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    grp = torch.tensor([0, 500, 1000, 1500], dtype=torch.int32, device="cuda")
    out = torch.zeros(R, N, device="cuda", dtype=torch.bfloat16)
    G.mfma_gemm_grouped(x, w, grp, "store", out=out)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        G.mfma_gemm_grouped(x, w, grp, "store", out=out)
    grp.copy_(torch.tensor([0, 100, 1400, 1500], dtype=torch.int32))
    gr.replay()
    torch.cuda.synchronize()
    for e, (a, b) in enumerate([(0, 100), (100, 1400), (1400, 1500)]):
        _check(out[a:b], _ref(x[a:b], w[e], "store", None))
