"""Decode-batch GEMM (csrc/kernels/gemm_dec.hip: 128 x 128 tiles, K split over two wave
groups per workgroup) vs a PyTorch fp32 reference of the same op: every epilogue (store,
residual add in place, SiLU / tanh-GELU gating of a [gate; up] weight), every LDS-region
count, row tails (M not a multiple of 128), strided inputs and hipGraph replay."""
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


def _rel(out, ref):
    return (out.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)


@pytest.mark.parametrize("nr,pipe", [(4, 1), (6, 1), (8, 1), (4, 2), (6, 2), (8, 2)])
@pytest.mark.parametrize("epi", ["store", "residual", "silu", "gelu_tanh"])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (256, 512, 512), (300, 384, 1024),
                                   (1024, 1024, 2048), (77, 256, 192)])
def test_dec_gemm_matches_fp32(hipk, nr, pipe, epi, M, N, K):
    g = torch.Generator(device="cuda").manual_seed(M * 31 + N + K + nr)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.05
    nout = N // 2 if epi in ("silu", "gelu_tanh") else N
    res = torch.randn(M, nout, device="cuda", dtype=torch.bfloat16, generator=g) if epi == "residual" else None
    ref = _ref(x, w, epi, res)
    out = G.dec_gemm(x, w, epi, residual=res, nr=nr, pipe=pipe)
    if epi == "residual":
        assert out.data_ptr() == res.data_ptr()
    assert out.shape == (M, nout) and _rel(out, ref) < 1.5e-2


@pytest.mark.parametrize("group_m", [1, 4, 8])
def test_dec_gemm_real_shapes_and_group_order(hipk, group_m):
    """Llama-3-8B o / down at the 1024-row decode bucket (one tile per CU), tile order
    grouped by 1 / 4 / 8 row tiles: the same bits whatever the order."""
    g = torch.Generator(device="cuda").manual_seed(7)
    for N, K in ((4096, 4096), (4096, 14336)):
        x = torch.randn(1024, K, device="cuda", dtype=torch.bfloat16, generator=g)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16, generator=g) * 0.02
        out = G.dec_gemm(x, w, group_m=group_m)
        assert _rel(out, x.float() @ w.float().t()) < 1e-2
        assert torch.equal(out, G.dec_gemm(x, w, group_m=8))


def test_dec_gemm_strided_input_and_graph_replay(hipk):
    """x as a row-strided view; captured in a hipGraph and replayed bitwise with new
    inputs, interleaved with a library GEMM graph (the decode graph mixes both)."""
    from drtc_amd import ops

    g = torch.Generator(device="cuda").manual_seed(3)
    big = torch.randn(512, 6144, device="cuda", dtype=torch.bfloat16, generator=g)
    x = big[:, :4096]
    w = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16, generator=g) * 0.02
    out = torch.empty(512, 4096, device="cuda", dtype=torch.bfloat16)
    G.dec_gemm(x, w, out=out)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        G.dec_gemm(x, w, out=out)
    lib_out = ops.linear(x, w)
    torch.cuda.synchronize()
    gl = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gl):
        lib_y = ops.linear(x, w)
    for _ in range(3):
        big.copy_(torch.randn(512, 6144, device="cuda", dtype=torch.bfloat16, generator=g))
        gr.replay()
        gl.replay()
        torch.cuda.synchronize()
        ref = x.float() @ w.float().t()
        assert _rel(out, ref) < 1e-2 and _rel(lib_y, ref) < 1e-2
    del lib_out


def test_dec_gemm_rejects_bad_shapes(hipk):
    x = torch.randn(64, 100, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(256, 100, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(AssertionError):
        G.dec_gemm(x, w)  # K % 64 != 0
    x = torch.randn(64, 128, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(200, 128, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(AssertionError):
        G.dec_gemm(x, w)  # N % 128 != 0
    assert not G.dec_supported(64, 200, 128) and G.dec_supported(64, 256, 128)
