"""End-to-end GPU numerics at the REAL model shapes (2-layer slices).

The tiny configs of test_model_gpu.py exercise control flow; these run the
production kernels at the shapes the benchmarks use - Llama-3-8B (H 4096,
GQA 32/8, vocab 128k), Gemma-2B (H 2048, MQA, head_dim 256, GELU, vocab
256k), Llama-3-70B (H 8192, GQA 64/8) and Mixtral 8x7B (8 experts, top-2) -
and compare them with the PyTorch reference implementation of every op
(``ops.reference_mode``) on the same weights:

* the packed varlen prefill (MFMA flash attention, fused RoPE, tuned
  hipBLASLt GEMMs, GEMM-epilogue residual, fused norms) -> last-token logits;
* the serving path (paged KV cache, hipGraph decode, fused sampler in greedy
  mode) -> every generated token must be a maximiser of the reference
  full-sequence forward within bf16 tolerance.
"""
import pytest
import torch

from drtc_amd import ops
from drtc_amd.engine import LLMEngine, SamplingParams
from drtc_amd.models import GEMMA_2B, LLAMA3_8B, LLAMA3_70B, MIXTRAL_8X7B, TransformerLM
from drtc_amd.models.transformer import PrefillMeta

pytestmark = pytest.mark.gpu

CFGS = [LLAMA3_8B, GEMMA_2B, LLAMA3_70B, MIXTRAL_8X7B]


def _slice(cfg):
    if cfg.num_experts:
        # all experts active: top-2 choices can flip between the two paths on
        # router logits tied within bf16 noise; the expert GEMMs, gating and
        # combine are the same kernels at k = 8
        return cfg.replace(num_layers=2, experts_per_token=cfg.num_experts)
    return cfg.replace(num_layers=2)


def _prefill_logits(m, seqs):
    dev = m.device
    cu = [0]
    for s in seqs:
        cu.append(cu[-1] + len(s))
    ids = torch.tensor(sum(seqs, []), dtype=torch.int32, device=dev)
    pos = torch.cat([torch.arange(len(s), dtype=torch.int32) for s in seqs]).to(dev)
    meta = PrefillMeta(positions=pos, slots=torch.full((cu[-1],), -1, dtype=torch.int64, device=dev),
                       cu_seqlens=torch.tensor(cu, dtype=torch.int32, device=dev), cu_host=cu,
                       tiles=None, last_idx=torch.tensor(cu[1:], dtype=torch.int64, device=dev) - 1)
    return m.forward_prefill(ids, meta, None).float()


@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: c.name)
def test_real_shape_prefill_matches_reference(hipk, cfg):
    m = TransformerLM(_slice(cfg), "cuda", seed=21, full_then_shard=False)
    g = torch.Generator().manual_seed(1)
    seqs = [torch.randint(3, cfg.vocab_size, (n,), generator=g).tolist() for n in (150, 37, 301, 1)]
    hip = _prefill_logits(m, seqs)
    with ops.reference_mode():
        ref = _prefill_logits(m, seqs)
    scale = ref.abs().max().item()
    err = (hip - ref).abs().max().item()
    assert err < 0.03 * max(1.0, scale), (err, scale)
    # the top-1 token agrees wherever the reference's top-2 gap exceeds the error
    top2 = ref.topk(2, dim=-1).values
    clear = (top2[:, 0] - top2[:, 1]) > 2 * err
    assert torch.equal(hip.argmax(-1)[clear], ref.argmax(-1)[clear])
    del m
    torch.cuda.empty_cache()


@pytest.mark.parametrize("cfg", CFGS, ids=lambda c: c.name)
def test_real_shape_serving_matches_reference(hipk, cfg):
    m = TransformerLM(_slice(cfg), "cuda", seed=22, full_then_shard=False)
    eng = LLMEngine(m, max_batch=8, max_model_len=1024, num_blocks=256, use_graphs=True)
    g = torch.Generator().manual_seed(2)
    prompts = [torch.randint(3, cfg.vocab_size, (n,), generator=g).tolist() for n in (148, 20, 260)]
    reqs = eng.generate(prompts, SamplingParams.greedy(10, ignore_eos=True))
    for p, r in zip(prompts, reqs):
        assert len(r.output_ids) == 10
        with ops.reference_mode():
            ref = m.forward_reference([p + r.output_ids[:-1]])[0].float()
        for j, tok in enumerate(r.output_ids):
            row = ref[len(p) - 1 + j]
            assert row[tok] >= row.max() - 0.03 * max(1.0, row.abs().max().item()), (j, tok)
    assert eng.alloc.num_used == 0
    del eng, m
    torch.cuda.empty_cache()
