"""Token sampling: greedy / temperature + top-k + top-p.

HIP kernel: csrc/kernels/sampling.hip (one workgroup per row; graph-replayable
because the RNG step counter lives in device memory).
"""
from __future__ import annotations

import torch

from ._ext import check, hipk, on_gpu, ptr, stream_ptr

MAX_CANDIDATES = 1024


def sample_ref(logits: torch.Tensor, temperature: torch.Tensor | None = None,
               top_k: torch.Tensor | None = None, top_p: torch.Tensor | None = None,
               generator: torch.Generator | None = None) -> torch.Tensor:
    """Reference semantics of the HIP sampler (draws differ: torch RNG).

    * temperature <= 0: argmax.
    * 0 < top_k < V: the tokens whose logit is >= the k-th largest (k capped
      at MAX_CANDIDATES; ties with the k-th value kept), softmax(l / T) over
      them, cut at the first sorted position whose inclusive mass reaches
      top_p, draw.
    * top_k == 0 (or >= V): exact top-p over the whole vocabulary: token i is
      kept iff the probability mass of tokens STRICTLY more likely than i is
      < top_p (so tied tokens are kept or dropped together)."""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    lf = logits.float()
    for b in range(B):
        t = float(temperature[b]) if temperature is not None else 0.0
        if t <= 0:
            out[b] = int(torch.argmax(lf[b]))
            continue
        pp = float(top_p[b]) if top_p is not None and 0 < float(top_p[b]) < 1 else 1.0
        k = int(top_k[b]) if top_k is not None else 0
        if 0 < k < V:
            k = min(k, MAX_CANDIDATES)
            kth = torch.topk(lf[b], k).values[-1]
            idx = torch.nonzero(lf[b] >= kth).flatten()
            vals = lf[b, idx]
            order = torch.argsort(-vals, stable=True)
            vals, idx = vals[order], idx[order]
            p = torch.softmax(vals / t, dim=-1)
            cum = torch.cumsum(p, 0)
            cut = int(torch.searchsorted(cum, torch.tensor(pp * float(cum[-1]))))
            cut = min(cut, len(idx) - 1)
            p = p[: cut + 1]
            j = int(torch.multinomial(p / p.sum(), 1, generator=generator))
            out[b] = int(idx[j])
            continue
        vals, idx = torch.sort(lf[b], descending=True, stable=True)
        p = torch.softmax(vals / t, dim=-1)
        if pp < 1.0:
            # mass strictly above each token: the exclusive cumsum at the first
            # position holding its value
            excl = torch.cumsum(p, 0) - p
            first = torch.searchsorted(-vals, -vals, right=False)
            keep = excl[first] < pp
            p = p * keep
        j = int(torch.multinomial(p / p.sum(), 1, generator=generator))
        out[b] = int(idx[j])
    return out


def sample(logits: torch.Tensor, temperature: torch.Tensor | None = None,
           top_k: torch.Tensor | None = None, top_p: torch.Tensor | None = None,
           seed: int = 0, step: torch.Tensor | None = None,
           out: torch.Tensor | None = None) -> torch.Tensor:
    """logits [B, V] bf16 -> int32 token ids [B].

    temperature/top_k/top_p are per-row device tensors (float32 / int32 /
    float32); ``step`` is an int64 device scalar the caller advances."""
    if not on_gpu(logits):
        # counter-based like the HIP sampler: the draws are a function of (seed, step), so a
        # step re-run with the same counter (EP capacity redo) draws the same tokens
        gen = None
        if step is not None:
            gen = torch.Generator().manual_seed(
                (seed * 0x9E3779B1 + int(step.reshape(-1)[0])) & 0x7FFFFFFFFFFFFFFF)
        r = sample_ref(logits, temperature, top_k, top_p, generator=gen)
        if out is not None:
            out.copy_(r)
            return out
        return r
    assert logits.dim() == 2 and logits.dtype == torch.bfloat16 and logits.stride(1) == 1
    B, V = logits.shape
    for t, dt in ((temperature, torch.float32), (top_k, torch.int32), (top_p, torch.float32)):
        assert t is None or (t.dtype == dt and t.numel() >= B and t.is_cuda)
    assert step is None or (step.dtype == torch.int64 and step.is_cuda)
    if out is None:
        out = torch.empty(B, dtype=torch.int32, device=logits.device)
    assert out.dtype == torch.int32 and out.is_contiguous()
    check(hipk().sample(out.data_ptr(), logits.data_ptr(), B, V, logits.stride(0),
                        ptr(temperature), ptr(top_k), ptr(top_p), int(seed) & ((1 << 64) - 1),
                        ptr(step), stream_ptr(logits)), "sample")
    return out
