"""Fused mixture-of-experts layer (router top-k -> grouped expert GEMMs -> combine).

HIP kernels: csrc/kernels/moe.hip.  One call enqueues four kernels with
static launch shapes (the per-expert tile table lives on the device), so the
layer is hipGraph-capturable and the Mixtral decode step replays with no
host synchronisation and exact sparse FLOPs (the earlier graph path ran every
expert on every token).  SURVEY.md §2 K8.

Routing semantics (Mixtral): top-k of the router logits, softmax over the
selected k logits; ties pick the lower expert id.  With expert parallelism a
rank holds experts [e_off, e_off + e_local) and returns only their
contribution (the caller all-reduces over the EP group).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from ._ext import check, hipk, on_gpu, stream_ptr
from .activation import ACTS, act_glu_ref

# Largest token chunk per kernel call: bounds the workspace (P = chunk * k rows of [I] and [H]
# intermediates: ~3 GB for Mixtral).  One Mixtral prefill step (ModelConfig.prefill_chunk,
# 32k tokens) in one call: 8k rows per expert on variant 4 (profiles/r6j: the 16k-token layer
# 8.94 ms in one call vs 9.56 ms in two of 8192; profiles/r6t: the batch-1024 wave +1.6 % with
# 32k-token prefill steps and MoE calls).
MOE_CHUNK = int(os.environ.get("DRTC_MOE_CHUNK", "32768"))

# Grouped-GEMM structure (csrc/kernels/moe.hip): 0 = 128-row two-barrier,
# 1 = 128-row 3-stage pipeline, 2 = 256-row 3-stage pipeline, 3 = gemm_xd's grouped mode
# (csrc/kernels/gemm_xd.hip: XCD-partitioned tiles, GLU epilogue, split-K, non-temporal
# weights where an expert's rows fit one tile), 4 = token rows gathered into expert order, then
# gemm_w4's grouped persistent 256 x 256 form (csrc/kernels/gemm_w4.hip; prefill-sized rows per
# expert), -1 = by rows per expert (4 from 256 rows per expert, 3 from 96).
MOE_GEMM_VARIANT = int(os.environ.get("DRTC_MOE_VARIANT", "-1"))
# gemm_xd forms of variant 3 (mt * 100 + nf * 10 + splitk, + 1000 non-temporal; 0 = by rows
# per expert, csrc/kernels/moe.hip launch_moe)
MOE_GU_FORM = int(os.environ.get("DRTC_MOE_GU_FORM", "0"))
MOE_DN_FORM = int(os.environ.get("DRTC_MOE_DN_FORM", "0"))


def route_ref(router_logits: torch.Tensor, top_k: int):
    """(expert ids [T, k], weights [T, k] fp32) with the kernel's tie rule."""
    lg = router_logits.float()
    v, i = torch.sort(lg, dim=-1, descending=True, stable=True)
    return i[:, :top_k], torch.softmax(v[:, :top_k], dim=-1)


def fused_moe_ref(x: torch.Tensor, router_logits: torch.Tensor, w_gu: torch.Tensor,
                  w_dn: torch.Tensor, top_k: int, act: str = "silu", e_off: int = 0) -> torch.Tensor:
    """fp32-accumulated PyTorch reference of :func:`fused_moe`."""
    topi, wts = route_ref(router_logits, top_k)
    out = torch.zeros(x.shape[0], x.shape[1], dtype=torch.float32, device=x.device)
    for le in range(w_gu.shape[0]):
        tok, slot = torch.nonzero(topi == e_off + le, as_tuple=True)
        if tok.numel() == 0:
            continue
        xe = x.index_select(0, tok).float()
        h = act_glu_ref(xe @ w_gu[le].float().t(), act).to(x.dtype).float()
        ye = (h @ w_dn[le].float().t()).to(x.dtype).float()
        out.index_add_(0, tok, ye * wts[tok, slot].unsqueeze(1))
    return out.to(x.dtype)


def workspace_bytes(tokens: int, hidden: int, inter: int, e_local: int, top_k: int) -> int:
    return int(hipk().moe_workspace_bytes(tokens, hidden, inter, e_local, top_k))


def make_workspace(tokens: int, hidden: int, inter: int, e_local: int, top_k: int,
                   device) -> torch.Tensor:
    """Persistent scratch for up to ``tokens`` tokens per call (allocate once,
    before any graph capture; also creates the device's split-K GEMM workspace that the
    gemm_xd forms of variant 3 use)."""
    from .gemm import gemm_workspace

    n = workspace_bytes(min(tokens, MOE_CHUNK), hidden, inter, e_local, top_k)
    if torch.device(device).type == "cuda":
        gemm_workspace(torch.device(device))
    return torch.empty(n, dtype=torch.uint8, device=device)


# fused_moe reads the router GEMM's [E, T] output in place (DRTC_ROUTER_VIEW=0: the
# transposed copy of round 5's first router form, for A/B)
ROUTER_VIEW = os.environ.get("DRTC_ROUTER_VIEW", "1") != "0"


def router_logits(x: torch.Tensor, w_router: torch.Tensor, contiguous: bool = True) -> torch.Tensor:
    """Router logits x [T, H] . w_router [E, H]^T -> [T, E], on the skinny HIP GEMM
    transposed: the E router rows are the kernel's few activation rows and the T tokens its
    streamed weight rows, so x is read once and no library GEMM runs in the MoE layer (ref
    llm_server/llm_server.py:403: the suggestions model).  ``contiguous=False`` returns the
    kernel's [E, T] output as a transposed [T, E] view (strides (1, T)), which ``fused_moe``
    reads in place (no transpose copy per layer).  A T that is not a multiple of the kernel's
    16-row block is zero-padded up to one, so every batch size routes through the same kernel
    and the same rounding (top-k choices on near-tied logits do not depend on T); E > 8 goes
    to F.linear."""
    from . import gemm as G

    T, H = x.shape
    E = w_router.shape[0]
    Tp = -(-T // 16) * 16
    if (on_gpu(x) and x.is_contiguous() and w_router.is_contiguous() and E <= 8 and T > 0
            and G.skinny_supports(3, E, Tp, H, w_router.stride(0))):
        if Tp != T:
            xp = x.new_zeros((Tp, H))
            xp[:T].copy_(x)
            x = xp
        y = G.skinny_linear(w_router, x, variant=3).t()[:T]
        return y.contiguous() if contiguous or not ROUTER_VIEW else y
    return F.linear(x, w_router)


def fused_moe(x: torch.Tensor, router_logits: torch.Tensor, w_gu: torch.Tensor,
              w_dn: torch.Tensor, top_k: int, act: str = "silu", num_experts: int | None = None,
              e_off: int = 0, workspace: torch.Tensor | None = None,
              out: torch.Tensor | None = None, variant: int | None = None,
              gu_form: int | None = None, dn_form: int | None = None) -> torch.Tensor:
    """y[t] = sum_j w[t,j] * down_e(act(gate_e x_t) * up_e x_t) over the top-k experts.

    x [T, H] bf16; router_logits [T, E] bf16, row-major or the transposed view of an [E, T]
    tensor (``router_logits(..., contiguous=False)``); w_gu [E_local, 2I, H] ([gate | up]
    rows); w_dn [E_local, H, I].
    """
    if not on_gpu(x):
        r = fused_moe_ref(x, router_logits, w_gu, w_dn, top_k, act, e_off)
        if out is not None:
            out.copy_(r)
            return out
        return r
    T, H = x.shape
    # every token count takes the fused kernels (prefill included: no host sync per layer;
    # the round-4 per-expert hipBLASLt path for T >= 4096 measured slower at T = 8192,
    # 6.05 / 5.86 ms fused vs 6.25 / 5.95 ms, profiles/r4ah, r4ak)
    E = num_experts if num_experts is not None else router_logits.shape[1]
    e_local, two_i, h2 = w_gu.shape
    inter = two_i // 2
    assert x.dtype == torch.bfloat16 and x.is_contiguous()
    assert router_logits.dtype == torch.bfloat16 and router_logits.shape == (T, E) and h2 == H
    lts, les = router_logits.stride()
    assert (lts, les) == (E, 1) or (lts == 1 and les >= T), router_logits.stride()
    assert w_gu.is_contiguous() and w_dn.is_contiguous() and w_dn.shape == (e_local, H, inter)
    assert E <= 256 and 1 <= top_k <= min(8, E) and H % 128 == 0 and inter % 64 == 0
    if out is None:
        out = torch.empty_like(x)
    assert out.is_contiguous() and out.shape == x.shape
    chunk = min(T, MOE_CHUNK) if T else 1
    need = workspace_bytes(chunk, H, inter, e_local, top_k)
    if workspace is None or workspace.numel() < need:
        assert not torch.cuda.is_current_stream_capturing(), \
            "fused_moe under graph capture needs a preallocated workspace"
        workspace = torch.empty(need, dtype=torch.uint8, device=x.device)
    lib, st = hipk(), stream_ptr(x)
    # the split-K slabs / counters of the gemm_xd forms: the device's shared GEMM workspace
    # (same stream), only when it exists already (never created inside a graph capture)
    from . import gemm as _gemm

    key = x.device.index if x.device.index is not None else torch.cuda.current_device()
    gws = _gemm._ws.get(key)
    slab, cnt = gws if gws is not None else (None, None)
    for t0 in range(0, T, MOE_CHUNK):
        n = min(MOE_CHUNK, T - t0)
        check(lib.moe(out[t0].data_ptr(), x[t0].data_ptr(), router_logits[t0].data_ptr(),
                      w_gu.data_ptr(), w_dn.data_ptr(), n, H, inter, E, top_k, e_off, e_local,
                      ACTS[act], workspace.data_ptr(), workspace.numel(),
                      MOE_GEMM_VARIANT if variant is None else variant,
                      MOE_GU_FORM if gu_form is None else gu_form,
                      MOE_DN_FORM if dn_form is None else dn_form,
                      slab.data_ptr() if slab is not None else 0,
                      slab.numel() * 4 if slab is not None else 0,
                      cnt.data_ptr() if cnt is not None else 0,
                      cnt.numel() if cnt is not None else 0, lts, les, st), "moe")
    return out

