"""Projection GEMMs with measured per-shape hipBLASLt solutions.

``linear(x, w)`` computes ``x @ w.T`` (bf16, fp32 accumulate).  For the
shapes listed in the tuning table (``ops/tuned/gemm_<arch>.json``: the
decode GEMMs of each model at every hipGraph batch bucket) it calls
hipBLASLt directly through ``csrc/kernels/gemm_lt.cpp`` with the solution
that measured fastest on MI355X.  Prefill-sized GEMMs (M above the decode
buckets) take the solution tuned at the nearest measured M (entries flagged
``prefill``, ``scripts/tune_prefill.py``) where it beat torch's own pick,
for the plain GEMM (beta = 0) and for the in-place residual form (beta = 1)
separately; every other shape (CPU, untuned) goes through
``torch.nn.functional.linear`` / ``addmm_``.

Why a table: a decode GEMM has a small fixed M (the batch bucket) and
model-fixed N/K, where hipBLASLt's heuristic pick can be far from the best
listed solution - e.g. Llama-3-70B ``down`` at M=256: 312 us heuristic vs
178 us tuned (profiles/r1g_tuned_gemm_prefill_attn.md).  Tables are produced by
``scripts/tune_gemms.py`` on the GPU and keyed by the hipBLASLt version
(solution indices are only valid for the library that listed them).

Small decode batches (M <= 8 rows) are weight-streaming GEMVs, where the
library reaches 3-4.5 TB/s on the 8B shapes; they run on the hand-written
skinny kernels of ``csrc/kernels/gemv.hip`` (VALU dot2 form and MFMA form,
several row/K-split decompositions) at up to 6.7 TB/s.  The table records,
per measured shape, whether a skinny variant beat the library
(``scripts/tune_skinny.py``); unmeasured shapes use ``skinny_variant``.
"""
from __future__ import annotations

import json
import math
import os
import threading

import torch
import torch.nn.functional as F

from ._ext import check, hipk, on_gpu, ptr, stream_ptr

TUNED_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")
_lock = threading.Lock()
# (M, N, K, ldx) -> (hipBLASLt solution index or -1, skinny-kernel variant or 0,
#                   medium-M kernel K splits or 0)
_table: dict[tuple[int, int, int, int], tuple[int, int, int]] | None = None
_ready: set[tuple[int, int, int, int]] = set()               # entries with a native plan
# (N, K, ldx) -> sorted [(tuned M, algo, beats F.linear, beats addmm_)]: prefill entries
_prefill: dict[tuple[int, int, int], list[tuple[int, int, bool, bool]]] = {}
# (M, N, K, ldx, beta) -> algo chosen for a prefill-sized call (-1: torch's path)
_prefill_pick: dict[tuple[int, int, int, int, int], int] = {}
DECODE_MAX_M = 1024  # decode buckets end here; larger M are prefill (or mixed) passes
_enabled = os.environ.get("DRTC_TUNED_GEMM", "1") != "0"
# prefill-sized entries (tuned at M = 2k..16k, scripts/tune_prefill.py)
_prefill_enabled = os.environ.get("DRTC_PREFILL_TUNED", "1") != "0"
# medium-M decode kernel (gemm_midm.hip) where the tuning table measured a win
_midm_enabled = os.environ.get("DRTC_MIDM_GEMM", "1") != "0"
# decode batches up to this many rows may take the hand-written skinny kernel
# (csrc/kernels/gemv.hip) instead of the library: the tuning table's choice
# where the shape was measured, skinny_variant()'s default otherwise; 0
# disables it
SKINNY_MAX_M = int(os.environ.get("DRTC_SKINNY_MAX_M", "16"))
SKINNY_DEFAULT_MAX_M = 8  # untuned shapes: measured gains up to M = 8 only


def table_path(arch: str = "gfx950") -> str:
    return os.path.join(TUNED_DIR, f"gemm_{arch}.json")


def load_table(path: str | None = None) -> dict:
    """Read the tuning file: {str(hipblaslt_version): {"M,N,K,ldx": {...}}}."""
    path = path or table_path()
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


def _activate() -> dict:
    """Parse the entries of the running hipBLASLt version (no GPU work; each
    entry is registered with the native plan cache on its first use)."""
    global _table
    if _table is not None:
        return _table
    with _lock:
        if _table is not None:
            return _table
        tab: dict[tuple[int, int, int, int], tuple[int, int, int]] = {}
        pre: dict[tuple[int, int, int], list[tuple[int, int, bool, bool]]] = {}
        if _enabled and torch.cuda.is_available():
            ver = str(hipk().lt_version())
            for ks, e in load_table().get(ver, {}).items():
                M, N, K, ldx = (int(v) for v in ks.split(","))
                if e.get("prefill"):
                    if _prefill_enabled:
                        pre.setdefault((N, K, ldx), []).append(
                            (M, int(e["algo"]), bool(e.get("beta0")), bool(e.get("beta1"))))
                    continue
                tab[(M, N, K, ldx)] = (int(e.get("algo", -1)), int(e.get("skinny", 0)),
                                       int(e.get("midm", 0)) if _midm_enabled else 0)
        for v in pre.values():
            v.sort()
        _ready.clear()
        _prefill.clear()
        _prefill.update(pre)
        _prefill_pick.clear()
        _table = tab
    return _table


def _plan(key: tuple[int, int, int, int]) -> bool:
    """Register a table entry's solution with the native plan cache (first
    use happens in the eager warm-up run that precedes each graph capture).
    A stale entry (solution no longer supports the problem) is dropped."""
    if key in _ready:
        return True
    M, N, K, ldx = key
    with _lock:
        if hipk().lt_set_algo(M, N, K, ldx, N, _table[key][0]) != 0:
            _table.pop(key, None)
            return False
        _ready.add(key)
    return True


def _prefill_algo(M: int, N: int, K: int, ldx: int, beta: int) -> int:
    """Solution for a prefill-sized GEMM: the entry tuned at the M nearest
    to this one (log scale) for the same (N, K, ldx), if that entry beat
    torch's pick for this beta; -1 = use torch's path.  The native plan is
    per exact M (registered on first use, outside graph capture: prefill
    passes run eagerly)."""
    key = (M, N, K, ldx, beta)
    algo = _prefill_pick.get(key)
    if algo is not None:
        return algo
    algo = -1
    cands = _prefill.get((N, K, ldx))
    if cands and M > DECODE_MAX_M:
        Mt, a, b0, b1 = min(cands, key=lambda c: abs(math.log(c[0] / M)))
        if (b1 if beta else b0) and abs(math.log(Mt / M)) <= math.log(2.0):
            with _lock:
                if hipk().lt_set_algo(M, N, K, ldx, N, a) == 0:
                    algo = a
    _prefill_pick[key] = algo
    return algo


def reset() -> None:
    """Forget the activated table (tests / after re-tuning)."""
    global _table
    with _lock:
        _table = None


def set_enabled(on: bool) -> None:
    global _enabled
    _enabled = bool(on)
    reset()


# rows of W per workgroup of each MFMA variant (gemv.hip launch_skinny_gemm)
SKINNY_ROWS = {2: 16, 3: 16, 4: 32, 5: 32, 6: 16, 7: 64, 8: 128, 9: 64}


def skinny_supports(v: int, M: int, N: int, K: int, ldx: int) -> bool:
    """Whether skinny variant ``v`` covers the shape (mirrors the launcher)."""
    if not 1 <= M <= 16 or ldx % 8 or N % 4:
        return False
    if v == 1:
        return M <= 8 and K % 512 == 0
    return v in SKINNY_ROWS and K % 128 == 0 and N % SKINNY_ROWS[v] == 0


def skinny_variant(M: int, N: int, K: int, ldx: int) -> int:
    """Default skinny-kernel form for an untuned shape: 1 = VALU dot2 for
    M <= 2, 3 = MFMA (1 tile, 8 K-split waves) up to M = 8; 0 = leave it to
    the library."""
    if M > min(SKINNY_MAX_M, SKINNY_DEFAULT_MAX_M):
        return 0
    for v in ((1, 3) if M <= 2 else (3,)):
        if skinny_supports(v, M, N, K, ldx):
            return v
    return 0


def skinny_ok(M: int, N: int, K: int, ldx: int) -> bool:
    return skinny_variant(M, N, K, ldx) != 0


def skinny_linear(x: torch.Tensor, w: torch.Tensor, variant: int = 0) -> torch.Tensor:
    """y = x @ w.T on the skinny decode kernel (M <= 16 rows of x)."""
    M, K = x.shape
    N = w.shape[0]
    variant = variant or skinny_variant(M, N, K, x.stride(0))
    y = torch.empty((M, N), dtype=x.dtype, device=x.device)
    check(hipk().skinny_gemm(y.data_ptr(), x.data_ptr(), w.data_ptr(), M, N, K, x.stride(0), N,
                             variant, stream_ptr(x)), "skinny_gemm")
    return y


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x @ w.T for x [M, K] (row stride ldx), w [N, K] contiguous."""
    if (on_gpu(x) and _enabled and x.dim() == 2 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.stride(1) == 1 and w.is_contiguous()):
        M, K = x.shape
        N = w.shape[0]
        key = (M, N, K, x.stride(0))
        ent = _activate().get(key)
        if (sk := w4_dec_splitk(M, N, K)) and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 \
                and w.data_ptr() % 16 == 0:
            return mfma_gemm(x, w, "store", variant=W4_VARIANT, splitk=sk, group_m=4)
        if ent is None and (sk := w4_rs_splitk(M, N, K)) and x.stride(0) % 8 == 0 \
                and x.data_ptr() % 16 == 0:
            return mfma_gemm(x, w, "store", variant=11, splitk=sk, group_m=4)
        if ent is None and M > DECODE_MAX_M:
            if w4_ok(x, w):
                return mfma_gemm(x, w, "store", variant=_w4v(K), group_m=w4_group_m(M, N, K))
            if _prefill_algo(M, N, K, x.stride(0), 0) >= 0:
                y = torch.empty((M, N), dtype=x.dtype, device=x.device)
                check(hipk().lt_gemm(y.data_ptr(), x.data_ptr(), w.data_ptr(), M, N, K,
                                     x.stride(0), N, 0.0, stream_ptr(x)), "lt_gemm")
                return y
        elif ent is None:
            v = skinny_variant(M, N, K, x.stride(0))
            if v:
                return skinny_linear(x, w, v)
        elif ent[1] and M <= SKINNY_MAX_M:
            return skinny_linear(x, w, ent[1])
        elif ent[2] and M <= MIDM_MAX_M:
            return midm_gemm(x, w, "store", splits=ent[2])
        elif (sk := w4_rs_splitk(M, N, K)) and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0:
            return mfma_gemm(x, w, "store", variant=11, splitk=sk, group_m=4)
        elif ent[0] >= 0 and _plan(key):
            y = torch.empty((M, N), dtype=x.dtype, device=x.device)
            check(hipk().lt_gemm(y.data_ptr(), x.data_ptr(), w.data_ptr(), M, N, K, x.stride(0),
                                 N, 0.0, stream_ptr(x)), "lt_gemm")
            return y
    return F.linear(x, w)


_fuse_residual = os.environ.get("DRTC_RESIDUAL_GEMM", "1") != "0"
# measured (scripts/residual_gemm_bench.py, MI355X, H=4096): at 16k rows the
# beta=1 GEMM costs the same as beta=0 while the following RMSNorm drops from
# ~90 us (read x + residual, write both) to ~39 us (read h, write out); at
# 1024 rows both norms are launch-latency bound (7-8 us) - no gain
RESIDUAL_FUSE_MIN_M = 4096


def residual_fusable(x: torch.Tensor, residual: torch.Tensor) -> bool:
    """Whether ``linear_residual`` pays for x [M, K] -> residual [M, N]: on
    the GPU at prefill-sized M (bf16).  Elsewhere the caller runs ``linear``
    and leaves the add to the next fused add-RMSNorm."""
    return (_fuse_residual and on_gpu(x) and x.dim() == 2 and x.shape[0] >= RESIDUAL_FUSE_MIN_M
            and x.dtype == residual.dtype == torch.bfloat16
            and residual.dim() == 2 and residual.shape[0] == x.shape[0]
            and residual.stride(1) == 1)


def linear_residual(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
    """residual += x @ w.T with the add in the GEMM epilogue (beta = 1, in
    place into the residual stream), for the o / down projections of a
    prefill pass; returns the updated residual.  One rounding to bf16 (of
    the fp32 accumulator plus the residual) instead of two (GEMM output,
    then the add in the norm kernel)."""
    assert residual.shape == (x.shape[0], w.shape[0]) and w.dtype == x.dtype
    M, K = x.shape
    N = w.shape[0]
    if w4_ok(x, w, residual):
        return mfma_gemm(x, w, "residual", residual=residual, out=residual, variant=_w4v(K),
                         group_m=w4_group_m(M, N, K))
    if (_enabled and x.stride(1) == 1 and w.is_contiguous() and residual.stride(0) == N
            and x.dtype == torch.bfloat16):
        _activate()
        if _prefill_algo(M, N, K, x.stride(0), 1) >= 0:
            check(hipk().lt_gemm(residual.data_ptr(), x.data_ptr(), w.data_ptr(), M, N, K,
                                 x.stride(0), N, 1.0, stream_ptr(x)), "lt_gemm")
            return residual
    return residual.addmm_(x, w.t())


_fuse_norm = os.environ.get("DRTC_FUSED_NORM_GEMM", "1") != "0"
# measured: the fused norm pays at M = 1 only (gemv.hip skinny_norm_gemm_kernel)
NORM_FUSE_MAX_M = 1


def _choice(M: int, N: int, K: int, ldx: int) -> int:
    """Skinny variant ops.linear would run for this shape (0 = library)."""
    ent = _activate().get((M, N, K, ldx))
    if ent is None:
        return skinny_variant(M, N, K, ldx)
    return ent[1] if M <= SKINNY_MAX_M else 0


def norm_linear(p, w: torch.Tensor, w_folded: torch.Tensor | None = None) -> torch.Tensor:
    """y = rmsnorm(p.x [+ p.residual]) @ w.T for an ``ops.PendingNorm`` p.

    When the projection would run on the skinny dot2 kernel anyway (small
    decode batches, measured per shape) the norm is fused into it
    (gemv.hip ``skinny_norm_gemm_kernel``): one launch instead of two, and
    the new residual stream is written by the GEMM.  When the producer left the
    norm's row statistic (``p.rinv``) and the caller passes the projection with
    the norm weight folded in (``w_folded``), the 4-wave GEMM reads the residual
    stream itself and scales its rows (``rs_linear``: no normalised copy).
    Otherwise the norm is materialised and ``linear`` runs."""
    x, res = p.x, p.residual
    if p.rinv is not None and p._out is None and w_folded is not None:
        y = rs_linear(x, w_folded, p.rinv)
        if y is not None:
            return y
    if (_fuse_norm and p._out is None and p.pc is None and isinstance(x, torch.Tensor)
            and on_gpu(x) and _enabled and x.dim() == 2
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.stride(1) == 1
            and w.is_contiguous() and p.w.is_contiguous()
            and (res is None or (res.stride(1) == 1 and res.shape == x.shape))):
        M, K = x.shape
        N = w.shape[0]
        if (M <= NORM_FUSE_MAX_M and K % 2048 == 0 and K <= 8192 and N % 4 == 0 and x.stride(0) % 8 == 0
                and (res is None or res.stride(0) % 8 == 0) and _choice(M, N, K, K) == 1):
            y = torch.empty((M, N), dtype=x.dtype, device=x.device)
            h = torch.empty((M, K), dtype=x.dtype, device=x.device) if res is not None else None
            check(hipk().skinny_norm_gemm(
                y.data_ptr(), ptr(h), x.data_ptr(), ptr(res), p.w.data_ptr(), w.data_ptr(), M, N,
                K, x.stride(0), res.stride(0) if res is not None else 0, K, N, float(p.eps),
                bool(p.gemma), stream_ptr(x)), "skinny_norm_gemm")
            p.applied(h if h is not None else x)
            return y
    return linear(p.materialize(), w)


_fuse_glu = os.environ.get("DRTC_FUSED_GLU_GEMM", "1") != "0"
GLU_FUSE_MAX_M = 1


def glu_linear(gu: torch.Tensor, w: torch.Tensor, act: str = "silu") -> torch.Tensor:
    """y = (act(gu[:, :I]) * gu[:, I:]) @ w.T (the down projection of a gated
    MLP).  When the projection would run on the skinny dot2 kernel the
    activation is computed inside it while loading its input (gemv.hip,
    no act_glu launch); otherwise ops.act_glu + linear."""
    from .activation import act_glu

    if (_fuse_glu and on_gpu(gu) and _enabled and gu.dim() == 2 and gu.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and gu.stride(1) == 1 and w.is_contiguous()
            and act in ("silu", "gelu_tanh")):
        M, I2 = gu.shape
        I, N = I2 // 2, w.shape[0]
        if (M <= GLU_FUSE_MAX_M and I2 % 2 == 0 and w.shape[1] == I and I % 512 == 0
                and N % 4 == 0 and gu.stride(0) % 8 == 0 and _choice(M, N, I, I) == 1):
            y = torch.empty((M, N), dtype=gu.dtype, device=gu.device)
            check(hipk().skinny_glu_gemm(y.data_ptr(), gu.data_ptr(), w.data_ptr(), M, N, I,
                                         gu.stride(0), N, 0 if act == "silu" else 1,
                                         stream_ptr(gu)), "skinny_glu_gemm")
            return y
    return linear(act_glu(gu, act), w)


# ------------------------------------------------------------ hand-written MFMA GEMM
EPI = {"store": 0, "residual": 1, "silu": 2, "gelu_tanh": 3, "partial": 4, "residual_sq": 5,
       "store_rs": 6, "silu_rs": 7, "gelu_tanh_rs": 8}
_ws_lock = threading.Lock()
_ws: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
WS_SLAB_BYTES = 128 << 20   # fp32 split-K slabs (per device)
WS_COUNTERS = 1 << 16


def gemm_workspace(dev: torch.device) -> tuple[torch.Tensor, torch.Tensor]:
    """Split-K workspace of a device: fp32 slabs + per-tile arrival counters
    (zeroed once; the last arriver of each tile re-arms its counter).  One
    per device, shared by every GEMM that runs on the engine's stream; a GEMM
    issued concurrently on another stream must pass its own (``ws=``).
    Create it before any graph capture (the engine's eager warm-up does)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    ws = _ws.get(key)
    if ws is None:
        with _ws_lock:
            ws = _ws.get(key)
            if ws is None:
                ws = (torch.empty(WS_SLAB_BYTES // 4, dtype=torch.float32, device=dev),
                      torch.zeros(WS_COUNTERS, dtype=torch.int32, device=dev))
                _ws[key] = ws
    return ws


def new_gemm_workspace(dev: torch.device) -> tuple[torch.Tensor, torch.Tensor]:
    """A private split-K workspace (for GEMMs on a second stream)."""
    return (torch.empty(WS_SLAB_BYTES // 4, dtype=torch.float32, device=dev),
            torch.zeros(WS_COUNTERS, dtype=torch.int32, device=dev))


def mfma_gemm(x: torch.Tensor, w: torch.Tensor, epi: str = "store",
              residual: torch.Tensor | None = None, out: torch.Tensor | None = None,
              variant: int = 2, splitk: int = 1, group_m: int = 8,
              ws: tuple[torch.Tensor, torch.Tensor] | None = None,
              side: torch.Tensor | None = None) -> torch.Tensor:
    """Hand-written CDNA4 GEMM (csrc/kernels/gemm.hip): y = epi(x @ w.T).

    epi "store": y = x @ w.T; "residual": y = x @ w.T + residual (``out`` may
    be ``residual`` itself: in-place add into the residual stream);
    "silu" / "gelu_tanh": w is the fused [gate; up] weight [2I, K] and
    y[:, n] = act(x . gate_n) * (x . up_n) has I columns (no act_glu pass).
    Shapes: K % 64 == 0, N % 256 == 0 (I % 128 == 0 for the gated forms),
    (K / 64) % splitk == 0; rows of x are unrestricted."""
    M, K = x.shape
    glu = epi in ("silu", "gelu_tanh", "silu_rs", "gelu_tanh_rs")
    N = w.shape[0] // 2 if glu else w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    st = stream_ptr(x)
    slab, cnt = ((ws or gemm_workspace(x.device)) if splitk > 1 else (None, None))
    if side is not None:  # folded-norm epilogues (gemm_w4): sq[M][N/128] or rinv[M], fp32
        assert gemm_w4_variant(variant) and splitk == 1 and side.dtype == torch.float32
        slab = side
    check(hipk().gemm(out.data_ptr(), x.data_ptr(), w.data_ptr(), ptr(residual), M, N, K,
                      x.stride(0), w.stride(0), out.stride(0),
                      residual.stride(0) if residual is not None else 0, EPI[epi],
                      N if glu else 0, variant, splitk, group_m, ptr(slab),
                      slab.numel() * 4 if slab is not None else 0, ptr(cnt),
                      cnt.numel() if cnt is not None else 0, st), "gemm")
    return out


def tune(M: int, N: int, K: int, device, iters: int = 20, max_candidates: int = 12) -> dict:
    """Measure every hipBLASLt solution for y[M,N] = x[M,K] @ W[N,K]^T on
    random operands; returns {"algo", "us", "heuristic_us", "candidates"}."""
    g = torch.Generator(device=device).manual_seed(M * 7 + N * 13 + K)
    x = torch.randn(M, K, device=device, dtype=torch.bfloat16, generator=g)
    w = torch.randn(N, K, device=device, dtype=torch.bfloat16, generator=g) * 0.02
    y = torch.empty(M, N, device=device, dtype=torch.bfloat16)
    torch.cuda.synchronize(device)
    res = hipk().lt_tune(y.data_ptr(), x.data_ptr(), w.data_ptr(), M, N, K, K, N, iters,
                         max_candidates, torch.cuda.current_stream(device).cuda_stream)
    if not res:
        raise RuntimeError(f"lt_tune found no solution for M={M} N={N} K={K}")
    heur = next((us for i, us in res if i == -1), float("inf"))
    best_i, best_us = min(((i, us) for i, us in res if i >= 0), key=lambda t: t[1],
                          default=(-1, heur))
    return {"algo": best_i, "us": round(best_us, 2), "heuristic_us": round(heur, 2),
            "candidates": len(res) - 1}


def save_entries(entries: dict[str, dict], path: str | None = None) -> str:
    """Merge ``entries`` ("M,N,K,ldx" -> tune() result) into the table of the
    running hipBLASLt version."""
    path = path or table_path()
    data = load_table(path)
    ver = str(hipk().lt_version())
    cur = data.setdefault(ver, {})
    for k, e in entries.items():
        cur[k] = {**cur.get(k, {}), **e}
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    reset()
    return path


def gemm_w4_variant(variant: int) -> bool:
    return 7 <= variant <= 15 or variant == 31


# ------------------------------------------------------------ folded RMSNorm (prefill)
# Opt-in (DRTC_FOLD_NORM=1): measured 1.1 % SLOWER on the headline than materialising the
# norm (profiles/r3m: 19,575 / 19,553 vs 19,795 / 19,776 tok/s, one box, temporal stores for
# the residual stream) - the row statistic (epilogue shuffles + a row-statistic pass for the
# library's down) and the consumers' reads of the un-normalised stream cost more than the
# 41 us norm pass they replace.
_fold_norm = os.environ.get("DRTC_FOLD_NORM", "0") == "1"


def linear_residual_rinv(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor, eps: float):
    """residual += x @ w.T (in place, ``linear_residual``) and, when the 4-wave hand GEMM takes
    the shape, the next RMSNorm's row statistic from the same epilogue: returns (h, rinv) with
    rinv = rsqrt(mean(h^2) + eps) fp32 [M] (each row's partial sums of squares over 128
    columns from gemm_w4 W4_RESIDUAL_SQ, finished by rowsq_rinv_kernel).  (h, None) when the
    shape runs elsewhere."""
    M, K = x.shape
    N = w.shape[0]
    if not (_fold_norm and on_gpu(x) and M >= W4_MIN_M and N % 512 == 0):
        return linear_residual(x, w, residual), None
    rinv = torch.empty(M, dtype=torch.float32, device=x.device)
    if not w4_ok(x, w, residual):
        # a library GEMM (down, K > W4_MAX_K): the statistic from one read of the rows
        h = linear_residual(x, w, residual)
        check(hipk().row_rinv(rinv.data_ptr(), h.data_ptr(), M, N, h.stride(0), float(eps),
                              stream_ptr(x)), "row_rinv")
        return h, rinv
    sq = torch.empty((M, N // 128), dtype=torch.float32, device=x.device)
    # plain (temporal) stores: the next GEMM reads h itself, so h should stay in the MALL
    # (the non-temporal default would send the consumer's first pass to HBM)
    mfma_gemm(x, w, "residual_sq", residual=residual, out=residual, variant=W4_VARIANT + 2,
              group_m=w4_group_m(M, N, K), side=sq)
    check(hipk().rowsq_rinv(rinv.data_ptr(), sq.data_ptr(), M, N // 128, N, float(eps),
                            stream_ptr(x)), "rowsq_rinv")
    return residual, rinv


def rs_linear(h: torch.Tensor, w_folded: torch.Tensor, rinv: torch.Tensor,
              act: str | None = None) -> torch.Tensor | None:
    """norm(h) @ W.T as (h @ (W diag(g)).T) * rinv[row] on gemm_w4 (``w_folded`` = W with the
    RMSNorm weight g folded into its columns), with the gated activation in the epilogue when
    ``act`` is given (``w_folded`` = the fused [gate; up]); None when the shape cannot take it
    (the caller materialises the norm)."""
    if act is None:
        if not w4_ok(h, w_folded):
            return None
        M, K = h.shape
        return mfma_gemm(h, w_folded, "store_rs", variant=_w4v(K),
                         group_m=w4_group_m(M, w_folded.shape[0], K), side=rinv)
    if not (w4_glu_ok(h, w_folded, act) and h.shape[0] >= W4_MIN_M):
        return None
    M, K = h.shape
    return mfma_gemm(h, w_folded, act + "_rs", variant=_w4v(K),
                     group_m=w4_group_m(M, w_folded.shape[0] // 2, K, glu=True), side=rinv)


# ------------------------------------------------------------ 4-wave GEMM dispatch
W4_VARIANT = 7  # gemm_w4.hip through launch_gemm
# Persistent gemm_w4 (variant 15: min(tiles, CUs) workgroups, the next tile's first K tiles
# staged during the current tile's last two steps) for the single-slice calls.  Against the
# per-tile form in one process (profiles/r3r/probe.log): prefill qkv +0.5 %, o +2.0 %,
# gate_up+GLU +0.9 %, a 4400-row chunk's gate_up+GLU +2.3 %, decode gate_up+GLU at M = 1024
# +4.0 % (now level with hipBLASLt + act_glu); headline neutral (19,837 vs 19,836 tok/s, two
# runs each, one box).  DRTC_W4_PERSIST=0 restores the per-tile form.
W4_PERSIST = os.environ.get("DRTC_W4_PERSIST", "1") == "1"


def _w4v(K: int) -> int:
    """Schedule variant of a single-slice gemm_w4 call with reduction length K."""
    return 15 if W4_PERSIST and K >= 128 else W4_VARIANT


_w4_glu = os.environ.get("DRTC_W4_GLU", "1") != "0"
_w4_plain = os.environ.get("DRTC_W4_GEMM", "1") != "0"
# Prefill-sized passes (M >= W4_MIN_M rows) run the 4-wave hand GEMM (profiles/r3a_w4_gemm.md,
# Llama-3-8B at M = 16384, interleaved with the library in one process):
#   gate_up + SiLU-GLU epilogue  1.03-1.05x hipBLASLt + act_glu   -> hand (no act_glu pass)
#   qkv (store), o (+residual)   0.98-0.99x                        -> hand
#   down (K = 14336, +residual)  0.94-0.96x                        -> library (K > W4_MAX_K)
# Decode buckets (M <= 1024) keep the tuned library / skinny / medium-M kernels.
# gate_up + GLU also wins at the larger decode buckets: 1.04x at M = 768, 1.06x at 1024
# (library + act_glu), 0.97x at 512, 0.72x at 256 (profiles/r3b_w4_decode.md)
W4_GLU_MIN_M = int(os.environ.get("DRTC_W4_GLU_MIN_M", "640"))
W4_MIN_M = int(os.environ.get("DRTC_W4_MIN_M", "4096"))
W4_MAX_K = int(os.environ.get("DRTC_W4_MAX_K", "8192"))
# Decode buckets with few 256 x 256 tiles and a long K (Llama-3-8B down at M = 1024: 64 tiles,
# K = 14336) can run gemm_w4 with the reduce-scatter split-K (variant 11): 1.13x the library
# in isolation (weights cache-resident between calls), but 142 vs ~116 us inside the decode
# step, where the weights stream from HBM (profiles/r3b_w4_decode.md) - off by default
# (DRTC_W4_RS_MIN_M=768 turns it on).
W4_RS_MIN_M = int(os.environ.get("DRTC_W4_RS_MIN_M", "100000"))  # off: see below
W4_RS_MIN_K = int(os.environ.get("DRTC_W4_RS_MIN_K", "8192"))
W4_RS_CUS = 256  # every workgroup resident: tiles x splitk <= CUs (MI355X)


# Full-batch decode projections on gemm_w4 with the last-arriver split-K (variant 7):
# (N, K) -> K slices, for the decode buckets M >= W4_DEC_MIN_M, where it measured faster
# than the tuned library with the weights streamed from HBM (scripts/gpu_r3e_probe.sh,
# w4_probe.py --rotate).  DRTC_W4_DEC="N:K:S,..." replaces the table ("" = off).
W4_DEC_MIN_M = int(os.environ.get("DRTC_W4_DEC_MIN_M", "768"))
W4_DEC: dict[tuple[int, int], int] = {}
if "DRTC_W4_DEC" in os.environ:
    W4_DEC = {(int(a), int(b)): int(c) for a, b, c in
              (e.split(":") for e in os.environ["DRTC_W4_DEC"].split(",") if e)}


def w4_dec_splitk(M: int, N: int, K: int) -> int:
    """K slices of the decode-bucket gemm_w4 form for y[M, N] = x[M, K] W^T (0: not taken)."""
    if not (W4_DEC and _w4_plain and W4_DEC_MIN_M <= M <= DECODE_MAX_M):
        return 0
    sk = W4_DEC.get((N, K), 0)
    if not sk or N % 256 or K % 64 or (K // 64) % sk:
        return 0
    return sk


# Full-batch decode o / down projections as gemm_w4 split-K WITHOUT an in-kernel combine:
# every K slice writes an fp32 partial plane and the residual-add + RMSNorm that follows the
# projection anyway sums the planes (ops.norm.rmsnorm_partials) - all CUs busy in the GEMM
# (64 tiles x 4 slices at M = 1024, N = 4096) and the reduction spread over every row's
# workgroup at HBM rate.  (N, K) -> slices; DRTC_W4_PARTIAL="N:K:S,..." replaces the table.
W4_PARTIAL_MIN_M = int(os.environ.get("DRTC_W4_PARTIAL_MIN_M", "768"))
W4_PARTIAL: dict[tuple[int, int], int] = {}
if "DRTC_W4_PARTIAL" in os.environ:
    W4_PARTIAL = {(int(a), int(b)): int(c) for a, b, c in
                  (e.split(":") for e in os.environ["DRTC_W4_PARTIAL"].split(",") if e)}
PARTIALS_BYTES = 64 << 20  # fp32 planes (per device): 4 x 1024 x 4096


class Partials:
    """fp32 split-K partial planes [sk, M, N] standing for the bf16 output of y = x @ w.T
    (gemm_w4 W4_PARTIAL).  Only ``ops.PendingNorm`` consumes one (materialize() sums the
    planes inside the residual-add + RMSNorm kernel); the tensor-like attributes serve the
    dispatch checks that look at a pending norm's input."""

    __slots__ = ("planes", "sk")
    dtype = torch.bfloat16  # the dtype of the value it stands for
    is_cuda = True

    def __init__(self, planes: torch.Tensor, sk: int):
        self.planes, self.sk = planes, sk

    @property
    def shape(self):
        return self.planes.shape[1:]

    @property
    def device(self):
        return self.planes.device

    def dim(self) -> int:
        return 2

    def stride(self, d: int | None = None):
        st = (self.planes.shape[2], 1)
        return st if d is None else st[d]

    def data_ptr(self) -> int:
        return self.planes.data_ptr()


_pws: dict[int, torch.Tensor] = {}


def partials_workspace(dev: torch.device) -> torch.Tensor:
    """The device's fp32 partial-plane buffer (one producer / consumer pair at a time on the
    engine's stream; allocated on first use, in the eager run ahead of a graph capture)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    buf = _pws.get(key)
    if buf is None:
        with _ws_lock:
            buf = _pws.get(key)
            if buf is None:
                buf = torch.empty(PARTIALS_BYTES // 4, dtype=torch.float32, device=dev)
                _pws[key] = buf
    return buf


def w4_partial_splitk(M: int, N: int, K: int) -> int:
    if not (W4_PARTIAL and _w4_plain and W4_PARTIAL_MIN_M <= M <= DECODE_MAX_M):
        return 0
    sk = W4_PARTIAL.get((N, K), 0)
    if not sk or N % 256 or K % 64 or (K // 64) % sk or sk * M * N * 4 > PARTIALS_BYTES:
        return 0
    return sk


def linear_partials(x: torch.Tensor, w: torch.Tensor):
    """y = x @ w.T for a projection whose output only feeds the next pending norm (decode
    o / down at TP = 1): a ``Partials`` when the split-K partial-plane form is configured
    for the shape, else ``linear``'s tensor."""
    if (on_gpu(x) and x.dim() == 2 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and x.stride(1) == 1 and w.is_contiguous() and x.stride(0) % 8 == 0
            and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0):
        M, K = x.shape
        N = w.shape[0]
        sk = w4_partial_splitk(M, N, K)
        if sk:
            planes = partials_workspace(x.device)[:sk * M * N].view(sk, M, N)
            check(hipk().gemm(0, x.data_ptr(), w.data_ptr(), 0, M, N, K, x.stride(0),
                              w.stride(0), N, 0, EPI["partial"], 0, W4_VARIANT, sk, 4,
                              planes.data_ptr(), planes.numel() * 4, 0, 0, stream_ptr(x)),
                  "gemm partial")
            return Partials(planes, sk)
    return linear(x, w)


def w4_rs_splitk(M: int, N: int, K: int) -> int:
    """Split of the reduce-scatter decode form for y[M, N] = x[M, K] W^T, 0 = not taken."""
    if not (_w4_plain and W4_RS_MIN_M <= M <= DECODE_MAX_M and K >= W4_RS_MIN_K
            and N % 256 == 0 and K % 64 == 0):
        return 0
    tiles = -(-M // 256) * (N // 256)
    for sk in (4, 2):
        if tiles * sk <= W4_RS_CUS and (K // 64) % sk == 0:
            return sk
    return 0


def w4_group_m(M: int, N: int, K: int, glu: bool = False) -> int:
    """Row-tile group of the XCD-aware tile order (scripts/gpu_w4_groups.sh): a group's A
    panels must stay cache-resident while it sweeps the columns - 2 for the long-K down
    projection (7 MB per 256-row panel), 8 for the gated gate_up, 4 otherwise."""
    if K >= 12288:
        return 2
    return 8 if glu else 4


def w4_ok(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None = None) -> bool:
    """Whether a prefill-sized projection y = x @ w.T (+ residual) takes gemm_w4."""
    if not (_w4_plain and on_gpu(x) and _enabled and x.dim() == 2 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and w.is_contiguous() and x.stride(1) == 1):
        return False
    M, K = x.shape
    N = w.shape[0]
    if not (M >= W4_MIN_M and K <= W4_MAX_K and K % 64 == 0 and N % 256 == 0
            and w.shape[1] == K and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0
            and w.data_ptr() % 16 == 0):
        return False
    if residual is not None:
        return (residual.dim() == 2 and residual.shape == (M, N) and residual.stride(1) == 1
                and residual.stride(0) % 8 == 0 and residual.data_ptr() % 16 == 0
                and residual.dtype == torch.bfloat16)
    return True


def w4_glu_ok(x: torch.Tensor, w: torch.Tensor, act: str) -> bool:
    """Whether ``norm_glu`` takes the fused-GLU hand GEMM for x [M, K] @ [gate; up]^T."""
    if not (_w4_glu and on_gpu(x) and _enabled and x.dim() == 2 and act in ("silu", "gelu_tanh")
            and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.is_contiguous()
            and x.stride(1) == 1):
        return False
    M, K = x.shape
    N2 = w.shape[0]
    return (M >= W4_GLU_MIN_M and K % 64 == 0 and w.shape[1] == K and N2 % 256 == 0
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0)


def norm_glu(p, w: torch.Tensor, act: str = "silu",
             w_folded: torch.Tensor | None = None) -> torch.Tensor:
    """h = act(norm(x) @ gate^T) * (norm(x) @ up^T) for an ``ops.PendingNorm`` p and the
    fused [gate; up] weight: on the 4-wave hand GEMM with the GLU in its epilogue when
    ``w4_glu_ok`` (one launch, no [M, 2I] intermediate), else norm_linear + act_glu."""
    from .activation import act_glu

    if p.rinv is not None and p._out is None and w_folded is not None:
        y = rs_linear(p.x, w_folded, p.rinv, act)  # folded norm (see norm_linear)
        if y is not None:
            return y
    if w4_glu_ok(p.x, w, act):
        x = p.materialize()
        M, K = x.shape
        return mfma_gemm(x, w, act, variant=_w4v(K),
                         group_m=w4_group_m(M, w.shape[0] // 2, K, glu=True))
    return act_glu(norm_linear(p, w), act)


__all__ = ["linear", "norm_linear", "glu_linear", "norm_glu", "w4_glu_ok", "skinny_linear", "skinny_ok", "skinny_variant",
           "skinny_supports", "mfma_gemm", "midm_gemm", "midm_supported", "dec_gemm", "dec_supported",
           "tune", "save_entries", "w4_ok", "w4_group_m", "w4_rs_splitk", "w4_dec_splitk",
           "Partials", "linear_partials", "w4_partial_splitk", "linear_residual_rinv", "rs_linear",
           "load_table", "reset", "set_enabled", "table_path"]


# ------------------------------------------------------------------ medium-M decode GEMM
MIDM_EPI = {"store": 0, "residual": 1, "silu": 2, "gelu_tanh": 3, "partial": 4, "residual_sq": 5,
       "store_rs": 6, "silu_rs": 7, "gelu_tanh_rs": 8}
MIDM_MAX_M = 256


def midm_splits(M: int, N: int, K: int, target_wgs: int | None = None) -> int:
    """K splits of the medium-M GEMM: the largest S <= 16 with K a multiple of
    256 S (whole 4-chunk register rings per split) and at most ~2 workgroups
    per CU (one above 128 rows, where the kernel runs one workgroup per CU)."""
    if target_wgs is None:
        target_wgs = 256 if M > 128 else 512
    nb = N // 128
    ring = 64 * midm_depth(M)
    best = 1
    for s in range(1, 17):
        if K % (ring * s) == 0 and nb * s <= target_wgs:
            best = s
    return best


def midm_depth(M: int) -> int:
    """Chunks of 64 k in flight per wave (gemm_midm.hip mid_depth)."""
    return 4


def midm_supported(M: int, N: int, K: int, epi: str = "store") -> bool:
    return (1 <= M <= MIDM_MAX_M and N % 128 == 0 and K % (64 * midm_depth(M)) == 0
            and epi in MIDM_EPI
            and (epi not in ("silu", "gelu_tanh") or (N // 2) % 4 == 0))


def midm_gemm(x: torch.Tensor, w: torch.Tensor, epi: str = "store",
              residual: torch.Tensor | None = None, out: torch.Tensor | None = None,
              splits: int | None = None) -> torch.Tensor:
    """Medium-M (17..256 rows) decode GEMM, csrc/kernels/gemm_midm.hip:
    y = x @ w^T with a store / residual (y = residual + x w^T, in place when
    out is residual) / SiLU- or GELU-gated [gate | up] epilogue.  W streams
    once from HBM into registers, x is shared through LDS, K is split over
    workgroups and the fp32 partials summed by a second small kernel."""
    M, K = x.shape
    N = w.shape[0]
    assert x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.is_cuda
    assert x.stride(1) == 1 and w.is_contiguous() and w.shape[1] == K
    assert midm_supported(M, N, K, epi), (M, N, K, epi)
    S = splits or midm_splits(M, N, K)
    while S > 1 and S * M * N * 4 > WS_SLAB_BYTES:
        S //= 2
    NO = N // 2 if epi in ("silu", "gelu_tanh") else N
    if out is None:
        out = residual if (epi == "residual" and residual is not None) else \
            torch.empty((M, NO), dtype=x.dtype, device=x.device)
    assert out.shape == (M, NO) and out.stride(1) == 1
    if epi == "residual":
        assert residual is not None and residual.shape == (M, N) and residual.stride(1) == 1
    slab = gemm_workspace(x.device)[0]
    check(hipk().midm_gemm(out.data_ptr(), x.data_ptr(), w.data_ptr(), ptr(residual), M, N, K,
                           x.stride(0), out.stride(0),
                           residual.stride(0) if residual is not None else 0, MIDM_EPI[epi], S,
                           slab.data_ptr(), slab.numel() * 4, stream_ptr(x)), "midm_gemm")
    return out


# ------------------------------------------------------------------ decode-batch GEMM
DEC_EPI = {"store": 0, "residual": 1, "silu": 2, "gelu_tanh": 3, "partial": 4, "residual_sq": 5,
       "store_rs": 6, "silu_rs": 7, "gelu_tanh_rs": 8}


def dec_supported(M: int, N: int, K: int, epi: str = "store") -> bool:
    """Shapes csrc/kernels/gemm_dec.hip covers: K % 64, N % 128 (N/2 % 64 gated)."""
    glu = epi in ("silu", "gelu_tanh")
    return (M >= 1 and K % 64 == 0 and epi in DEC_EPI
            and ((N // 2) % 64 == 0 and N % 2 == 0 if glu else N % 128 == 0))


def dec_gemm(x: torch.Tensor, w: torch.Tensor, epi: str = "store",
             residual: torch.Tensor | None = None, out: torch.Tensor | None = None,
             nr: int = 8, group_m: int = 8, pipe: int = 2) -> torch.Tensor:
    """Decode-batch GEMM (csrc/kernels/gemm_dec.hip): y = epi(x @ w.T) on 128 x 128 tiles
    with the K loop split over two wave groups of each workgroup (one tile per CU at
    M = 1024, N = 4096; no cross-workgroup reduction).  ``epi`` as ``mfma_gemm``; ``nr``
    = LDS regions (4: 64 KiB, two workgroups per CU; 6 / 8: 96 / 128 KiB, deeper
    prefetch); ``pipe`` 1 = fragments read after each barrier, 2 = fragments double-
    buffered in registers with the DMA spread over the MFMAs."""
    M, K = x.shape
    glu = epi in ("silu", "gelu_tanh")
    N = w.shape[0] // 2 if glu else w.shape[0]
    assert x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.is_cuda
    assert x.stride(1) == 1 and w.is_contiguous() and w.shape[1] == K
    assert dec_supported(M, w.shape[0], K, epi), (M, w.shape[0], K, epi)
    if out is None:
        out = residual if (epi == "residual" and residual is not None) else \
            torch.empty((M, N), dtype=x.dtype, device=x.device)
    assert out.shape == (M, N) and out.stride(1) == 1
    if epi == "residual":
        assert residual is not None and residual.shape == (M, N) and residual.stride(1) == 1
    check(hipk().gemm_dec(out.data_ptr(), x.data_ptr(), w.data_ptr(), ptr(residual), M, N, K,
                          x.stride(0), w.stride(0), out.stride(0),
                          residual.stride(0) if residual is not None else 0, DEC_EPI[epi],
                          N if glu else 0, 10 * pipe + nr, group_m, stream_ptr(x)), "gemm_dec")
    return out
