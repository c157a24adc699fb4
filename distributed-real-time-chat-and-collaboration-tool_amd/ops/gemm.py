"""Projection GEMMs: one table-driven router over the hand kernels and tuned hipBLASLt.

``linear(x, w)`` computes ``x @ w.T`` (bf16, fp32 accumulate).  Every call resolves its
shape (M, N, K, row stride of x) ONCE to a route, cached per shape (``route``):

  kind      kernel                                          taken for
  "w4"      gemm_w4.hip: 4-wave hand-scheduled MFMA GEMM,   prefill-sized passes (M >= W4_MIN_M,
            persistent, 256 x 256 tiles (``mfma_gemm``)     K <= W4_MAX_K)
  "skinny"  gemv.hip weight-streaming kernels (M <= 16)     decode buckets where the table (or
                                                            ``skinny_variant`` untuned) says so
  "midm"    gemm_midm.hip medium-M kernel (M <= 256)        decode buckets where the table says so
  "xd"      gemm_xd.hip: 128-row tiles, full K, tile order  decode buckets where the table says so
            partitioned by XCD (``xd_gemm``)                (full-batch qkv / o / down)
  "lt"      hipBLASLt with the per-shape measured solution  the other decode buckets, and
            (``csrc/kernels/gemm_lt.cpp``)                  prefill shapes the hand GEMM does not
                                                            take (tuned at the nearest M)
  "torch"   torch.nn.functional.linear (on the GPU:         decode buckets where the tuner measured
            hipBLASLt's heuristic pick)                     that pick fastest; CPU

The tuning table (``ops/tuned/gemm_<arch>.json``, keyed by the hipBLASLt version) holds, per
model decode shape and hipGraph batch bucket, the fastest measured choice among the library
solutions and the hand kernels (``scripts/tune_gemms.py``, ``tune_skinny.py``,
``tune_midm.py``, ``tune_prefill.py``); a bucket without an entry measured the library's
heuristic pick (torch's path) fastest.  A decode M that is not a bucket (e.g. an engine
``max_batch`` of 208) takes what the bucket above it measured (224: the bucket its hipGraph
batch would pad to), not an unmeasured guess.

The full-batch gate_up projection with its SiLU/GELU-GLU epilogue and the prefill o / down
projections with the residual add in their epilogue do not go through ``linear``: see
``norm_glu`` and ``linear_residual``.
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
#                   medium-M kernel K splits or 0, gemm_xd form or 0, gemm_xd gated form for
#                   a [gate; up] weight or 0): the decode buckets of the tuning table
_table: dict[tuple[int, int, int, int], tuple[int, int, int, int, int]] | None = None
# (N, K, ldx) -> sorted [(tuned M, algo, beats F.linear, beats addmm_)]: prefill entries
_prefill: dict[tuple[int, int, int], list[tuple[int, int, bool, bool]]] = {}
# (M, N, K, ldx, beta) -> algo chosen for a prefill-sized call (-1: torch's path)
_prefill_pick: dict[tuple[int, int, int, int, int], int] = {}
# (M, N, K, ldx) -> resolved route (kind, arg)
_routes: dict[tuple[int, int, int, int], tuple[str, int]] = {}
DECODE_MAX_M = 1024  # decode buckets end here; larger M are prefill (or mixed) passes
# the decode batch buckets (hipGraph captures, engine/decode_runner.py) the tuner measured
DECODE_BUCKETS = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256, 320, 384,
                  448, 512, 640, 768, 896, 1024)
_enabled = os.environ.get("DRTC_TUNED_GEMM", "1") != "0"
_prefill_enabled = os.environ.get("DRTC_PREFILL_TUNED", "1") != "0"
_midm_enabled = os.environ.get("DRTC_MIDM_GEMM", "1") != "0"
_xd_enabled = os.environ.get("DRTC_XD_GEMM", "1") != "0"
# tuned gemm_xd forms whose batch fits one row tile take non-temporal weight loads (each weight
# byte enters one CU once: MI355X_MICROARCH.md nt-weights; profiles/r4aa: Llama-3-70B down at
# M = 256 159.6 -> 136.8 us, gated gate_up 265.7 -> 230.2, the 70B ask wave +5.2 %)
_xd_nt = os.environ.get("DRTC_XD_NT", "1") != "0"
# decode batches up to this many rows may take the skinny kernel: the table's choice where
# the shape was measured, skinny_variant()'s default otherwise; 0 disables it
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
    """Parse the entries of the running hipBLASLt version (no GPU work; a library entry is
    registered with the native plan cache on its first use, outside graph capture)."""
    global _table
    if _table is not None:
        return _table
    with _lock:
        if _table is not None:
            return _table
        tab: dict[tuple[int, int, int, int], tuple[int, int, int, int, int]] = {}
        pre: dict[tuple[int, int, int], list[tuple[int, int, bool, bool]]] = {}
        if _enabled and torch.cuda.is_available():
            ver = str(hipk().lt_version())
            for ks, e in load_table().get(ver, {}).items():
                M, N, K, ldx = (int(v) for v in ks.split(","))
                if e.get("prefill"):
                    if _prefill_enabled:
                        pre.setdefault((N, K, ldx), []).append(
                            (M, int(e["algo"]), bool(e.get("beta0")), bool(e.get("beta1"))))
                    if not e.get("xd"):
                        continue
                    # a prefill-table shape that is also a decode batch above the buckets
                    # (Gemma-2B's 2048 rows) with a measured gemm_xd winner: the gemm_xd form
                    # only (its library algo stays with the prefill table)
                    tab[(M, N, K, ldx)] = (-1, 0, 0, int(e["xd"]), 0)
                    continue
                nt_tuned = bool(e.get("nt_tuned"))
                tab[(M, N, K, ldx)] = (int(e.get("algo", -1)), int(e.get("skinny", 0)),
                                       int(e.get("midm", 0)) if _midm_enabled else 0,
                                       _xd_policy(M, int(e.get("xd", 0)), nt_tuned),
                                       _xd_policy(M, int(e.get("xd_glu", 0)), nt_tuned))
        for v in pre.values():
            v.sort()
        _prefill.clear()
        _prefill.update(pre)
        _prefill_pick.clear()
        _routes.clear()
        _table = tab
    return _table


def xd_nt_ok(M: int, form: int) -> bool:
    """Whether ``form`` (plain) has a non-temporal build and M fits one of its row tiles."""
    mt, nf, _ = xd_form(form)
    return form < 1000 and (mt, nf) in XD_NT_TILES and M <= 128 * mt


def _xd_policy(M: int, form: int, nt_tuned: bool = False) -> int:
    """A tuned gemm_xd form as the router runs it (0: none / gemm_xd disabled).  An entry the
    tuner measured with the non-temporal forms among its candidates (``nt_tuned``: the
    profiles/r4ab re-tune, M = 128-256) runs exactly the form it picked - a plain winner
    stays plain; a plain form picked before the nt forms existed takes its nt twin where the
    batch fits one row tile.  DRTC_XD_NT=0 runs every form plain (an nt pick included)."""
    if not (_xd_enabled and form):
        return 0
    if not _xd_nt:
        return form % 1000
    if not nt_tuned and xd_nt_ok(M, form):
        return form + 1000
    return form


def reset() -> None:
    """Forget the activated table and every resolved route (tests / after re-tuning)."""
    global _table
    with _lock:
        _table = None
        _routes.clear()


def set_enabled(on: bool) -> None:
    global _enabled
    _enabled = bool(on)
    reset()


# ------------------------------------------------------------------ routing
def _decode_entry(M: int, N: int, K: int,
                  ldx: int) -> tuple[int, tuple[int, int, int, int, int]] | None:
    """(tuned bucket, entry) for a decode-sized shape, None for torch's (hipBLASLt heuristic)
    path.  The tuner measured every (model shape, DECODE_BUCKETS M) and kept an entry only
    where something beat the heuristic pick, so a bucket without an entry means "the
    heuristic".  A non-bucket M takes what its bucket above - the bucket the hipGraph of that
    batch would pad to - measured."""
    tab = _activate()
    ent = tab.get((M, N, K, ldx))
    if ent is not None:
        return M, ent
    if M in DECODE_BUCKETS:
        return None
    Mt = next((b for b in DECODE_BUCKETS if b >= M), None)
    if Mt is None:
        return None
    ent = tab.get((Mt, N, K, ldx))
    return (Mt, ent) if ent is not None else None


def _prefill_algo(M: int, N: int, K: int, ldx: int, beta: int) -> int:
    """Solution for a prefill-sized library GEMM: the entry tuned at the M nearest to this one
    (log scale, within 2x) for the same (N, K, ldx), if it beat torch's pick for this beta;
    -1 = use torch's path.  The native plan is per exact M (registered on first use, outside
    graph capture: prefill passes run eagerly)."""
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


def _resolve(M: int, N: int, K: int, ldx: int) -> tuple[str, int]:
    tab = _activate()
    ent = tab.get((M, N, K, ldx))
    if M > DECODE_MAX_M and ent is not None and _xd_big_m and ent[3] and xd_supported(M, N, K, ent[3]):
        # a decode batch above the 1024 buckets with a measured gemm_xd winner (Gemma-2B's
        # 2048: qkv / o / down, profiles/r6ak)
        return ("xd", ent[3])
    if M > DECODE_MAX_M and ent is not None and ent[0] >= 0:
        # a decode batch above the 1024 buckets that was tuned as such (Gemma-2B's 2048)
        with _lock:
            if hipk().lt_set_algo(M, N, K, ldx, N, ent[0]) == 0:
                return ("lt", ent[0])
    if M > DECODE_MAX_M:
        if w4_shape_ok(M, N, K):
            return ("w4", 0)
        a = _prefill_algo(M, N, K, ldx, 0)
        return ("lt", a) if a >= 0 else ("torch", 0)
    found = _decode_entry(M, N, K, ldx)
    if found is None:
        v = skinny_variant(M, N, K, ldx)
        return ("skinny", v) if v else ("torch", 0)
    _, (algo, sk, midm, xd, _) = found
    if algo < 0 and not (sk or midm or xd):
        return ("torch", 0)  # measured: the library's heuristic pick beat every candidate
    if sk and M <= SKINNY_MAX_M and skinny_supports(sk, M, N, K, ldx):
        return ("skinny", sk)
    if xd and xd_supported(M, N, K, xd):
        return ("xd", xd)
    if midm and midm_supported(M, N, K):
        return ("midm", midm)
    if algo >= 0:
        with _lock:  # the native plan is per exact M: validate the solution at this M
            if hipk().lt_set_algo(M, N, K, ldx, N, algo) == 0:
                return ("lt", algo)
    v = skinny_variant(M, N, K, ldx)
    return ("skinny", v) if v else ("torch", 0)


# DRTC_XD_BIG_M=0: decode batches above DECODE_MAX_M ignore tuned gemm_xd entries (A/B knob)
_xd_big_m = os.environ.get("DRTC_XD_BIG_M", "1") != "0"


def route(M: int, N: int, K: int, ldx: int) -> tuple[str, int]:
    """The kernel ``linear`` runs for y[M, N] = x[M, K] @ W[N, K]^T with x's row stride ldx on
    the GPU: (kind, arg) as in the module docstring, resolved once per shape."""
    key = (M, N, K, ldx)
    r = _routes.get(key)
    if r is None:
        r = _resolve(M, N, K, ldx)
        _routes[key] = r
    return r


def _gpu_bf16(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (on_gpu(x) and _enabled and x.dim() == 2 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.stride(1) == 1 and w.is_contiguous())


def _aligned(x: torch.Tensor, w: torch.Tensor) -> bool:
    return x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0


def linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """y = x @ w.T for x [M, K] (row stride ldx), w [N, K] contiguous."""
    if not _gpu_bf16(x, w):
        return F.linear(x, w)
    M, K = x.shape
    N = w.shape[0]
    kind, arg = route(M, N, K, x.stride(0))
    if kind == "w4" and _aligned(x, w):
        return mfma_gemm(x, w, "store", variant=_w4v(K), group_m=w4_group_m(M, N, K))
    if kind == "lt":
        y = torch.empty((M, N), dtype=x.dtype, device=x.device)
        check(hipk().lt_gemm(y.data_ptr(), x.data_ptr(), w.data_ptr(), M, N, K, x.stride(0), N,
                             0.0, stream_ptr(x)), "lt_gemm")
        return y
    if kind == "skinny":
        return skinny_linear(x, w, arg)
    if kind == "midm":
        return midm_gemm(x, w, "store", splits=arg)
    if kind == "xd" and _aligned(x, w):
        return xd_gemm(x, w, form=arg)
    return F.linear(x, w)


# ------------------------------------------------------------------ skinny decode kernels
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
    """Default skinny-kernel form for an untuned shape: 1 = VALU dot2 for M <= 2, 3 = MFMA
    (1 tile, 8 K-split waves) up to M = 8; 0 = leave it to the library."""
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


def _choice(M: int, N: int, K: int, ldx: int) -> int:
    """Skinny variant ``linear`` runs for this shape (0 = another kernel)."""
    kind, arg = route(M, N, K, ldx)
    return arg if kind == "skinny" else 0


# ------------------------------------------------------------------ fused forms
_fuse_residual = os.environ.get("DRTC_RESIDUAL_GEMM", "1") != "0"
# measured (scripts/residual_gemm_bench.py, MI355X, H=4096): at 16k rows the beta=1 GEMM
# costs the same as beta=0 while the following RMSNorm drops from ~90 us (read x + residual,
# write both) to ~39 us (read h, write out); at 1024 rows both norms are launch-latency
# bound (7-8 us) - no gain
RESIDUAL_FUSE_MIN_M = 4096


def residual_fusable(x: torch.Tensor, residual: torch.Tensor) -> bool:
    """Whether ``linear_residual`` pays for x [M, K] -> residual [M, N]: on the GPU at
    prefill-sized M (bf16).  Elsewhere the caller runs ``linear`` and leaves the add to the
    next fused add-RMSNorm."""
    return (_fuse_residual and on_gpu(x) and x.dim() == 2 and x.shape[0] >= RESIDUAL_FUSE_MIN_M
            and x.dtype == residual.dtype == torch.bfloat16
            and residual.dim() == 2 and residual.shape[0] == x.shape[0]
            and residual.stride(1) == 1)


def linear_residual(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
    """residual += x @ w.T with the add in the GEMM epilogue (in place into the residual
    stream), for the o / down projections of a prefill pass; returns the updated residual.
    One rounding to bf16 (of the fp32 accumulator plus the residual) instead of two."""
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


def norm_linear(p, w: torch.Tensor) -> torch.Tensor:
    """y = rmsnorm(p.x [+ p.residual]) @ w.T for an ``ops.PendingNorm`` p.

    When the projection would run on the skinny dot2 kernel anyway (small decode batches,
    measured per shape) the norm is fused into it (gemv.hip ``skinny_norm_gemm_kernel``):
    one launch instead of two, and the new residual stream is written by the GEMM.
    Otherwise the norm is materialised and ``linear`` runs."""
    x, res = p.x, p.residual
    if (_fuse_norm and p._out is None and p.pc is None and isinstance(x, torch.Tensor)
            and _gpu_bf16(x, w) and p.w.is_contiguous()
            and (res is None or (res.stride(1) == 1 and res.shape == x.shape))):
        M, K = x.shape
        N = w.shape[0]
        if (M <= NORM_FUSE_MAX_M and K % 2048 == 0 and K <= 8192 and N % 4 == 0
                and x.stride(0) % 8 == 0 and (res is None or res.stride(0) % 8 == 0)
                and _choice(M, N, K, K) == 1):
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
    """y = (act(gu[:, :I]) * gu[:, I:]) @ w.T (the down projection of a gated MLP).  When the
    projection would run on the skinny dot2 kernel the activation is computed inside it while
    loading its input (gemv.hip, no act_glu launch); otherwise ops.act_glu + linear."""
    from .activation import act_glu

    if _fuse_glu and _gpu_bf16(gu, w) and act in ("silu", "gelu_tanh"):
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
EPI = {"store": 0, "residual": 1, "silu": 2, "gelu_tanh": 3}
_ws_lock = threading.Lock()
_ws: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}
WS_SLAB_BYTES = 128 << 20   # fp32 split-K slabs (per device)
WS_COUNTERS = 1 << 16


# every split-K workspace created in this process (the shared per-device ones and the private
# ones of second streams): check_splitk_fault reads the fault word of each
_all_ws: list[tuple[torch.Tensor, torch.Tensor]] = []


# per-thread override of the device workspace: GEMMs issued inside ``private_workspace(ws)``
# (the second micro-batch stream of a decode step) use ``ws``
_ws_local = threading.local()


class private_workspace:
    """Context manager: every split-K / medium-M GEMM issued by this thread inside it takes
    ``ws`` (from ``new_gemm_workspace``) instead of the device's shared workspace - for GEMMs
    that run concurrently with the shared workspace's users on another stream."""

    def __init__(self, ws: tuple[torch.Tensor, torch.Tensor] | None):
        self.ws = ws

    def __enter__(self):
        self.prev = getattr(_ws_local, "ws", None)
        _ws_local.ws = self.ws
        return self.ws

    def __exit__(self, *exc):
        _ws_local.ws = self.prev
        return False


def gemm_workspace(dev: torch.device) -> tuple[torch.Tensor, torch.Tensor]:
    """Split-K workspace of a device: fp32 slabs + per-tile arrival counters (zeroed once;
    the last arriver of each tile re-arms its counter; the LAST counter is the fault word,
    ``check_splitk_fault``).  One per device, shared by every GEMM on the engine's stream (and
    the medium-M kernel's partial slabs); a GEMM issued concurrently on another stream passes
    its own (``ws=``, or ``private_workspace``).  Created before any graph capture (the
    engine's eager warm-up does)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    own = getattr(_ws_local, "ws", None)
    if own is not None and own[0].device.index == key:
        return own
    ws = _ws.get(key)
    if ws is None:
        with _ws_lock:
            ws = _ws.get(key)
            if ws is None:
                ws = (torch.empty(WS_SLAB_BYTES // 4, dtype=torch.float32, device=dev),
                      torch.zeros(WS_COUNTERS, dtype=torch.int32, device=dev))
                _ws[key] = ws
                _all_ws.append(ws)
    return ws


def new_gemm_workspace(dev: torch.device) -> tuple[torch.Tensor, torch.Tensor]:
    """A private split-K workspace (for GEMMs on a second stream)."""
    ws = (torch.empty(WS_SLAB_BYTES // 4, dtype=torch.float32, device=dev),
          torch.zeros(WS_COUNTERS, dtype=torch.int32, device=dev))
    with _ws_lock:
        _all_ws.append(ws)
    return ws


class SplitKFault(RuntimeError):
    """A split-K combine gave up waiting for another slice's partial (gemm_xd / gemm_w4): the
    GEMM that recorded it stored a wrong sum."""


def check_splitk_fault(dev: torch.device | None = None) -> None:
    """Read the fault word (the last counter) of every split-K workspace on ``dev`` (all
    devices: None).  A combine whose poll for the other slices timed out sets it and leaves
    its tile's counters un-armed, so on a fault the counters are zeroed (the next GEMM starts
    clean) and SplitKFault is raised.  Synchronises with the workspace's device: call it after
    warm-up / graph capture and from health checks, not per GEMM."""
    if dev is not None:
        dev = torch.device(dev)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
    with _ws_lock:
        wss = list(_all_ws)
    for slab, cnt in wss:
        if dev is not None and cnt.device != dev:
            continue
        if int(cnt[-1].item()):
            cnt.zero_()
            raise SplitKFault(f"split-K combine timed out on {cnt.device}: a GEMM result since "
                              "the last check is wrong (counters reset)")


class SplitKWatch:
    """Per-step split-K fault detection without a device sync, for one device.

    ``poll()`` (the engine calls it after every step) enqueues, on the current stream, a copy of
    every split-K workspace's fault word into pinned host memory and records an event; a later
    poll reads those words once the event has completed.  A combine that timed out is therefore
    reported one step after the step that ran it (two when the GPU runs a step behind the host),
    instead of up to ``HEALTH_EVERY`` steps later with a blocking read.  On a fault the device's
    counters are zeroed (the next GEMMs start clean) and SplitKFault is raised - or, with
    ``raise_=False``, True is returned."""

    def __init__(self, dev: torch.device):
        dev = torch.device(dev)
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.dev = dev
        self._host: torch.Tensor | None = None
        self._ev = None
        self._n = 0

    def _counters(self) -> list[torch.Tensor]:
        with _ws_lock:
            return [cnt for _, cnt in _all_ws if cnt.device == self.dev]

    def poll(self, raise_: bool = True) -> bool:
        if self.dev.type != "cuda":
            return False
        if self._ev is not None and self._ev.query():
            fault = bool(self._host[:self._n].any())
            self._ev = None
            if fault:
                for cnt in self._counters():
                    cnt.zero_()
                if raise_:
                    raise SplitKFault(f"split-K combine timed out on {self.dev}: a GEMM result "
                                      "of the last steps is wrong (counters reset)")
                return True
        if self._ev is None:
            cnts = self._counters()
            if not cnts:
                return False
            if self._host is None or self._host.numel() < len(cnts):
                self._host = torch.zeros(max(4, len(cnts)), dtype=torch.int32, pin_memory=True)
            for i, cnt in enumerate(cnts):
                self._host[i:i + 1].copy_(cnt[-1:], non_blocking=True)
            self._n = len(cnts)
            self._ev = torch.cuda.Event()
            self._ev.record()
        return False


def set_splitk_spin_limit(limit: int) -> int:
    """Bound of the split-K combines' poll for the other slices (polls of ~64 cycles;
    default 1 << 24); < 0 makes every combine fault (tests).  Returns the previous bound."""
    prev = int(hipk().splitk_spin_limit())
    hipk().set_splitk_spin_limit(int(limit))
    return prev


def gemm_w4_variant(variant: int) -> bool:
    """mfma_gemm variants: 7 per-tile (split-K with the last-arriver combine), 9 the same
    with temporal epilogue stores, 11 / 13 per-tile with the parallel split-K combine (every
    slice finishes a row band of its tile; the grid must fit the CUs), 15 persistent, 31
    persistent with the per-XCD K rotation, 47 / 63 those two with the next tile's fragment
    reads spread over half 1."""
    return variant in (7, 9, 11, 13, 15, 31, 47, 63)


def mfma_gemm(x: torch.Tensor, w: torch.Tensor, epi: str = "store",
              residual: torch.Tensor | None = None, out: torch.Tensor | None = None,
              variant: int = 7, splitk: int = 1, group_m: int = 8,
              ws: tuple[torch.Tensor, torch.Tensor] | None = None) -> torch.Tensor:
    """Hand-written CDNA4 GEMM (csrc/kernels/gemm_w4.hip): y = epi(x @ w.T).

    epi "store": y = x @ w.T; "residual": y = x @ w.T + residual (``out`` may be ``residual``
    itself: in-place add into the residual stream); "silu" / "gelu_tanh": w is the fused
    [gate; up] weight [2I, K] and y[:, n] = act(x . gate_n) * (x . up_n) has I columns (no
    act_glu pass).  Shapes: K % 64 == 0, N % 256 == 0 (I % 128 == 0 for the gated forms),
    (K / 64) % splitk == 0; rows of x are unrestricted.  ``group_m`` < 0 selects the
    K-slice-by-XCD tile order of the split-K form."""
    assert gemm_w4_variant(variant), variant
    M, K = x.shape
    glu = epi in ("silu", "gelu_tanh")
    N = w.shape[0] // 2 if glu else w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=x.dtype, device=x.device)
    assert out.shape == (M, N) and out.stride(1) == 1, (out.shape, M, N)  # written through ldc
    slab, cnt = ((ws or gemm_workspace(x.device)) if splitk > 1 else (None, None))
    check(hipk().gemm(out.data_ptr(), x.data_ptr(), w.data_ptr(), ptr(residual), M, N, K,
                      x.stride(0), w.stride(0), out.stride(0),
                      residual.stride(0) if residual is not None else 0, EPI[epi],
                      N if glu else 0, variant, splitk, group_m, ptr(slab),
                      slab.numel() * 4 if slab is not None else 0, ptr(cnt),
                      cnt.numel() if cnt is not None else 0, stream_ptr(x)), "gemm")
    return out


def mfma_gemm_grouped(x: torch.Tensor, w: torch.Tensor, grp: torch.Tensor, epi: str = "store",
                      out: torch.Tensor | None = None, group_m: int = 0,
                      ksplit: int = 1) -> torch.Tensor:
    """Grouped persistent gemm_w4 (csrc/kernels/gemm_w4.hip, V & 64): for every group g,
    out[r] = epi(x[r] @ w[g].T) over the rows r in [grp[g], grp[g + 1]).

    x [R, K] bf16 (rows in group order); w [G, N, K] ("silu" / "gelu_tanh": [G, 2I, K] with
    the gate rows first); grp int32 [G + 1] on the device, non-decreasing, grp[G] <= R -
    read by the kernel, never by the host (a routing kernel writes it: no sync, graph-safe).
    Rows outside [grp[0], grp[G]) of ``out`` are not written.  ``ksplit`` > 1 ("store"): K is
    cut into ksplit slices and out is [ksplit, R, N], slice s holding the bf16 partial product
    over its K range (the consumer sums them; the MoE combine does)."""
    R, K = x.shape
    G_, n2, k2 = w.shape
    glu = epi in ("silu", "gelu_tanh")
    N = n2 // 2 if glu else n2
    assert k2 == K and w.is_contiguous() and x.stride(1) == 1 and x.dtype == torch.bfloat16
    assert grp.dtype == torch.int32 and grp.numel() == G_ + 1 and grp.device == x.device
    shape = (ksplit, R, N) if ksplit > 1 else (R, N)
    if out is None:
        out = torch.empty(shape, dtype=x.dtype, device=x.device)
    assert out.shape == shape and out.stride(-1) == 1
    if ksplit > 1:
        assert out.is_contiguous()
    check(hipk().gemm_grouped(out.data_ptr(), x.data_ptr(), w.data_ptr(), grp.data_ptr(), G_,
                              R, N, K, x.stride(0), K, out.stride(-2), n2 * K, EPI[epi],
                              N if glu else 0, group_m or (4 if glu else 8), ksplit,
                              R * N if ksplit > 1 else 0, stream_ptr(x)),
          "gemm_grouped")
    return out


def tune(M: int, N: int, K: int, device, iters: int = 20, max_candidates: int = 12) -> dict:
    """Measure every hipBLASLt solution for y[M,N] = x[M,K] @ W[N,K]^T on random operands;
    returns {"algo", "us", "heuristic_us", "candidates"}."""
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
    """Merge ``entries`` ("M,N,K,ldx" -> tune() result) into the table of the running
    hipBLASLt version."""
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


# ------------------------------------------------------------ 4-wave GEMM dispatch
# Persistent gemm_w4 (variant 15: min(tiles, CUs) workgroups, the next tile's first K tiles
# staged during the current tile's last two steps) for every single-slice call.  Against the
# per-tile form in one process (profiles/r3r/probe.log): prefill qkv +0.5 %, o +2.0 %,
# gate_up+GLU +0.9 %, a 4400-row chunk's gate_up+GLU +2.3 %, decode gate_up+GLU at M = 1024
# +4.0 %.  DRTC_W4_PERSIST=0 restores the per-tile form (variant 7).
# Variant 31 (the default since round 4) adds the per-XCD K rotation: each XCD label starts its
# K loop at its own eighth of K, so the eight XCDs' epilogue store bursts do not coincide.
# Same box, interleaved (profiles/r4d/seam.log): decode gate_up + GLU at M = 1024 207.4 vs
# 231.1 us (v15), prefill shapes within +-1 % (K = 14336 1.2 % faster).  Fewer than 8 tiles
# run the plain persistent form.
W4_PERSIST = os.environ.get("DRTC_W4_PERSIST", "1") == "1"
# Variant 63 (the default since profiles/r4q) also spreads the next tile's fragment reads
# over half 1 (one per 4 MFMAs after a barrier at MFMA 63, instead of a burst of one per MFMA
# at 104-119): interleaved on one box, prefill gate_up+GLU 2557 vs 2597 us, o+residual 384.9
# vs 392.9, down 1256.6 vs 1280.5, qkv 534.7 vs 531.4, decode gate_up+GLU at M = 1024 199.2
# vs 214.1; headline 20,599 / 20,572 vs 20,338 tok/s.
W4_PERSIST_VARIANT = int(os.environ.get("DRTC_W4_VARIANT", "63"))


def _w4v(K: int) -> int:
    """Schedule variant of a single-slice gemm_w4 call with reduction length K."""
    return W4_PERSIST_VARIANT if W4_PERSIST and K >= 128 else 7


_w4_glu = os.environ.get("DRTC_W4_GLU", "1") != "0"
_w4_plain = os.environ.get("DRTC_W4_GEMM", "1") != "0"
# Prefill-sized passes (M >= W4_MIN_M rows) run the 4-wave hand GEMM (profiles/r3a_w4_gemm.md,
# Llama-3-8B at M = 16384, interleaved with the library in one process):
#   gate_up + SiLU-GLU epilogue  1.03-1.05x hipBLASLt + act_glu   -> hand (no act_glu pass)
#   qkv (store), o (+residual)   0.98-0.99x                        -> hand
#   down (K = 14336, +residual)  0.94-0.96x                        -> library (K > W4_MAX_K)
# gate_up + GLU also wins at the larger decode buckets: 1.04x at M = 768, 1.06x at 1024
# (library + act_glu), 0.97x at 512, 0.72x at 256 (profiles/r3b_w4_decode.md).
W4_GLU_MIN_M = int(os.environ.get("DRTC_W4_GLU_MIN_M", "640"))
W4_MIN_M = int(os.environ.get("DRTC_W4_MIN_M", "4096"))
W4_MAX_K = int(os.environ.get("DRTC_W4_MAX_K", "8192"))


def w4_group_m(M: int, N: int, K: int, glu: bool = False) -> int:
    """Row-tile group of the XCD-aware tile order.  An XCD's 32 workgroups take 32 consecutive
    tiles: with groups of 8 (4) rows that is an 8 x 4 (4 x 8) block of tiles, whose 12 operand
    panels stream through the XCD's L2 per K step, against 18 for the 2 x 16 block of groups
    of 2 (round 5, profiles/r5c: hipBLASLt's down kernel 23.4 M L2 misses, gemm_w4 at group 2
    34.1 M).  Interleaved on one box (profiles/r5d): down at K = 14336 1217 us at 8 vs 1247 at
    2; qkv 524 vs 532 at 4; o + residual 376 vs 378; the gated gate_up 2513 at 4 vs 2537 at 8."""
    return 4 if glu else 8


def w4_shape_ok(M: int, N: int, K: int) -> bool:
    """Shapes the prefill-sized hand GEMM takes (tensor strides / alignment aside)."""
    return (_w4_plain and _enabled and M >= W4_MIN_M and K <= W4_MAX_K and K % 64 == 0
            and N % 256 == 0)


def w4_ok(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None = None) -> bool:
    """Whether a prefill-sized projection y = x @ w.T (+ residual) takes gemm_w4."""
    if not _gpu_bf16(x, w):
        return False
    M, K = x.shape
    N = w.shape[0]
    if not (w4_shape_ok(M, N, K) and w.shape[1] == K and _aligned(x, w)):
        return False
    if residual is not None:
        return (residual.dim() == 2 and residual.shape == (M, N) and residual.stride(1) == 1
                and residual.stride(0) % 8 == 0 and residual.data_ptr() % 16 == 0
                and residual.dtype == torch.bfloat16)
    return True


def w4_glu_ok(x: torch.Tensor, w: torch.Tensor, act: str) -> bool:
    """Whether ``norm_glu`` takes the fused-GLU hand GEMM for x [M, K] @ [gate; up]^T."""
    if not (_w4_glu and act in ("silu", "gelu_tanh") and _gpu_bf16(x, w)):
        return False
    M, K = x.shape
    N2 = w.shape[0]
    return (M >= W4_GLU_MIN_M and K % 64 == 0 and w.shape[1] == K and N2 % 256 == 0
            and _aligned(x, w))


def glu_form(M: int, N2: int, K: int, ldx: int) -> int:
    """gemm_xd gated form the tuning table measured fastest for a decode batch M through the
    [gate; up] weight [N2, K] (bucket-above for an off-bucket M), 0 if none."""
    if not (_xd_enabled and _enabled) or M > DECODE_MAX_M:
        return 0
    found = _decode_entry(M, N2, K, ldx)
    form = found[1][4] if found is not None else 0
    return form if form and xd_supported(M, N2 // 2, K, form, glu=True) else 0


def fused_glu_ok(x: torch.Tensor, w: torch.Tensor, act: str) -> bool:
    """Whether ``norm_glu`` computes x [M, K] @ [gate; up]^T with the GLU inside a GEMM
    epilogue (gemm_w4 at prefill-sized / full decode batches, or a tuned gated gemm_xd form)."""
    if w4_glu_ok(x, w, act):
        return True
    return (act in ("silu", "gelu_tanh") and _gpu_bf16(x, w) and w.shape[1] == x.shape[1]
            and _aligned(x, w) and glu_form(x.shape[0], w.shape[0], x.shape[1], x.shape[1]) != 0)


def norm_glu(p, w: torch.Tensor, act: str = "silu") -> torch.Tensor:
    """h = act(norm(x) @ gate^T) * (norm(x) @ up^T) for an ``ops.PendingNorm`` p and the fused
    [gate; up] weight: on the 4-wave hand GEMM with the GLU in its epilogue when
    ``w4_glu_ok`` (one launch, no [M, 2I] intermediate); at the decode batches where the
    tuner measured it faster, gemm_xd with the GLU in its epilogue; else norm_linear +
    act_glu."""
    from .activation import act_glu

    x = p.x
    if (act in ("silu", "gelu_tanh") and isinstance(x, torch.Tensor) and _gpu_bf16(x, w)
            and w.shape[1] == x.shape[1] and _aligned(x, w)):
        form = glu_form(x.shape[0], w.shape[0], x.shape[1], x.shape[1])  # normed x: dense
        if form:  # a decode batch where the tuner measured the gated gemm_xd fastest
            xm = p.materialize()
            return xd_gemm(xm, w, act, form=form)
    if w4_glu_ok(p.x, w, act):
        x = p.materialize()
        M, K = x.shape
        return mfma_gemm(x, w, act, variant=_w4v(K),
                         group_m=w4_group_m(M, w.shape[0] // 2, K, glu=True))
    return act_glu(norm_linear(p, w), act)


# ------------------------------------------------------------------ XCD-partitioned decode GEMM
XD_EPI = {"store": 0, "residual": 1, "silu": 2, "gelu_tanh": 3}
# tile shapes built in gemm_xd.hip, (mt, nf) -> LDS ring depth (128 mt x 32 nf tiles); a form
# is mt * 100 + nf * 10 + splitk (K split over 1..8 slices), + 1000 for non-temporal weight
# loads (the tiles of XD_NT_TILES)
XD_TILES = {(1, 2): 4, (1, 4): 4, (1, 6): 3, (2, 4): 3, (2, 6): 2, (2, 8): 2}
XD_NT_TILES = {(1, 4), (1, 6), (2, 4), (2, 6), (2, 8)}
XD_MAX_SPLITK = 8
# the forms the tuner (scripts/tune_xd.py) measures
XD_FORMS = tuple(sorted([mt * 100 + nf * 10 + 1 for mt, nf in XD_TILES] +
                        [200 + nf * 10 + sk for nf in (4, 6, 8) for sk in (2, 3, 4)]))


def xd_form(form: int) -> tuple[int, int, int]:
    return form % 1000 // 100, form // 10 % 10, form % 10


def xd_nt(form: int) -> bool:
    """Form with non-temporal weight loads (MI355X_MICROARCH.md nt-weights)."""
    return form >= 1000


def xd_supported(M: int, N: int, K: int, form: int, glu: bool = False) -> bool:
    """Shapes gemm_xd.hip takes in ``form`` (mt * 100 + nf * 10 + splitk); N = output
    columns (gated: half the rows of the [gate; up] weight)."""
    mt, nf, sk = xd_form(form)
    if (mt, nf) not in XD_TILES or not 1 <= sk <= XD_MAX_SPLITK or (glu and nf % 2):
        return False
    if form // 1000 > 1 or (xd_nt(form) and (mt, nf) not in XD_NT_TILES):
        return False
    tno = 16 * nf if glu else 32 * nf
    if not (M >= 1 and N % tno == 0 and K % 64 == 0 and K // 64 // sk > XD_TILES[(mt, nf)]):
        return False
    # split-K: the partial slots and tile counters fit the device workspace
    tiles = -(-M // (128 * mt)) * (N // tno)
    return sk == 1 or (tiles * sk * (128 * mt) * (32 * nf) * 4 <= WS_SLAB_BYTES
                       and 2 * tiles + 2 <= WS_COUNTERS)  # + the fault word (last counter)


def xd_default_form(M: int, N: int, K: int, glu: bool = False) -> int:
    """Form of an untuned shape, by a per-CU operand-bytes model (profiles/r4i): a CU's
    time ~ (tile rows + columns) x (K / splitk) x 2 B per round of 256 work items, plus the
    split-K combine (its fp32 partials, weighted 5x: measured far costlier than their bytes)."""
    best, cost = 0, None
    for form in XD_FORMS:
        if not xd_supported(M, N, K, form, glu):
            continue
        mt, nf, sk = xd_form(form)
        tno = 16 * nf if glu else 32 * nf
        items = -(-M // (128 * mt)) * (N // tno) * sk
        rounds = -(-items // 256)
        c = rounds * ((128 * mt + 32 * nf) * (K // sk) * 2 + 100_000
                      + 5 * (sk - 1) * (128 * mt) * (32 * nf) * 4)
        if cost is None or c < cost:
            best, cost = form, c
    return best


def xd_gemm(x: torch.Tensor, w: torch.Tensor, epi: str = "store",
            residual: torch.Tensor | None = None, out: torch.Tensor | None = None,
            form: int = 0, ws: tuple[torch.Tensor, torch.Tensor] | None = None) -> torch.Tensor:
    """Decode-shaped hand GEMM, csrc/kernels/gemm_xd.hip: y = epi(x @ w.T) on 128 mt x 32 nf
    tiles, K split over 1..8 slices, with the tile order partitioned by XCD (each XCD streams
    its own weight column panels through its L2 for every row tile).  epi "store";
    "residual" (``out`` may be ``residual``); "silu" / "gelu_tanh": w is the fused [gate; up]
    weight [2I, K] and y[:, n] = act(x . gate_n) * (x . up_n).  ``form`` = mt * 100 +
    nf * 10 + splitk (+ 1000: non-temporal weight loads; 0: ``xd_default_form``)."""
    M, K = x.shape
    glu = epi in ("silu", "gelu_tanh")
    N = w.shape[0] // 2 if glu else w.shape[0]
    form = form or xd_default_form(M, N, K, glu)
    assert xd_supported(M, N, K, form, glu), (M, N, K, form, epi)
    assert x.dtype == w.dtype == torch.bfloat16 and x.stride(1) == 1 and w.is_contiguous()
    mt, nf, sk = xd_form(form)
    if out is None:
        out = residual if (epi == "residual" and residual is not None) else \
            torch.empty((M, N), dtype=x.dtype, device=x.device)
    # the kernel writes M x N through ldc: the output must hold exactly that
    assert out.shape == (M, N) and out.stride(1) == 1 and out.dtype == x.dtype, (out.shape, M, N)
    if epi == "residual":
        assert residual is not None and residual.shape == (M, N) and residual.stride(1) == 1
    slab, cnt = ((ws or gemm_workspace(x.device)) if sk > 1 else (None, None))
    check(hipk().gemm_xd(out.data_ptr(), x.data_ptr(), w.data_ptr(), ptr(residual), M, N, K,
                         x.stride(0), w.stride(0), out.stride(0),
                         residual.stride(0) if residual is not None else 0, XD_EPI[epi],
                         mt | (16 if xd_nt(form) else 0), nf,
                         sk, ptr(slab), slab.numel() * 4 if slab is not None else 0, ptr(cnt),
                         cnt.numel() if cnt is not None else 0, stream_ptr(x)), "gemm_xd")
    return out


# ------------------------------------------------------------------ medium-M decode GEMM
MIDM_EPI = {"store": 0, "residual": 1, "silu": 2, "gelu_tanh": 3}  # gemm_midm.hip accepts 0-3
MIDM_MAX_M = 256


def midm_splits(M: int, N: int, K: int, target_wgs: int | None = None) -> int:
    """K splits of the medium-M GEMM: the largest S <= 16 with K a multiple of 256 S (whole
    4-chunk register rings per split) and at most ~2 workgroups per CU (one above 128 rows,
    where the kernel runs one workgroup per CU)."""
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
    """Medium-M (17..256 rows) decode GEMM, csrc/kernels/gemm_midm.hip: y = x @ w^T with a
    store / residual (y = residual + x w^T, in place when out is residual) / SiLU- or
    GELU-gated [gate | up] epilogue.  W streams once from HBM into registers, x is shared
    through LDS, K is split over workgroups and the fp32 partials summed by a second small
    kernel."""
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


__all__ = ["linear", "route", "norm_linear", "glu_linear", "norm_glu", "fused_glu_ok",
           "linear_residual",
           "residual_fusable", "w4_glu_ok", "w4_ok", "w4_shape_ok", "w4_group_m", "mfma_gemm",
           "mfma_gemm_grouped",
           "gemm_workspace", "new_gemm_workspace", "private_workspace", "check_splitk_fault", "SplitKFault", "SplitKWatch",
           "set_splitk_spin_limit", "skinny_linear", "skinny_ok",
           "skinny_variant", "skinny_supports", "midm_gemm", "midm_supported", "midm_splits",
           "xd_gemm", "xd_supported", "xd_default_form", "tune", "save_entries", "load_table", "reset", "set_enabled", "table_path"]
