"""RMSNorm (+ fused residual add).  HIP kernel: csrc/kernels/norm_act_rope.hip."""
from __future__ import annotations

import torch

from ._ext import check, hipk, on_gpu, ptr, stream_ptr


def rmsnorm_ref(x: torch.Tensor, w: torch.Tensor, eps: float, gemma: bool = False,
                residual: torch.Tensor | None = None) -> torch.Tensor:
    """fp32 PyTorch reference.  With ``residual`` the sum x + residual is
    rounded to the activation dtype, written back into ``residual`` and
    normalised (the HF pre-norm residual stream semantics)."""
    if residual is not None:
        s = (x.float() + residual.float()).to(residual.dtype)
        residual.copy_(s)
        x = s
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    ww = w.float() + (1.0 if gemma else 0.0)
    return (xf * r * ww).to(x.dtype)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, gemma: bool = False,
            residual: torch.Tensor | None = None,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """out = norm(x [+ residual]) * w (Gemma: * (1 + w)); x: [rows, H]."""
    if not on_gpu(x):
        r = rmsnorm_ref(x, w, eps, gemma, residual)
        if out is not None:
            out.copy_(r)
            return out
        return r
    assert x.dim() == 2 and x.dtype == torch.bfloat16 and x.stride(1) == 1
    rows, H = x.shape
    assert w.shape == (H,) and w.dtype == torch.bfloat16 and w.is_contiguous()
    assert H % 8 == 0 and H <= 8192 * 2
    if out is None:
        out = torch.empty((rows, H), dtype=x.dtype, device=x.device)
    assert out.stride(1) == 1 and out.shape == (rows, H)
    res_stride = 0
    if residual is not None:
        assert residual.shape == (rows, H) and residual.stride(1) == 1
        res_stride = residual.stride(0)
    check(hipk().rmsnorm(out.data_ptr(), ptr(residual), x.data_ptr(), w.data_ptr(),
                         rows, H, float(eps), x.stride(0), out.stride(0), res_stride,
                         bool(gemma), stream_ptr(x)), "rmsnorm")
    return out


class PendingNorm:
    """A pre-norm sublayer input whose RMSNorm has not run yet: norm(x [+
    residual]) * w.  The consumer either fuses the norm into its projection
    (``ops.norm_linear``: small decode batches, csrc/kernels/gemv.hip) or
    calls ``materialize()`` for the plain normalised tensor.  Either way
    ``stream()`` afterwards is the post-add residual stream h = x + residual
    (x itself when there is no residual), which the next PendingNorm adds to.
    """

    __slots__ = ("x", "residual", "w", "eps", "gemma", "_h", "_out", "pc")

    def __init__(self, x: torch.Tensor, residual: torch.Tensor | None, w: torch.Tensor,
                 eps: float, gemma: bool, pc=None):
        """``pc``: a ParallelContext when ``x`` is still a tensor-parallel PARTIAL
        sum: materialize() then runs the all-reduce fused with the residual add
        and the norm (ParallelContext.reduce_norm)."""
        self.x, self.residual, self.w, self.eps, self.gemma = x, residual, w, eps, gemma
        self.pc = pc
        self._h: torch.Tensor | None = None
        self._out: torch.Tensor | None = None

    def applied(self, h: torch.Tensor) -> None:
        """Record that a fused consumer computed h = x (+ residual)."""
        self._h, self.x, self.residual = h, h, None

    def materialize(self) -> torch.Tensor:
        if self._out is None:
            res = self.residual
            if self.pc is not None:
                self._out = self.pc.reduce_norm(self.x, res, self.w, self.eps, self.gemma)
                self.pc = None
            else:
                self._out = rmsnorm(self.x, self.w, self.eps, self.gemma, residual=res)
            self._h = res if res is not None else self.x  # rmsnorm updated res in place
            self.x, self.residual = self._h, None
        return self._out

    def stream(self) -> torch.Tensor:
        if self._h is None:
            self.materialize()
        return self._h

    def select_rows(self, idx: torch.Tensor) -> None:
        """Keep only the rows ``idx`` (int64) of every tensor this input holds:
        the last layer of a prefill pass continues with each sequence's last
        token only once its attention has read (and cached) every position."""
        if self._out is not None:
            self._out = self._out.index_select(0, idx)
        if self._h is not None:  # x is _h (materialize / applied alias them)
            self._h = self.x = self._h.index_select(0, idx)
            return
        self.x = self.x.index_select(0, idx)
        if self.residual is not None:
            self.residual = self.residual.index_select(0, idx)
