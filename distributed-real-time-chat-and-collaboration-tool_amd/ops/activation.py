"""Gated activations over a fused [gate | up] projection.

HIP kernel: csrc/kernels/norm_act_rope.hip (act_glu_kernel).
"""
from __future__ import annotations

import math

import torch

from ._ext import check, hipk, on_gpu, stream_ptr

ACTS = {"silu": 0, "gelu_tanh": 1}


def act_glu_ref(gu: torch.Tensor, act: str = "silu") -> torch.Tensor:
    inter = gu.shape[-1] // 2
    g = gu[..., :inter].float()
    u = gu[..., inter:].float()
    if act == "silu":
        a = g * torch.sigmoid(g)
    else:
        a = 0.5 * g * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (g + 0.044715 * g.pow(3))))
    return (a * u).to(gu.dtype)


def act_glu(gu: torch.Tensor, act: str = "silu", out: torch.Tensor | None = None) -> torch.Tensor:
    """out[t, :I] = act(gu[t, :I]) * gu[t, I:2I]."""
    if not on_gpu(gu):
        r = act_glu_ref(gu, act)
        if out is not None:
            out.copy_(r)
            return out
        return r
    assert gu.dim() == 2 and gu.dtype == torch.bfloat16 and gu.stride(1) == 1
    T, two_i = gu.shape
    inter = two_i // 2
    assert inter % 8 == 0
    if out is None:
        out = torch.empty((T, inter), dtype=gu.dtype, device=gu.device)
    assert out.is_contiguous() and out.shape == (T, inter)
    check(hipk().act_glu(out.data_ptr(), gu.data_ptr(), T, inter, gu.stride(0),
                         ACTS[act], stream_ptr(gu)), "act_glu")
    return out
