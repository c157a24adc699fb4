#!/usr/bin/env python3
"""A/B: residual add in the o/down GEMM epilogue (beta=1, in place into the
residual stream) + plain RMSNorm, versus GEMM + fused add-RMSNorm.

usage (GPU): python scripts/residual_gemm_bench.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from drtc_amd import ops  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000 * e0.elapsed_time(e1) / iters


d = torch.device("cuda", 0)
H = 4096
w_ln = torch.randn(H, device=d, dtype=torch.bfloat16)
for M in (16384, 1024):
    for name, K in (("o", 4096), ("down", 14336)):
        a = torch.randn(M, K, device=d, dtype=torch.bfloat16)
        W = torch.randn(H, K, device=d, dtype=torch.bfloat16) * 0.02
        res = torch.randn(M, H, device=d, dtype=torch.bfloat16)
        y = torch.empty(M, H, device=d, dtype=torch.bfloat16)
        out = torch.empty(M, H, device=d, dtype=torch.bfloat16)
        g_lin = timeit(lambda: torch.matmul(a, W.t(), out=y))
        g_tuned = timeit(lambda: ops.linear(a, W))
        n_res = timeit(lambda: ops.rmsnorm(y, w_ln, 1e-5, residual=res, out=out))
        g_add = timeit(lambda: res.addmm_(a, W.t()))
        n_plain = timeit(lambda: ops.rmsnorm(res, w_ln, 1e-5, out=out))
        print(json.dumps({"M": M, "gemm": name, "linear_us": round(g_lin, 1),
                          "tuned_linear_us": round(g_tuned, 1),
                          "addnorm_us": round(n_res, 1), "addmm_beta1_us": round(g_add, 1),
                          "norm_us": round(n_plain, 1),
                          "before_us": round(min(g_lin, g_tuned) + n_res, 1),
                          "after_us": round(g_add + n_plain, 1)}), flush=True)
