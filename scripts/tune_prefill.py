#!/usr/bin/env python3
"""Prefill-sized projection GEMMs: hipBLASLt's heuristic pick (what torch's
F.linear / addmm_ run) vs the best solution found by an exhaustive search
(ops.gemm.tune -> lt_tune: every supported solution, the fastest re-timed).

usage (GPU): python scripts/tune_prefill.py --model llama-3-8b --ms 16384
             [--out gpurun_out/prefill_tuned.json]
Writes tuning entries keyed like the decode table ("M,N,K,ldx") plus a
"prefill" flag; merge with scripts/tune_gemms.py --merge FILE.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from drtc_amd.models import get_config  # noqa: E402


def shapes(name: str) -> dict[str, tuple[int, int, bool]]:
    """(N, K, residual epilogue) of each prefill projection (TP=1)."""
    cfg = get_config(name)
    H, D = cfg.hidden_size, cfg.head_dim
    s = {"qkv": ((cfg.num_heads + 2 * cfg.num_kv_heads) * D, H, False),
         "o": (H, cfg.num_heads * D, True)}
    if not cfg.is_moe:
        s["gate_up"] = (2 * cfg.intermediate_size, H, False)
        s["down"] = (H, cfg.intermediate_size, True)
    return s


def time_fn(fn, iters: int) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / iters


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b", help="comma list of models")
    ap.add_argument("--ms", default="16384")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--min-gain", type=float, default=0.02)
    ap.add_argument("--out", default="gpurun_out/prefill_tuned.json")
    a = ap.parse_args()
    from drtc_amd.ops import gemm
    from drtc_amd.ops._ext import hipk

    dev = torch.device("cuda", 0)
    ver = str(hipk().lt_version())
    out: dict[str, dict] = {}
    todo = [(model, M, name, spec) for model in a.model.split(",")
            for M in (int(m) for m in a.ms.split(",")) for name, spec in shapes(model).items()]
    for model, M, name, (N, K, res) in todo:
        if f"{M},{N},{K},{K}" in out:  # same shape in another model (e.g. 70B o vs ...)
            continue
        if True:
            g = torch.Generator(device=dev).manual_seed(M + N + K)
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16, generator=g)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16, generator=g) * 0.02
            r = torch.randn(M, N, device=dev, dtype=torch.bfloat16, generator=g)
            t_lin = time_fn(lambda: torch.nn.functional.linear(x, w), a.iters)
            t_add = time_fn(lambda: r.addmm_(x, w.t()), a.iters) if res else None
            t = gemm.tune(M, N, K, dev, iters=a.iters, max_candidates=16)
            # the tuned solution through the engine's path (ops.gemm.linear /
            # linear_residual), both forms forced on
            gemm._activate()
            gemm._prefill[(N, K, K)] = [(M, t["algo"], True, True)]
            gemm._prefill_pick.clear()
            t_tuned = time_fn(lambda: gemm.linear(x, w), a.iters)
            t_tres = time_fn(lambda: gemm.linear_residual(x, w, r), a.iters) if res else None
            gemm._prefill.pop((N, K, K))
            gemm._prefill_pick.clear()
            fl = 2.0 * M * N * K
            row = {"gemm": name, "model": model, "tp": 1, "prefill": 1, "algo": t["algo"],
                   "us": round(t_tuned, 1), "heuristic_us": t["heuristic_us"],
                   "torch_linear_us": round(t_lin, 1), "candidates": t["candidates"],
                   "tflops": round(fl / t_tuned / 1e6, 1),
                   "torch_tflops": round(fl / t_lin / 1e6, 1)}
            # keep a form only where it beat torch's pick by >= min_gain
            row["beta0"] = int(t_tuned < (1 - a.min_gain) * t_lin)
            if res:
                row["torch_addmm_us"] = round(t_add, 1)
                row["residual_us"] = round(t_tres, 1)
                row["beta1"] = int(t_tres < (1 - a.min_gain) * t_add)
            print(json.dumps({f"{M},{N},{K},{K}": row}), flush=True)
            out[f"{M},{N},{K},{K}"] = row
            del x, w, r
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({ver: out}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
