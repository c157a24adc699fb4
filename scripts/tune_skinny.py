#!/usr/bin/env python3
"""Choose, per small-batch decode GEMM, between the library (tuned hipBLASLt
solution or torch's pick) and the hand-written skinny kernels of
csrc/kernels/gemv.hip (every variant that covers the shape).

Each candidate is timed inside one hipGraph over enough weight copies
(> 1 GiB) that every call streams W from HBM, not the 256 MB MALL - the
regime of a real decode step.  The result for every shape goes into the
tuning table as {"skinny": v (0 = library), "skinny_us", "lib_us"}, merged
with any hipBLASLt entry of the same key.

usage (GPU): python scripts/tune_skinny.py --model llama-3-8b [--tp 1]
             [--ms 1,2,4,8] [--out gpurun_out/skinny_tuned.json]
merge (CPU): python scripts/tune_gemms.py --merge gpurun_out/skinny_tuned.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tune_gemms import projection_shapes  # noqa: E402


def graph_us(fn, xs, ws, iters: int) -> float:
    n = len(ws)
    for i in range(2):
        fn(xs[i % n], ws[i % n])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(xs[i % n], ws[i % n])
    best = float("inf")
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / iters * 1e6)
    del g
    return best


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--ms", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--min-gain", type=float, default=0.02,
                    help="pick a skinny variant only if it beats the library by this fraction")
    ap.add_argument("--out", default="gpurun_out/skinny_tuned.json")
    a = ap.parse_args()
    from drtc_amd.ops import gemm
    from drtc_amd.ops._ext import hipk

    dev = torch.device("cuda", 0)
    ver = str(hipk().lt_version())
    table = gemm.load_table().get(ver, {})
    out = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            out = json.load(f)
    entries = out.setdefault(ver, {})
    t0 = time.time()
    for name, (N, K) in projection_shapes(a.model, a.tp).items():
        copies = max(2, min(16, (1 << 30) // (N * K * 2) + 1))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in (int(m) for m in a.ms.split(",")):
            key = f"{M},{N},{K},{K}"
            xs = [torch.randn(M, K, device=dev, dtype=torch.bfloat16) for _ in range(copies)]
            gemm.SKINNY_MAX_M = 0  # library path (tuned hipBLASLt entry if any)
            gemm.reset()
            lib = graph_us(gemm.linear, xs, ws, a.iters)
            gemm.SKINNY_MAX_M = 16
            ref = xs[0].float() @ ws[0].float().t()
            cand = {}
            for v in range(1, 10):
                if not gemm.skinny_supports(v, M, N, K, K):
                    continue
                err = (gemm.skinny_linear(xs[0], ws[0], v).float() - ref).abs().max().item()
                if err > 0.02 * ref.abs().max().item() + 0.02:
                    raise RuntimeError(f"skinny variant {v} wrong on {key}: max err {err}")
                cand[v] = graph_us(lambda x, w, v=v: gemm.skinny_linear(x, w, v), xs, ws, a.iters)
            best_v, best_us = min(cand.items(), key=lambda kv: kv[1], default=(0, float("inf")))
            pick = best_v if best_us < lib * (1.0 - a.min_gain) else 0
            ent = dict(table.get(key, {}))
            ent.update(skinny=pick, skinny_us=round(best_us, 2), lib_us=round(lib, 2),
                       model=a.model, tp=a.tp, gemm=name)
            entries[key] = ent
            print(json.dumps({"M": M, "N": N, "K": K, "gemm": name, "lib_us": round(lib, 2),
                              "variants": {v: round(u, 2) for v, u in cand.items()},
                              "pick": pick, "t": round(time.time() - t0, 1)}), flush=True)
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            with open(a.out, "w") as f:
                json.dump(out, f, indent=1, sort_keys=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
