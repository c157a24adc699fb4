#!/usr/bin/env python3
"""Small-batch decode GEMM study: hand-written skinny kernel (gemv.hip) vs the
tuned hipBLASLt path vs torch F.linear, for the projection shapes of a model
at M = 1..8.  Weights are cycled over enough copies (> 1 GiB) that every call
streams from HBM rather than the 256 MB MALL, as in a real decode step.
Prints one JSON line per (shape, M) with us/call and achieved TB/s."""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtc_amd.ops import gemm  # noqa: E402

SHAPES = {
    "8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
           "down": (4096, 14336), "lm_head": (128256, 4096)},
    "70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192),
            "down": (8192, 28672)},
}


def timed(fn, xs, ws, iters):
    n = len(ws)
    for i in range(3):
        fn(xs[i % n], ws[i % n])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(iters):
            fn(xs[i % n], ws[i % n])
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="8b", choices=sorted(SHAPES))
    ap.add_argument("--ms", default="1,2,4,8,16")
    ap.add_argument("--variants", default="1,2,3,4,5")
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for name, (N, K) in SHAPES[a.model].items():
        copies = max(2, min(16, (1 << 30) // (N * K * 2) + 1))
        ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
        for M in (int(v) for v in a.ms.split(",")):
            xs = [torch.randn(M, K, device=dev, dtype=torch.bfloat16) for _ in range(copies)]
            ref = xs[0].float() @ ws[0].float().t()
            err = (gemm.skinny_linear(xs[0], ws[0]).float() - ref).abs().max().item()
            row = {"shape": name, "M": M, "N": N, "K": K, "copies": copies,
                   "skinny_max_err": round(err, 4)}
            gemm.SKINNY_MAX_M = 0
            row["lt_us"] = timed(lambda x, w: gemm.linear(x, w), xs, ws, a.iters)
            row["torch_us"] = timed(lambda x, w: F.linear(x, w), xs, ws, a.iters)
            gemm.SKINNY_MAX_M = 16
            keys = ["lt", "torch"]
            for v in (int(s) for s in a.variants.split(",")):
                if (v == 1 and (M > 8 or K % 512)) or (v >= 2 and (N % 32 or K % 128)):
                    continue
                row[f"v{v}_us"] = timed(lambda x, w, v=v: gemm.skinny_linear(x, w, v), xs, ws,
                                        a.iters)
                keys.append(f"v{v}")
            for k in keys:
                row[k + "_us"] = round(row[k + "_us"], 2)
                row[k + "_tbs"] = round(N * K * 2 / row[k + "_us"] / 1e6, 2)
            print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
