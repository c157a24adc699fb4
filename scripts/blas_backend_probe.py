#!/usr/bin/env python3
"""rocBLAS (Tensile) vs hipBLASLt for the Llama-3-8B projection GEMMs at the
decode batch (M = 1024) and a prefill chunk (M = 16384): torch's two BLAS
backends on ROCm (preferred_blas_library "cublas" = rocBLAS, "cublaslt" =
hipBLASLt), plus the engine's tuned path (ops.linear).  Arms interleaved in
one process, median of rounds.

usage (GPU): python scripts/blas_backend_probe.py [--ms 1024,16384]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return 1000.0 * e0.elapsed_time(e1) / iters


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1024,16384")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from drtc_amd import ops

    dev = torch.device("cuda", 0)
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
              "down": (4096, 14336), "lm_head": (128256, 4096)}
    for M in (int(m) for m in a.ms.split(",")):
        for name, (N, K) in shapes.items():
            if name == "lm_head" and M > 1024:
                continue
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            iters = max(3, int(2e5 / (2 * M * N * K / 1.2e9)))  # ~200 ms of GEMM per arm-round
            iters = min(iters, 200)
            arms = {
                "rocblas": lambda: (torch.backends.cuda.preferred_blas_library("cublas"),
                                    F.linear(x, w)),
                "hipblaslt": lambda: (torch.backends.cuda.preferred_blas_library("cublaslt"),
                                      F.linear(x, w)),
                "engine": lambda: ops.linear(x, w),
            }
            res = {k: [] for k in arms}
            for k, f in arms.items():  # warm (solution load / code objects)
                f()
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for k, f in arms.items():
                    if k == "rocblas":
                        torch.backends.cuda.preferred_blas_library("cublas")
                        res[k].append(timed(lambda: F.linear(x, w), iters))
                    elif k == "hipblaslt":
                        torch.backends.cuda.preferred_blas_library("cublaslt")
                        res[k].append(timed(lambda: F.linear(x, w), iters))
                    else:
                        res[k].append(timed(f, iters))
            torch.backends.cuda.preferred_blas_library("cublaslt")
            fl = 2.0 * M * N * K
            row = {"M": M, "gemm": name}
            for k, v in res.items():
                us = statistics.median(v)
                row[k + "_us"] = round(us, 1)
                row[k + "_tflops"] = round(fl / us / 1e6, 1)
            print(json.dumps(row), flush=True)
            del x, w


if __name__ == "__main__":
    main()
