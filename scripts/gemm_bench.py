#!/usr/bin/env python3
"""Projection-GEMM study for Llama-3-8B shapes on MI355X.

Times y = x @ W^T (bf16) for the decode (M = batch) and prefill (M = tokens)
shapes of the four per-layer projections + LM head, with
  * the default library choice (hipBLASLt),
  * rocBLAS (torch.backends.cuda.preferred_blas_library),
  * PyTorch TunableOp (exhaustive hipBLASLt/rocBLAS solution search; results
    saved to a CSV that the engine can load with PYTORCH_TUNABLEOP_FILENAME).
Prints achieved TB/s (weight bytes / time) and TFLOP/s per shape.
"""
import argparse
import json
import os
import time

import torch
import torch.nn.functional as F

SHAPES = {  # name: (N, K)
    "qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
    "lm_head": (128256, 4096),
}
SHAPES_70B = {  # Llama-3-70B (TP=1): hidden 8192, inter 28672, GQA 64/8
    "qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192), "down": (8192, 28672),
    "lm_head": (128256, 8192),
}


def bench(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="64,128,256,512,1024,16384")
    ap.add_argument("--tunable-file", default="gpurun_out/tunableop_results.csv")
    ap.add_argument("--modes", default="default,rocblas,tunable")
    ap.add_argument("--model", default="8b", choices=["8b", "70b"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = []
    shapes = SHAPES_70B if a.model == "70b" else SHAPES
    W = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for k, (n, kk) in shapes.items()}
    H, inter = shapes["o"][0], shapes["down"][1]
    wts = {}
    for mode in a.modes.split(","):
        if mode == "rocblas":
            torch.backends.cuda.preferred_blas_library("cublas")
        else:
            torch.backends.cuda.preferred_blas_library("cublaslt")
        if mode in ("tunable", "nn_tunable"):
            torch.cuda.tunable.enable(True)
            torch.cuda.tunable.tuning_enable(True)
            torch.cuda.tunable.set_max_tuning_duration(200)
            torch.cuda.tunable.set_filename(a.tunable_file)
        for M in [int(x) for x in a.ms.split(",")]:
            x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
            xd = torch.randn(M, inter, device=dev, dtype=torch.bfloat16)
            for name, w in W.items():
                if name == "lm_head" and M > 1024:
                    continue
                inp = xd if name == "down" else x
                if mode == "tunable":
                    F.linear(inp, w)  # tune outside the graph
                    torch.cuda.synchronize()
                if mode == "transposed":  # out^T = W @ x^T (library sees M'=N, N'=M)
                    t = bench(lambda: torch.mm(w, inp.t()).t().contiguous())
                elif mode in ("nn", "nn_tunable"):  # weights stored [K, N]: x @ Wt
                    wt = wts.setdefault(name, w.t().contiguous())
                    if mode == "nn_tunable":
                        torch.mm(inp, wt)
                        torch.cuda.synchronize()
                    t = bench(lambda: torch.mm(inp, wt))
                else:
                    t = bench(lambda: F.linear(inp, w))
                n, k = w.shape
                r = {"mode": mode, "M": M, "gemm": name, "us": round(t * 1e6, 1),
                     "TBps_weights": round(n * k * 2 / t / 1e12, 2),
                     "TFLOPs": round(2 * M * n * k / t / 1e12, 1)}
                res.append(r)
                print(json.dumps(r), flush=True)
        if mode == "tunable":  # results are flushed to set_filename()'s file at exit
            torch.cuda.tunable.enable(False)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/gemm_bench.json", "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
