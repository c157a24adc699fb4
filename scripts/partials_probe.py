#!/usr/bin/env python3
"""Decode o / down projection + the following residual-add RMSNorm at M = 1024 (Llama-3-8B):
the library GEMM + rmsnorm against gemm_w4 split-K partial planes + rmsnorm_partials, each
half timed on its own and as the pair, weights rotated over copies (HBM-streamed, as in a
decode step), arms interleaved in one process."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtc_amd import ops  # noqa: E402
from drtc_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=20, rounds=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / iters)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1024,4096,14336,4;1024,4096,4096,4;1024,4096,14336,2")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for spec in a.shapes.split(";"):
        M, N, K, sk = (int(v) for v in spec.split(","))
        nw = max(2, -(-512 * 2**20 // (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16) for _ in range(nw)]
        x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
        res = torch.randn(M, N, device=dev, generator=g).to(torch.bfloat16)
        lw = torch.ones(N, device=dev, dtype=torch.bfloat16)
        it = [0]

        def w():
            it[0] = (it[0] + 1) % nw
            return ws[it[0]]
        G.W4_PARTIAL = {(N, K): sk}
        y = ops.linear(x, ws[0])
        part = ops.linear_partials(x, ws[0])
        arms = {
            "lib_gemm": lambda: ops.linear(x, w()),
            "lib_norm": lambda: ops.rmsnorm(y, lw, 1e-5, residual=res),
            "lib_pair": lambda: ops.rmsnorm(ops.linear(x, w()), lw, 1e-5, residual=res),
            "part_gemm": lambda: ops.linear_partials(x, w()),
            "part_norm": lambda: ops.rmsnorm_partials(part, lw, 1e-5, residual=res),
            "part_pair": lambda: ops.rmsnorm_partials(ops.linear_partials(x, w()), lw, 1e-5,
                                                      residual=res),
        }
        out = {"M": M, "N": N, "K": K, "sk": sk}
        for k, f in arms.items():
            out[k] = round(timeit(f), 1)
        print(json.dumps(out), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
