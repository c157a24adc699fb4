#!/usr/bin/env python3
"""Decode GEMMs at small/medium batch (M = 16..512): time of the engine's
library path (ops.linear: tuned hipBLASLt where the table has a solution)
per Llama-3-8B projection, as weight-streaming bandwidth (W bytes / time) and
TFLOP/s - how far each shape sits from the HBM bound of one W pass."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtc_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    ws = {n: (torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
          for n, (N, K) in SHAPES.items()}
    # rotate over copies so W streams from HBM, not the 256 MB Infinity Cache
    copies = {n: [w] + [w.clone() for _ in range(5)] for n, w in ws.items()}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for M in (16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512):
        for n, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            cs = copies[n]
            for w in cs:
                ops.linear(x, w)
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0.record()
                for i in range(24):
                    ops.linear(x, cs[i % len(cs)])
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 24)
            us = statistics.median(ts)
            print(json.dumps({"M": M, "gemm": n, "us": round(us, 1),
                              "w_TBps": round(N * K * 2 / us / 1e6, 2),
                              "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
