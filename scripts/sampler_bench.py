#!/usr/bin/env python3
"""Fused sampler (csrc/kernels/sampling.hip) timing at the headline decode shape:
B rows x Llama-3 vocab (128256) bf16 logits, per sampling mode, interleaved
rounds of back-to-back launches; the read bound is one pass over the logits
(B * V * 2 bytes at ~8 TB/s)."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtc_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    B, V = a.batch, a.vocab
    g = torch.Generator(device=dev).manual_seed(0)
    # LM-head-like logits: N(0, 2) (random-init model rows are flatter; both timed)
    rows = {"randn_s2": (torch.randn(B, V, device=dev, generator=g) * 2).to(torch.bfloat16),
            "randn_s0.5": (torch.randn(B, V, device=dev, generator=g) * 0.5).to(torch.bfloat16)}
    step = torch.zeros(1, dtype=torch.int64, device=dev)
    ones = torch.ones(B, device=dev)
    modes = {
        "greedy": (torch.zeros(B, device=dev), None, None),
        "topk64_topp0.95": (ones, torch.full((B,), 64, dtype=torch.int32, device=dev),
                            torch.full((B,), 0.95, device=dev)),
        "topk0_topp0.95": (ones, torch.zeros(B, dtype=torch.int32, device=dev),
                           torch.full((B,), 0.95, device=dev)),
        "topk0_topp1": (ones, torch.zeros(B, dtype=torch.int32, device=dev), ones),
    }
    out = torch.empty(B, dtype=torch.int32, device=dev)
    bound_us = B * V * 2 / 8e12 * 1e6
    for dname, lg in rows.items():
        res = {m: [] for m in modes}
        for _ in range(a.rounds):
            for m, (t, k, p) in modes.items():
                ops.sample(lg, t, k, p, seed=1, step=step, out=out)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    ops.sample(lg, t, k, p, seed=1, step=step, out=out)
                e.record()
                e.synchronize()
                res[m].append(s.elapsed_time(e) * 1e3 / a.iters)
        for m, ts in res.items():
            print(json.dumps({"logits": dname, "mode": m, "B": B, "V": V,
                              "us_med": round(statistics.median(ts), 1),
                              "us_min": round(min(ts), 1),
                              "read_bound_us": round(bound_us, 1)}), flush=True)


if __name__ == "__main__":
    main()
