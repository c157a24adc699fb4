#!/usr/bin/env python3
"""Prefill MLP in row sub-chunks: does keeping the gate_up output cache-resident pay?

The prefill MLP of a 16k-token chunk writes a [16384, 2 x 14336] bf16 gate_up output (940 MB)
to HBM, act_glu reads it back (8.1 ms per chunk, 5 % of prefill: profiles/r2o), and the down
projection reads the 470 MB activation.  Processed in row sub-chunks of c tokens, the
gate_up output of a sub-chunk (c x 57 KB) can stay in the 256 MB Infinity Cache for the
act_glu that follows; the price is smaller-M GEMMs.

Arms (the engine's own ops, eager, timed back to back and interleaved over rounds):
  full   gu = linear(x); a = act_glu(gu); linear_residual(a, down, res)   on all rows
  sub<c> the same per row block of c tokens
Prints one JSON line per arm; the numerics of every arm equal the full arm bitwise.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import drtc_amd  # noqa: E402,F401
from drtc_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16384)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--chunks", default="8192,4096,2048")
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    T, H, I = a.tokens, a.hidden, a.inter
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    wgu = torch.randn(2 * I, H, device=dev, dtype=torch.bfloat16) * 0.02
    wd = torch.randn(H, I, device=dev, dtype=torch.bfloat16) * 0.02
    res0 = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    res = res0.clone()

    def mlp(rows: slice):
        gu = ops.linear(x[rows], wgu)
        act = ops.act_glu(gu, "silu")
        ops.linear_residual(act, wd, res[rows])

    def arm(c: int):
        def run():
            for s in range(0, T, c):
                mlp(slice(s, min(T, s + c)))
        return run

    arms = {"full": arm(T)}
    for c in [int(v) for v in a.chunks.split(",")]:
        arms[f"sub{c}"] = arm(c)
    # numerics: every arm from the same residual gives the same bits as the full arm
    outs = {}
    for name, fn in arms.items():
        res.copy_(res0)
        fn()
        torch.cuda.synchronize()
        outs[name] = res.clone()
    same = {n: bool(torch.equal(o, outs["full"])) for n, o in outs.items()}
    max_diff = {n: float((o.float() - outs["full"].float()).abs().max()) for n, o in outs.items()}
    del outs
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {n: [] for n in arms}
    for _ in range(a.rounds):
        for n, fn in arms.items():
            fn()
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            e.synchronize()
            times[n].append(s.elapsed_time(e) / a.iters)
    full = statistics.median(times["full"])
    for n in arms:
        med = statistics.median(times[n])
        print(json.dumps({"arm": n, "tokens": T, "ms": round(med, 3), "min_ms": round(min(times[n]), 3),
                          "vs_full": round(full / med, 3), "bitwise_equal": same[n],
                          "max_abs_diff": max_diff[n]}), flush=True)


if __name__ == "__main__":
    main()
