#!/usr/bin/env python3
"""Decode-sized RMSNorm timing (us per call, CUDA events over many calls): (rows, H) with and
without the fused residual add."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import drtc_amd  # noqa: E402,F401
from drtc_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    for rows, H in ((1024, 4096), (256, 8192), (1024, 2048), (16384, 4096)):
        x = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
        w = torch.randn(H, device=dev, dtype=torch.bfloat16)
        res = torch.randn(rows, H, device=dev, dtype=torch.bfloat16)
        out = torch.empty_like(x)
        for resid in (False, True):
            f = (lambda: ops.rmsnorm(x, w, 1e-5, residual=res, out=out)) if resid else \
                (lambda: ops.rmsnorm(x, w, 1e-5, out=out))
            for _ in range(20):
                f()
            n = 400 if rows <= 1024 else 50
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = None
            for _ in range(5):
                s.record()
                for _ in range(n):
                    f()
                e.record()
                e.synchronize()
                us = s.elapsed_time(e) * 1e3 / n
                best = us if best is None else min(best, us)
            print(json.dumps({"rows": rows, "H": H, "residual": resid, "us": round(best, 2),
                              "pf": os.environ.get("DRTC_NORM_NOPF") is None}), flush=True)


def graph_ab():
    """Graph-replayed norms (as inside the decode hipGraph): us per norm over 64 back-to-back
    launches on alternating buffers.  (Round 5 also timed a non-temporal store form here:
    3.3 vs 3.9 us at 1024 x 4096, but it slowed the decode pass by 1.5 % - the next GEMM reads
    the normed rows from L2 - profiles/r5ax, r5ay; removed.)"""
    dev = torch.device("cuda")
    for rows, H in ((1024, 4096), (256, 8192), (1024, 2048)):
        xs = [torch.randn(rows, H, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        rs = [torch.randn(rows, H, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        outs = [torch.empty(rows, H, device=dev, dtype=torch.bfloat16) for _ in range(2)]
        w = torch.randn(H, device=dev, dtype=torch.bfloat16)
        for resid in (False, True):
            for i in range(2):  # warm
                ops.rmsnorm(xs[i], w, 1e-5, residual=rs[i] if resid else None, out=outs[i])
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(64):
                    ops.rmsnorm(xs[i & 1], w, 1e-5, residual=rs[i & 1] if resid else None,
                                out=outs[i & 1])
            best = None
            for _ in range(5):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(10):
                    g.replay()
                e.record()
                e.synchronize()
                us = s.elapsed_time(e) * 1e3 / 640
                best = us if best is None else min(best, us)
            print(json.dumps({"rows": rows, "H": H, "residual": resid, "graph": True,
                              "us": round(best, 2)}), flush=True)


if __name__ == "__main__":
    if "--graph" in sys.argv:
        graph_ab()
    else:
        main()
