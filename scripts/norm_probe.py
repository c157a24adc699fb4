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


if __name__ == "__main__":
    main()
