#!/usr/bin/env python3
"""gemm_xd with padded operand row strides: does the per-CU operand rate depend on how the
rows of a K tile map onto L2 channels?  (lda / ldb = K + pad elements; weights rotated.)

  python scripts/xd_pad_probe.py --shape 1024,4096,4096 --nf 4 --pads 0,64,128
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import drtc_amd  # noqa: E402,F401
from drtc_amd.ops._ext import hipk, stream_ptr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="1024,4096,4096")
    ap.add_argument("--nf", type=int, default=4)
    ap.add_argument("--pads", default="0,64,128,256")
    ap.add_argument("--rotate", type=int, default=10)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    M, N, K = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda")
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    arms = {}
    for pad in (int(p) for p in a.pads.split(",")):
        xa = torch.randn(M, K + pad, device=dev, dtype=torch.bfloat16)
        ws = [torch.randn(N, K + pad, device=dev, dtype=torch.bfloat16) * 0.02
              for _ in range(a.rotate)]
        arms[pad] = (xa, ws)
    k = hipk()
    st = stream_ptr(out)

    def run(pad, i):
        xa, ws = arms[pad]
        rc = k.gemm_xd(out.data_ptr(), xa.data_ptr(), ws[i % len(ws)].data_ptr(), 0, M, N, K,
                       K + pad, K + pad, N, 0, 0, 1, a.nf, 1, 0, 0, 0, 0, st)
        assert rc == 0, rc
    for pad, (xa, ws) in arms.items():  # correctness
        run(pad, 0)
        ref = xa[:, :K].float() @ ws[0][:, :K].float().t()
        err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
        assert err < 2e-2, (pad, err)
    times = {p: [] for p in arms}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for p in arms:
            s.record()
            for i in range(a.iters):
                run(p, i)
            e.record()
            e.synchronize()
            times[p].append(s.elapsed_time(e) * 1e3 / a.iters)
    for p, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"shape": [M, N, K], "nf": a.nf, "pad": p, "us_med": round(med, 1),
                          "us_min": round(min(ts), 1),
                          "TFLOPs": round(2.0 * M * N * K / med / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
