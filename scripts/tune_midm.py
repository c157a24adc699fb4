#!/usr/bin/env python3
"""Measure the medium-M decode GEMM (csrc/kernels/gemm_midm.hip) against the
engine's current path (ops.linear: tuned hipBLASLt / F.linear) for every decode
projection of a model at the decode buckets 17..256, and write a tuning entry
{"midm": S} (K splits) where the hand kernel wins by at least --min-gain.

W is rotated over copies (>= 512 MB in all) so it streams from HBM, as in a
decode step, not from the 256 MB Infinity Cache; arms are interleaved.

usage (GPU): python scripts/tune_midm.py --configs llama-3-8b:1,llama-3-70b:8
Merge on the CPU side: python scripts/tune_gemms.py --merge gpurun_out/midm_tuned.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tune_gemms import projection_shapes  # noqa: E402

BUCKETS = (24, 32, 48, 64, 96, 128, 160, 192, 224, 256)


def time_arm(fn, ws, rounds=5, iters=24):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for w in ws:
        fn(w)
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0.record()
        for i in range(iters):
            fn(ws[i % len(ws)])
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / iters)
    return statistics.median(ts)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="llama-3-8b:1,gemma-2b:1,llama-3-70b:1,llama-3-70b:8")
    ap.add_argument("--ms", default=",".join(map(str, BUCKETS)))
    ap.add_argument("--min-gain", type=float, default=0.05)
    ap.add_argument("--out", default="gpurun_out/midm_tuned.json")
    a = ap.parse_args()
    from drtc_amd.ops import gemm as G
    from drtc_amd.ops._ext import hipk

    dev = torch.device("cuda", 0)
    G._midm_enabled = False  # the baseline is the path the engine takes without midm
    G.reset()
    G.gemm_workspace(dev)
    ver = str(hipk().lt_version())
    out = {ver: {}}
    g = torch.Generator(device=dev).manual_seed(0)
    for spec in a.configs.split(","):
        model, tp = spec.split(":")
        for name, (N, K) in projection_shapes(model, int(tp)).items():
            wbytes = N * K * 2
            ncopy = max(2, min(6, -(-512 * 2**20 // wbytes)))
            ws = [(torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
                  for _ in range(ncopy)]
            for M in (int(m) for m in a.ms.split(",")):
                if not G.midm_supported(M, N, K):
                    continue
                x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
                lib = time_arm(lambda w: G.linear(x, w), ws)
                ref = x.float() @ ws[0].float().t()
                best = None
                ring = 64 * G.midm_depth(M)
                for S in range(1, 17):
                    if K % (ring * S) or S * M * N * 4 > G.WS_SLAB_BYTES or (N // 128) * S > 1024:
                        continue
                    y = G.midm_gemm(x, ws[0], splits=S)
                    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                    if err > 2e-2:
                        print(json.dumps({"model": model, "tp": tp, "gemm": name, "M": M,
                                          "S": S, "err": err, "FAILED": True}), flush=True)
                        continue
                    us = time_arm(lambda w, S=S: G.midm_gemm(x, w, splits=S), ws)
                    if best is None or us < best[1]:
                        best = (S, us)
                rec = {"model": model, "tp": int(tp), "gemm": name, "M": M, "N": N, "K": K,
                       "lib_us": round(lib, 1)}
                if best is not None:
                    rec.update(midm_S=best[0], midm_us=round(best[1], 1),
                               gain=round(lib / best[1] - 1, 3))
                    if best[1] < lib * (1 - a.min_gain):
                        out[ver][f"{M},{N},{K},{K}"] = {
                            "midm": best[0], "midm_us": round(best[1], 1),
                            "midm_base_us": round(lib, 1), "gemm": name, "model": model,
                            "tp": int(tp)}
                print(json.dumps(rec), flush=True)
            del ws
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {len(out[ver])} midm entries to {a.out}", flush=True)


if __name__ == "__main__":
    main()
