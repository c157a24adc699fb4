#!/usr/bin/env python3
"""Measure the XCD-partitioned decode GEMM (csrc/kernels/gemm_xd.hip) against the engine's
path without it (ops.linear: tuned hipBLASLt / midm / F.linear) for every decode projection
of a model at the larger decode buckets, and write a tuning entry {"xd": form} where the hand
kernel wins by at least --min-gain.

W is rotated over copies (>= 512 MB in all) so it streams from HBM, as in a decode step;
arms are interleaved (time_arm of tune_midm.py).

usage (GPU): python scripts/tune_xd.py --configs llama-3-8b:1,llama-3-70b:1
Merge on the CPU side: python scripts/tune_gemms.py --merge gpurun_out/xd_tuned.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tune_gemms import projection_shapes  # noqa: E402
from tune_midm import time_arm  # noqa: E402

BUCKETS = (128, 160, 192, 224, 256, 320, 384, 448, 512, 640, 768, 896, 1024)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="llama-3-8b:1,gemma-2b:1,llama-3-70b:1,llama-3-70b:8")
    ap.add_argument("--ms", default=",".join(map(str, BUCKETS)))
    ap.add_argument("--min-gain", type=float, default=0.03)
    ap.add_argument("--out", default="gpurun_out/xd_tuned.json")
    a = ap.parse_args()
    from drtc_amd.ops import gemm as G
    from drtc_amd.ops._ext import hipk

    dev = torch.device("cuda", 0)
    G._xd_enabled = False  # the baseline is the path the engine takes without gemm_xd
    G.reset()
    G.gemm_workspace(dev)
    ver = str(hipk().lt_version())
    out = {ver: {}}
    g = torch.Generator(device=dev).manual_seed(0)
    for spec in a.configs.split(","):
        model, tp = spec.split(":")
        for name, (N, K) in projection_shapes(model, int(tp)).items():
            if name == "lm_head":  # 256 x 256 library tiles win at vocabulary widths
                continue
            wbytes = N * K * 2
            ncopy = max(2, min(10, -(-512 * 2**20 // wbytes)))
            ws = [(torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
                  for _ in range(ncopy)]
            for M in (int(m) for m in a.ms.split(",")):
                forms = [f for f in G.XD_FORMS if G.xd_supported(M, N, K, f)]
                if not forms:
                    continue
                x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
                base = time_arm(lambda w: G.linear(x, w), ws)
                kind = G.route(M, N, K, K)[0]
                ref = x.float() @ ws[0].float().t()
                best = None
                for nf in forms:
                    y = G.xd_gemm(x, ws[0], form=nf)
                    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                    if err > 2e-2:
                        print(json.dumps({"model": model, "tp": tp, "gemm": name, "M": M,
                                          "form": nf, "err": err, "FAILED": True}), flush=True)
                        continue
                    us = time_arm(lambda w, nf=nf: G.xd_gemm(x, w, form=nf), ws)
                    if best is None or us < best[1]:
                        best = (nf, us)
                rec = {"model": model, "tp": int(tp), "gemm": name, "M": M, "N": N, "K": K,
                       "base": kind, "base_us": round(base, 1)}
                if best is not None:
                    rec.update(xd_form=best[0], xd_us=round(best[1], 1),
                               gain=round(base / best[1] - 1, 3))
                    if best[1] < base * (1 - a.min_gain):
                        out[ver][f"{M},{N},{K},{K}"] = {
                            "xd": best[0], "xd_us": round(best[1], 1),
                            "xd_base_us": round(base, 1), "gemm": name, "model": model,
                            "tp": int(tp)}
                print(json.dumps(rec), flush=True)
                del ref
            del ws
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {len(out[ver])} xd entries to {a.out}", flush=True)


if __name__ == "__main__":
    main()
