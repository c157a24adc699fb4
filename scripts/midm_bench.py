#!/usr/bin/env python3
"""Medium-M decode GEMM (csrc/kernels/gemm_midm.hip) vs the engine's library path
(ops.linear, + act_glu for the gated MLP, + addmm for the residual forms), Llama-3-8B
projections at decode batches M = 24..256: correctness vs an fp32 reference, then
interleaved timing with W rotated over 6 copies (streams from HBM, not the 256 MB
Infinity Cache), sweeping the K-split count S."""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtc_amd import ops  # noqa: E402
from drtc_amd.ops import gemm as G  # noqa: E402

SHAPES = {"qkv": (6144, 4096, "store"), "o": (4096, 4096, "residual"),
          "gate_up": (28672, 4096, "silu"), "down": (4096, 14336, "residual")}


def ref(x, w, epi, res):
    y = x.float() @ w.float().t()
    if epi == "residual":
        return y + res.float()
    if epi == "silu":
        i = w.shape[0] // 2
        g, u = y[:, :i].to(torch.bfloat16).float(), y[:, i:].to(torch.bfloat16).float()
        return F.silu(g) * u
    return y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="24,32,48,64,96,128")
    ap.add_argument("--splits", default="auto,1,2,4,7,8,14,16")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    G.gemm_workspace(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for M in [int(m) for m in a.ms.split(",")]:
        for name, (N, K, epi) in SHAPES.items():
            if a.only and name not in a.only.split(","):
                continue
            ws = [(torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
                  for _ in range(6)]
            x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
            NO = N // 2 if epi == "silu" else N
            res = torch.randn(M, NO, device=dev, generator=g).to(torch.bfloat16) \
                if epi == "residual" else None
            r = ref(x, ws[0], epi, res)
            arms = {}
            if epi == "residual":
                rr = res.clone()
                arms["lib"] = lambda w, rr=rr: rr.addmm_(x, w.t())
            elif epi == "silu":
                arms["lib"] = lambda w: ops.act_glu(ops.linear(x, w), "silu")
            else:
                arms["lib"] = lambda w: ops.linear(x, w)
            errs = {}
            for sp in a.splits.split(","):
                S = G.midm_splits(M, N, K) if sp == "auto" else int(sp)
                if K % (64 * G.midm_depth(M) * S) or S * M * N * 4 > G.WS_SLAB_BYTES:
                    continue
                o = torch.empty(M, NO, device=dev, dtype=torch.bfloat16)
                rr = res.clone() if res is not None else None
                G.midm_gemm(x, ws[0], epi, residual=rr, out=o if rr is None else None,
                            splits=S)
                torch.cuda.synchronize()
                got = rr if rr is not None else o
                err = ((got.float() - r).abs().max() / r.abs().max().clamp(min=1e-6)).item()
                errs[f"S{S}"] = round(err, 5)
                if err > 2e-2:
                    print(json.dumps({"M": M, "gemm": name, "arm": f"S{S}", "err": err,
                                      "FAILED": True}), flush=True)
                    continue
                if epi == "residual":
                    arms[f"S{S}"] = lambda w, S=S, rr=rr: G.midm_gemm(x, w, epi, residual=rr,
                                                                      splits=S)
                else:
                    arms[f"S{S}"] = lambda w, S=S, o=o: G.midm_gemm(x, w, epi, out=o, splits=S)
            times = {k: [] for k in arms}
            for fn in arms.values():
                for w in ws:
                    fn(w)
            torch.cuda.synchronize()
            for _ in range(5):
                for k, fn in arms.items():
                    e0.record()
                    for i in range(24):
                        fn(ws[i % len(ws)])
                    e1.record()
                    e1.synchronize()
                    times[k].append(e0.elapsed_time(e1) * 1e3 / 24)
            lib = statistics.median(times["lib"])
            for k, ts in times.items():
                us = statistics.median(ts)
                print(json.dumps({"M": M, "gemm": name, "arm": k, "us": round(us, 1),
                                  "w_TBps": round(N * K * 2 / us / 1e6, 2),
                                  "vs_lib": round(lib / us, 2), "err": errs.get(k, "lib")}),
                      flush=True)


if __name__ == "__main__":
    main()
