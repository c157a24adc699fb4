#!/usr/bin/env python3
"""Measure the XCD-partitioned decode GEMM (csrc/kernels/gemm_xd.hip) against the engine's
path without it (ops.linear: tuned hipBLASLt / midm / F.linear) for every decode projection
of a model at the larger decode buckets (forms with non-temporal weight loads, form + 1000,
where the batch fits one row tile), and write a tuning entry {"xd": form} where the hand
kernel wins by at least --min-gain; for gate_up below the fused-GLU gemm_w4 batches also the
GLU epilogue form against the route + act_glu ({"xd_glu": form}).

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


def measure(G, x, ws, N, K, epi, base_fn, name, model, tp, M, nt_any=False):
    """Time the engine's current route (base_fn) and every gemm_xd form for one shape
    (epi "store" or a GLU: N = output columns); print and return the record."""
    glu = epi != "store"
    forms = [f for f in G.XD_FORMS if G.xd_supported(M, N, K, f, glu)]
    # non-temporal weight loads where the batch fits one row tile (nobody re-reads a weight)
    # (--nt-any: at every M, for the tiles built with them)
    forms += [f + 1000 for f in forms
              if G.xd_nt_ok(M, f) or (nt_any and G.xd_supported(M, N, K, f + 1000, glu))]
    if not forms:
        return None
    base = time_arm(base_fn, ws)
    y = x.float() @ ws[0].float().t()
    if glu:
        y = torch.nn.functional.silu(y[:, :N]) * y[:, N:]
    best = None
    for f in forms:
        got = G.xd_gemm(x, ws[0], epi, form=f)
        err = ((got.float() - y).abs().max() / y.abs().max()).item()
        if err > 2e-2:
            print(json.dumps({"model": model, "tp": tp, "gemm": name, "epi": epi, "M": M,
                              "form": f, "err": err, "FAILED": True}), flush=True)
            continue
        us = time_arm(lambda w, f=f: G.xd_gemm(x, w, epi, form=f), ws)
        if best is None or us < best[1]:
            best = (f, us)
    del y
    rec = {"model": model, "tp": int(tp), "gemm": name, "epi": epi, "M": M, "N": N, "K": K,
           "base": G.route(M, N * (2 if glu else 1), K, K)[0], "base_us": round(base, 1)}
    if best is not None:
        rec.update(xd_form=best[0], xd_us=round(best[1], 1), gain=round(base / best[1] - 1, 3))
    print(json.dumps(rec), flush=True)
    return rec if best is not None else None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="llama-3-8b:1,gemma-2b:1,llama-3-70b:1,llama-3-70b:8")
    ap.add_argument("--ms", default=",".join(map(str, BUCKETS)))
    ap.add_argument("--min-gain", type=float, default=0.03)
    ap.add_argument("--out", default="gpurun_out/xd_tuned.json")
    ap.add_argument("--gemms", default="qkv,o,gate_up,down",
                    help="projections to tune (lm_head too: profiles/r5ak)")
    ap.add_argument("--nt-any", action="store_true",
                    help="non-temporal forms among the candidates at every M, not only where "
                         "the batch fits one row tile")
    a = ap.parse_args()
    from drtc_amd import ops
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
            if name not in a.gemms.split(","):
                continue
            wbytes = N * K * 2
            ncopy = max(2, min(10, -(-512 * 2**20 // wbytes)))
            ws = [(torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
                  for _ in range(ncopy)]
            for M in (int(m) for m in a.ms.split(",")):
                x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
                key = f"{M},{N},{K},{K}"
                ent = {}
                # plain projection (ops.linear) against the engine's route without gemm_xd
                rec = measure(G, x, ws, N, K, "store", lambda w: G.linear(x, w), name, model, tp, M,
                              a.nt_any)
                if rec and rec["xd_us"] < rec["base_us"] * (1 - a.min_gain):
                    ent.update(xd=rec["xd_form"], xd_us=rec["xd_us"], xd_base_us=rec["base_us"])
                    ent.update(nt_tuned=True)  # nt forms were candidates: the router keeps the pick
                # gate_up with the GLU in the epilogue against norm_glu's route without gemm_xd
                # (the fused-GLU gemm_w4 from W4_GLU_MIN_M rows, else the route + act_glu)
                if name == "gate_up":
                    act = "silu"
                    if M >= G.W4_GLU_MIN_M:
                        def glu_base(w, act=act):
                            return G.mfma_gemm(x, w, act, variant=G._w4v(K),
                                               group_m=G.w4_group_m(M, N // 2, K, glu=True))
                    else:
                        def glu_base(w, act=act):
                            return ops.act_glu(G.linear(x, w), act)
                    rec = measure(G, x, ws, N // 2, K, act, glu_base, name, model, tp, M, a.nt_any)
                    if rec and rec["xd_us"] < rec["base_us"] * (1 - a.min_gain):
                        ent.update(nt_tuned=True)
                        ent.update(xd_glu=rec["xd_form"], xd_glu_us=rec["xd_us"],
                                   xd_glu_base_us=rec["base_us"])
                if ent:
                    out[ver][key] = {**ent, "gemm": name, "model": model, "tp": int(tp)}
            del ws
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {len(out[ver])} xd entries to {a.out}", flush=True)


if __name__ == "__main__":
    main()
