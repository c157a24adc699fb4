#!/usr/bin/env python3
"""Extended gemm_xd form search against the CURRENT tuned route, for the decode shapes that
dominate a model's step (round 6: Llama-3-70B ask at 192-256 rows, Llama-3-8B at 768-1024).

tune_xd.py's candidate list holds single-slice forms of every tile and split-K 2-4 of the
256-row tiles.  Here every built tile (``ops.gemm.XD_TILES``) runs with K split 1..8 ways,
plain and non-temporal, and the baseline is the form the router runs today (the tuning table's
pick for that shape; the GLU form for a gate_up), timed in the same process with the weights
streamed from HBM (rotated copies >= 512 MB) and arms interleaved (tune_midm.time_arm).  Every
form is checked against an fp32 reference first.

Prints one JSON line per shape and writes the entries that beat today's pick by at least
--min-gain as a merge file for ``scripts/tune_gemms.py --merge`` ({"xd": form} / {"xd_glu":
form}, nt_tuned so the router runs the pick as chosen).

usage (GPU): python scripts/tune_xd_ext.py --configs llama-3-70b:1 --ms 192,224,256
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


def ext_forms(G, M, N, K, glu):
    out = []
    for (mt, nf) in sorted(G.XD_TILES):
        for sk in range(1, G.XD_MAX_SPLITK + 1):
            f = mt * 100 + nf * 10 + sk
            for form in (f, f + 1000):
                if G.xd_supported(M, N, K, form, glu):
                    out.append(form)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="llama-3-70b:1")
    ap.add_argument("--ms", default="192,224,256")
    ap.add_argument("--gemms", default="qkv,o,gate_up,down")
    ap.add_argument("--min-gain", type=float, default=0.02)
    ap.add_argument("--out", default="gpurun_out/xd_ext_tuned.json")
    a = ap.parse_args()
    from drtc_amd.ops import gemm as G
    from drtc_amd.ops._ext import hipk

    dev = torch.device("cuda", 0)
    G.gemm_workspace(dev)
    ver = str(hipk().lt_version())
    out = {ver: {}}
    g = torch.Generator(device=dev).manual_seed(0)
    for spec in a.configs.split(","):
        model, tp = spec.split(":")
        for name, (N, K) in projection_shapes(model, int(tp)).items():
            if name not in a.gemms.split(","):
                continue
            ncopy = max(2, min(10, -(-512 * 2**20 // (N * K * 2))))
            ws = [(torch.randn(N, K, device=dev, generator=g) * 0.02).to(torch.bfloat16)
                  for _ in range(ncopy)]
            for M in (int(m) for m in a.ms.split(",")):
                x = torch.randn(M, K, device=dev, generator=g).to(torch.bfloat16)
                for epi in (("silu",) if name == "gate_up" else ("store",)):
                    glu = epi != "store"
                    No = N // 2 if glu else N
                    # today's route for this shape (what the engine runs)
                    if glu:
                        cur = G.glu_form(M, N, K, K)
                        if not cur:
                            continue
                        def base(w, cur=cur):
                            return G.xd_gemm(x, w, epi, form=cur)
                    else:
                        kind, arg = G.route(M, N, K, K)
                        cur = arg if kind == "xd" else f"{kind}:{arg}"
                        def base(w):
                            return G.linear(x, w)
                    y = x.float() @ ws[0].float().t()
                    if glu:
                        y = torch.nn.functional.silu(y[:, :No]) * y[:, No:]
                    time_arm(base, ws)  # clocks up: the first arm timed is not favoured
                    base_us = time_arm(base, ws)
                    best = None
                    times = {}
                    for f in ext_forms(G, M, No, K, glu):
                        got = G.xd_gemm(x, ws[0], epi, form=f)
                        err = ((got.float() - y).abs().max() / y.abs().max()).item()
                        if err > 2e-2:
                            print(json.dumps({"M": M, "gemm": name, "form": f, "err": err,
                                              "FAILED": True}), flush=True)
                            continue
                        us = time_arm(lambda w, f=f: G.xd_gemm(x, w, epi, form=f), ws)
                        times[f] = us
                        if best is None or us < best[1]:
                            best = (f, us)
                    del y
                    rec = {"model": model, "tp": int(tp), "gemm": name, "epi": epi, "M": M,
                           "N": No, "K": K, "current": cur, "current_us": round(base_us, 1),
                           "best": best[0] if best else None,
                           "best_us": round(best[1], 1) if best else None}
                    if best:
                        # against today's form timed in the same sweep where it is a candidate
                        ref = times.get(cur, base_us) if isinstance(cur, int) else base_us
                        rec.update(current_in_sweep_us=round(ref, 1),
                                   gain=round(ref / best[1] - 1, 3),
                                   top3=sorted(((round(v, 1), k) for k, v in times.items()))[:3])
                        base_us = ref
                    print(json.dumps(rec), flush=True)
                    if best and best[1] < base_us * (1 - a.min_gain):
                        key = f"{M},{N},{K},{K}"
                        ent = out[ver].setdefault(key, {"gemm": name, "model": model,
                                                        "tp": int(tp), "nt_tuned": True})
                        if glu:
                            ent.update(xd_glu=best[0], xd_glu_us=round(best[1], 1))
                        else:
                            ent.update(xd=best[0], xd_us=round(best[1], 1))
            del ws
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {len(out[ver])} entries to {a.out}", flush=True)


if __name__ == "__main__":
    main()
