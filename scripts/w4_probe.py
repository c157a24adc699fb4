#!/usr/bin/env python3
"""Focused A/B probe of one GEMM shape: hipBLASLt (ops.linear / addmm_ beta=1) against the
hand-written kernels of ops.gemm.mfma_gemm, interleaved in one process (rule 24), for
rocprofv3 PMC passes and quick timing.

  python scripts/w4_probe.py --shape 16384,6144,4096 --epi store --arms lib,v7 --iters 10
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
from drtc_amd.ops import gemm as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="16384,6144,4096", help="M,N,K (N = rows of W)")
    ap.add_argument("--epi", default="store")
    ap.add_argument("--arms", default="lib,v7")
    ap.add_argument("--splitk", type=int, default=1)
    ap.add_argument("--group-m", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--rotate", type=int, default=1,
                    help="cycle through this many weight copies (> the 256 MB MALL in total: "
                         "weights stream from HBM as inside a model step)")
    a = ap.parse_args()
    M, N, K = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(a.rotate)]
    w = ws[0]
    cur = [0]

    def nxt():  # the weight copy of the next call (same copy when --rotate 1)
        cur[0] = (cur[0] + 1) % a.rotate
        return ws[cur[0]]
    glu = a.epi in ("silu", "gelu_tanh")
    nout = N // 2 if glu else N
    res = torch.randn(M, nout, device=dev, dtype=torch.bfloat16) if a.epi == "residual" else None
    out = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
    G.gemm_workspace(dev)
    # "lib" is the library path the engine had before the hand decode GEMMs: route around the
    # gemm_xd table entries (ops.linear would otherwise dispatch them)
    G._xd_enabled = False
    G.reset()
    fns = {}
    for arm in a.arms.split(","):
        if arm == "lib":
            if a.epi == "residual":
                fns[arm] = lambda: res.addmm_(x, nxt().t())
            elif glu:
                fns[arm] = lambda: ops.act_glu(ops.linear(x, nxt()), a.epi)
            else:
                fns[arm] = lambda: ops.linear(x, nxt())
        elif arm[0] == "x":  # "xFORM": gemm_xd form mt*100 + nf*10 + splitk (x0: by shape)
            form = int(arm[1:] or 0)
            if a.epi == "residual":
                fns[arm] = lambda form=form: G.xd_gemm(x, nxt(), "residual", residual=res,
                                                       out=res, form=form)
            else:
                fns[arm] = lambda form=form: G.xd_gemm(x, nxt(), a.epi, out=out, form=form)
        else:
            # "vV" or "vV:splitk:group_m[:kR]" (group_m < 0: K-slice-by-XCD tile order;
            # kR: R distinct per-XCD K start offsets of the rotating variants, w4_set_krot)
            f = arm[1:].split(":")
            v = int(f[0])
            sk = int(f[1]) if len(f) > 1 else a.splitk
            gm = int(f[2]) if len(f) > 2 else a.group_m
            kr = int(f[3][1:]) if len(f) > 3 else 8
            if a.epi == "residual":
                fns[arm] = (lambda v=v, sk=sk, gm=gm: G.mfma_gemm(
                    x, nxt(), "residual", residual=res, out=res, variant=v, splitk=sk, group_m=gm))
            else:
                fns[arm] = (lambda v=v, sk=sk, gm=gm: G.mfma_gemm(
                    x, nxt(), a.epi, out=out, variant=v, splitk=sk, group_m=gm))
            from drtc_amd.ops._ext import hipk as _hk

            def with_krot(f0=fns[arm], kr=kr):  # every call runs with this arm's K rotation
                _hk().w4_set_krot(kr)
                try:
                    return f0()
                finally:
                    _hk().w4_set_krot(8)
            fns[arm] = with_krot
    # correctness of every hand arm against an fp32 reference (one call each)
    ref = x.float() @ w.float().t()
    if a.epi == "residual":
        ref = ref + res.float()
    elif glu:
        ref = (torch.nn.functional.silu(ref[:, :nout]) if a.epi == "silu" else
               torch.nn.functional.gelu(ref[:, :nout], approximate="tanh")) * ref[:, nout:]
    errs = {}
    for k, f in fns.items():
        if k == "lib":
            continue
        cur[0] = a.rotate - 1  # the next call uses ws[0] = w
        if a.epi == "residual":
            r0 = res.clone()
            f()
            got, res.data = res.clone(), r0
        else:
            got = f()
        torch.cuda.synchronize()
        errs[k] = round((got.float() - ref).abs().max().item() / ref.abs().max().item(), 5)
    del ref
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in fns}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for k, f in fns.items():
            s.record()
            for _ in range(a.iters):
                f()
            e.record()
            e.synchronize()
            times[k].append(s.elapsed_time(e) * 1e3 / a.iters)
    fl = 2.0 * M * N * K
    for k, ts in times.items():
        med = statistics.median(ts)
        print(json.dumps({"shape": [M, N, K], "epi": a.epi, "arm": k, "splitk": a.splitk,
                          "rotate": a.rotate, "us_med": round(med, 1),
                          "us_min": round(min(ts), 1), "TFLOPs": round(fl / med / 1e6, 1),
                          "err": errs.get(k)}),
              flush=True)


if __name__ == "__main__":
    main()
