#!/usr/bin/env python3
"""Decode-batch GEMM (csrc/kernels/gemm_dec.hip) vs the engine's library path.

For each projection of a model at decode batch buckets (default M = 256, 512, 1024):
  1. numerics of every (nr, group_m) arm against an fp32 PyTorch reference of the same op
     (store; SiLU-gated [gate; up] for gate_up; residual add for o / down with --residual);
  2. interleaved timing (rounds x arms, each a hipGraph of --iters launches) of the arms
     and of the library path the engine runs today: ops.linear (tuned hipBLASLt solution)
     and, for gate_up, ops.act_glu after it.

Prints one JSON line per (shape, arm) and writes --out.
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import drtc_amd  # noqa: E402,F401
from drtc_amd import ops  # noqa: E402
from drtc_amd.ops import gemm as G  # noqa: E402

MODELS = {  # name: (hidden, intermediate, qkv_out)
    "8b": (4096, 14336, 6144),
    "70b": (8192, 28672, 10240),
    "gemma2b": (2048, 16384, 2560),
}


def reference(x, w, epi, res):
    y = x.float() @ w.float().t()
    if epi == "residual":
        y = y + res.float()
    elif epi in ("silu", "gelu_tanh"):
        i = w.shape[0] // 2
        a = F.silu(y[:, :i]) if epi == "silu" else F.gelu(y[:, :i], approximate="tanh")
        y = a * y[:, i:]
    return y


def graph_timer(fn, iters):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run():
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1e3 / iters

    # the graph holds raw pointers to the tensors fn's closure keeps alive (its output
    # buffer): keep fn with the graph, or the next capture's empty_cache() hands that
    # memory back to the driver and the next replay writes into freed memory
    run.keep = (fn, g)
    return run


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="8b", choices=list(MODELS))
    ap.add_argument("--ms", default="256,512,1024")
    ap.add_argument("--cfgs", default="18,24,26,28", help="10 * pipeline + LDS regions")
    ap.add_argument("--group-ms", default="8")
    ap.add_argument("--only", default="")
    ap.add_argument("--residual", action="store_true", help="o / down with the residual epilogue")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/decgemm_bench.json")
    ap.add_argument("--no-lib", action="store_true", help="time the hand-kernel arms only")
    ap.add_argument("--diag", action="store_true",
                    help="per arm: --iters eager launches + sync, then one graph replay + sync, "
                         "printed before each step (finds a faulting arm); no timing table")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    H, I, QKV = MODELS[a.model]
    results = []
    for M in [int(m) for m in a.ms.split(",")]:
        for name, N, K, epi in (("qkv", QKV, H, "store"), ("o", H, H, "residual" if a.residual else "store"),
                                ("gate_up", 2 * I, H, "silu"),
                                ("down", H, I, "residual" if a.residual else "store")):
            if a.only and name not in a.only.split(","):
                continue
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            glu = epi == "silu"
            nout = N // 2 if glu else N
            res = torch.randn(M, nout, device=dev, dtype=torch.bfloat16) if epi == "residual" else None
            ref = reference(x, w, epi, res)
            arms = {} if a.no_lib else {"lib": None}
            for c in [int(v) for v in a.cfgs.split(",")]:
                for gm in [int(v) for v in a.group_ms.split(",")]:
                    arms[f"dec_v{c // 10}nr{c % 10}_g{gm}"] = (c % 10, gm, c // 10)
            errs = {}
            outs = {}
            for arm, cfg in arms.items():
                print(f"# check {name} M={M} {arm}", flush=True)
                if cfg is None:
                    if epi == "residual":
                        r2 = res.clone()
                        o = r2.addmm_(x, w.t())
                    else:
                        o = ops.linear(x, w)
                        if glu:
                            o = ops.act_glu(o, "silu")
                else:
                    r2 = res.clone() if res is not None else None
                    o = G.dec_gemm(x, w, epi, residual=r2, out=r2, nr=cfg[0], group_m=cfg[1],
                                   pipe=cfg[2])
                torch.cuda.synchronize()  # a fault stops here, naming the arm above
                errs[arm] = round((o.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6), 5)
                outs[arm] = o
                print(f"#   err {errs[arm]}", flush=True)
            del ref, outs
            runners = {}
            for arm, cfg in (reversed(list(arms.items())) if a.diag else arms.items()):
                if cfg is None:
                    if epi == "residual":
                        fn = (lambda: res.addmm_(x, w.t()))
                    elif glu:
                        fn = (lambda: ops.act_glu(ops.linear(x, w), "silu"))
                    else:
                        fn = (lambda: ops.linear(x, w))
                else:
                    o = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
                    fn = (lambda cfg=cfg, o=o: G.dec_gemm(x, w, epi, residual=res, out=o,
                                                          nr=cfg[0], group_m=cfg[1], pipe=cfg[2]))
                if a.diag:
                    print(f"# diag eager {name} M={M} {arm}", flush=True)
                    for _ in range(a.iters):
                        fn()
                    torch.cuda.synchronize()
                    print(f"# diag graph {name} M={M} {arm}", flush=True)
                    graph_timer(fn, a.iters)()
                    torch.cuda.synchronize()
                    print(f"# diag ok {name} M={M} {arm}", flush=True)
                    continue
                runners[arm] = graph_timer(fn, a.iters)
            if a.diag:
                continue
            times = {arm: [] for arm in arms}
            for _ in range(a.rounds):
                for arm, run in runners.items():
                    times[arm].append(run())
            flops = 2.0 * M * N * K
            lib = statistics.median(times["lib"]) if "lib" in times else float("nan")
            for arm in arms:
                med = statistics.median(times[arm])
                r = {"model": a.model, "gemm": name, "M": M, "N": N, "K": K, "epi": epi, "arm": arm,
                     "us": round(med, 2), "min_us": round(min(times[arm]), 2),
                     "tflops": round(flops / med / 1e6, 1), "vs_lib": round(lib / med, 3),
                     "err": errs[arm]}
                results.append(r)
                print(json.dumps(r), flush=True)
            del runners
            torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
