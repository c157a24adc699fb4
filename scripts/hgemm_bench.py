#!/usr/bin/env python3
"""Hand-written MFMA GEMM (csrc/kernels/gemm.hip) vs the library path, Llama-3 shapes.

For each projection of the model at a decode batch (M = 1024) and a prefill chunk
(M = 16384) this script
  1. checks every requested kernel variant against an fp32 PyTorch reference of the same
     op (including the fused epilogue: residual add, SiLU/GELU gating), and
  2. times the variants and the library baseline INTERLEAVED in one process (rounds x
     variants, each `--iters` back-to-back launches, or a hipGraph of them with --graphs;
     cdna_hip_programming.md §5.4 rule 24)
     on random operands, reporting the median and min per arm.

Library baseline = what the engine ran before this kernel: ops.linear (tuned
hipBLASLt solution where the table has one) + ops.act_glu for the gated MLP,
residual.addmm_ (hipBLASLt beta=1) for the residual forms.

Output: one JSON line per (shape, arm) and gpurun_out/hgemm_bench.json.
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import drtc_amd  # noqa: E402
from drtc_amd import ops  # noqa: E402
from drtc_amd.ops import gemm as G  # noqa: E402

MODELS = {
    # name: (hidden, intermediate, qkv_out, vocab)
    "8b": (4096, 14336, 6144, 128256),
    "70b": (8192, 28672, 10240, 128256),
    "gemma2b": (2048, 16384, 2560, 256000),
}


def cases(model: str, ms: list[int]):
    H, I, QKV, V = MODELS[model]
    out = []
    for M in ms:
        out.append(("qkv", M, QKV, H, "store"))
        out.append(("o", M, H, H, "residual"))
        out.append(("gate_up", M, 2 * I, H, "silu"))
        out.append(("down", M, H, I, "residual"))
        if M <= 1024:
            out.append(("lm_head", M, V, H, "store"))
    return out


def reference(x, w, epi, res):
    y = x.float() @ w.float().t()
    if epi == "residual":
        y = y + res.float()
    elif epi in ("silu", "gelu_tanh"):
        i = w.shape[0] // 2
        g, u = y[:, :i], y[:, i:]
        a = F.silu(g) if epi == "silu" else F.gelu(g, approximate="tanh")
        y = a * u
    return y


def lib_fn(x, w, epi, res, out):
    if epi == "residual":
        return lambda: res.addmm_(x, w.t())
    if epi in ("silu", "gelu_tanh"):
        return lambda: ops.act_glu(ops.linear(x, w), epi)
    return lambda: ops.linear(x, w)


def eager_time(fn, iters):
    """Back-to-back launches between two events (kernels here run 20-3000 us, far
    above the host's launch cost, so the queue stays full)."""
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run():
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1e3 / iters  # us

    return run


def graph_time(fn, iters):
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
        return s.elapsed_time(e) * 1e3 / iters  # us

    run.keep = (fn, g)  # the graph writes into buffers fn's closure keeps alive
    return run


def smoke(variants):
    """Tiny shapes first (every variant x epilogue x split), one launch + sync each."""
    dev = torch.device("cuda")
    for M, N, K in ((256, 256, 256), (300, 512, 512)):
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
        for epi in ("store", "residual", "silu"):
            nout = N // 2 if epi == "silu" else N
            res = torch.randn(M, nout, device=dev, dtype=torch.bfloat16) if epi == "residual" else None
            ref = reference(x, w, epi, res)
            for v in variants:
                for sk in (1, 2):
                    print(f"# smoke M={M} N={N} K={K} {epi} v{v} sk{sk}", flush=True)
                    o = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
                    G.mfma_gemm(x, w, epi, residual=res, out=o, variant=v, splitk=sk)
                    torch.cuda.synchronize()
                    err = (o.float() - ref).abs().max().item() / ref.abs().max().item()
                    print(f"#   err {err:.5f}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="8b", choices=list(MODELS))
    ap.add_argument("--ms", default="1024,16384")
    ap.add_argument("--variants", default="1,2,3")
    ap.add_argument("--splitk", default="auto", help="'auto' or comma list tried for every shape")
    ap.add_argument("--only", default="", help="comma list of gemm names")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--group-ms", default="8", help="comma list of row-tile group sizes")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--smoke", action="store_true", help="tiny-shape launch checks first")
    ap.add_argument("--smoke-only", action="store_true")
    ap.add_argument("--graphs", action="store_true", help="time hipGraph replays (default: eager)")
    ap.add_argument("--out", default="gpurun_out/hgemm_bench.json")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    variants = [int(v) for v in a.variants.split(",")]
    G.gemm_workspace(dev)  # split-K workspace exists before any capture
    if a.smoke or a.smoke_only:
        smoke(variants)
    if a.smoke_only:
        return
    results = []
    for name, M, N, K, epi in cases(a.model, [int(m) for m in a.ms.split(",")]):
        if a.only and name not in a.only.split(","):
            continue
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = (torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02)
        nout = N // 2 if epi in ("silu", "gelu_tanh") else N
        res = torch.randn(M, nout, device=dev, dtype=torch.bfloat16) if epi == "residual" else None
        if a.splitk == "auto":
            tiles = -(-M // 256) * (nout // (128 if epi in ("silu", "gelu_tanh") else 256))
            sks = [1] + [s for s in (2, 3, 4, 6, 8) if (K // 64) % s == 0 and tiles * s <= 320
                         and tiles * s * (1 << 18) <= G.WS_SLAB_BYTES]
        else:
            sks = [int(s) for s in a.splitk.split(",") if (K // 64) % int(s) == 0]
        arms = {"lib": None}
        gms = [int(g) for g in a.group_ms.split(",")]
        for v in variants:
            for sk in sks:
                for gm_ in gms:
                    arms[f"v{v}_sk{sk}" + (f"_g{gm_}" if len(gms) > 1 else "")] = (v, sk, gm_)
        # correctness
        ref = None if a.no_check else reference(x, w, epi, res)
        status = {}
        print(f"# case {name} M={M} N={N} K={K} {epi}", flush=True)
        for arm, cfg in arms.items():
            if cfg is None:
                continue
            v, sk, gm_ = cfg
            o = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
            r_in = res.clone() if res is not None else None
            print(f"# check {name} M={M} {arm}", flush=True)
            G.mfma_gemm(x, w, epi, residual=r_in, out=o, variant=v, splitk=sk, group_m=gm_)
            torch.cuda.synchronize()  # a fault ends the run here, naming the arm above
            if ref is not None:
                err = (o.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
                status[arm] = round(err, 5)
            else:
                status[arm] = "unchecked"
            print(f"#   err {status[arm]}", flush=True)
        if ref is not None:
            del ref
        torch.cuda.empty_cache()
        # timing (interleaved rounds)
        runners = {}
        for arm, cfg in arms.items():
            if cfg is not None and isinstance(status.get(arm), float) and status[arm] > 2e-2:
                continue  # wrong result: do not time
            o = torch.empty(M, nout, device=dev, dtype=torch.bfloat16)
            rr = res.clone() if res is not None else None
            if cfg is None:
                fn = lib_fn(x, w, epi, rr, o)
            else:
                v, sk, gm_ = cfg
                if epi == "residual":
                    fn = (lambda v=v, sk=sk, rr=rr, gm_=gm_: G.mfma_gemm(
                        x, w, epi, residual=rr, out=rr, variant=v, splitk=sk, group_m=gm_))
                else:
                    fn = (lambda v=v, sk=sk, o=o, gm_=gm_: G.mfma_gemm(
                        x, w, epi, out=o, variant=v, splitk=sk, group_m=gm_))
            runners[arm] = (graph_time if a.graphs else eager_time)(fn, a.iters)
        times = {arm: [] for arm in runners}
        for _ in range(a.rounds):
            for arm, run in runners.items():
                times[arm].append(run())
        flops = 2.0 * M * N * K
        for arm, ts in times.items():
            med = statistics.median(ts)
            r = {"model": a.model, "gemm": name, "M": M, "N": N, "K": K, "epi": epi, "arm": arm,
                 "us_med": round(med, 1), "us_min": round(min(ts), 1),
                 "TFLOPs": round(flops / med / 1e6, 1), "err": status.get(arm, "lib")}
            results.append(r)
            print(json.dumps(r), flush=True)
        del runners
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(results, f, indent=0)


if __name__ == "__main__":
    main()
