#!/usr/bin/env python3
"""MoE layer at Mixtral prefill size: where does the fused MoE's time go, against the dense
gemm_w4 GEMMs of the same per-expert shapes?  (Round 6: the suggestions wave spends half its
time in 16k-token prefill chunks whose MoE layers run at ~1.1 PF/s.)

Runs ops.fused_moe at T tokens (default 16384: ~4k rows per expert, top-2 of 8) N times - for
a rocprofv3 kernel trace - and times, interleaved: the fused MoE layer; 8 x the dense expert
GEMMs on gemm_w4 (gate_up + SiLU-GLU epilogue, then down) with the rows already in expert
order, i.e. the layer with no routing / gather / combine and perfect per-expert shapes.
Round 6 (r6j): the fused layer on variant 3 (gemm_xd grouped forms) and variant 4 (rows
gathered into expert order + gemm_w4's grouped persistent form), each checked against the
other first.  DRTC_MOE_CHUNK sets the token chunk per kernel call."""
import statistics
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from drtc_amd import ops  # noqa: E402
from drtc_amd.ops import gemm as G  # noqa: E402
from drtc_amd.ops import moe as moe_ops  # noqa: E402


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    H, I, E, k = 4096, 14336, 8, 2
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    wgu = ((torch.rand(E, 2 * I, H, device=dev, generator=g) * 2 - 1) * 0.02).to(torch.bfloat16)
    wdn = ((torch.rand(E, H, I, device=dev, generator=g) * 2 - 1) * 0.02).to(torch.bfloat16)
    ws = moe_ops.make_workspace(moe_ops.MOE_CHUNK, H, I, E, k, dev)
    G.gemm_workspace(torch.device(dev))
    x = ((torch.rand(T, H, device=dev, generator=g) * 2 - 1)).to(torch.bfloat16)
    lg = torch.randn(T, E, device=dev, generator=g).to(torch.bfloat16)
    out = torch.empty_like(x)
    rows = T * k // E
    xe = x[:rows].contiguous()
    he = torch.empty(rows, I, device=dev, dtype=torch.bfloat16)
    ye = torch.empty(rows, H, device=dev, dtype=torch.bfloat16)

    def fused(v):
        return lambda: ops.fused_moe(x, lg, wgu, wdn, k, workspace=ws, out=out, variant=v)

    o3 = ops.fused_moe(x, lg, wgu, wdn, k, workspace=ws, variant=3).float()
    o4 = ops.fused_moe(x, lg, wgu, wdn, k, workspace=ws, variant=4).float()
    print(f"T={T} v3 vs v4 max abs diff {(o3 - o4).abs().max().item():.4g} "
          f"(scale {o3.abs().max().item():.4g})", flush=True)
    del o3, o4

    def dense():
        for e in range(E):
            G.mfma_gemm(xe, wgu[e], "silu", out=he, variant=G._w4v(H),
                        group_m=G.w4_group_m(rows, I, H, glu=True))
            G.mfma_gemm(he, wdn[e], "store", out=ye, variant=G._w4v(I),
                        group_m=G.w4_group_m(rows, H, I))

    def dense_lib_down():
        for e in range(E):
            G.mfma_gemm(xe, wgu[e], "silu", out=he, variant=G._w4v(H),
                        group_m=G.w4_group_m(rows, I, H, glu=True))
            torch.matmul(he, wdn[e].t(), out=ye)

    lib = __import__("drtc_amd.ops._ext", fromlist=["hipk"]).hipk()

    def fused_rot():  # variant 4 with the per-XCD K rotation in the grouped GEMMs (A/B arm)
        lib.w4_set_grouped_rot(1)
        ops.fused_moe(x, lg, wgu, wdn, k, workspace=ws, out=out, variant=4)
        lib.w4_set_grouped_rot(0)

    def fused_gm(gu, dn):  # variant 4 with other row groups in the grouped tile order
        def f():
            lib.moe_set_w4_group_m(gu, dn)
            ops.fused_moe(x, lg, wgu, wdn, k, workspace=ws, out=out, variant=4)
            lib.moe_set_w4_group_m(0, 0)
        return f

    gms = [tuple(int(v) for v in a.split("/")) for a in
           __import__("os").environ.get("MOE_GM_ARMS", "").split(",") if a]
    arms = {"fused_moe_v3": fused(3), "fused_moe_v4": fused(4), "fused_moe_v4_rot": fused_rot,
            **{f"fused_moe_v4_gm{gu}/{dn}": fused_gm(gu, dn) for gu, dn in gms},
            "dense_w4_x8": dense,
            "dense_w4_gu_lib_down_x8": dense_lib_down}
    for f in arms.values():
        f()
    torch.cuda.synchronize()
    ts = {n: [] for n in arms}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        for n, f in arms.items():
            e0.record()
            for _ in range(3):
                f()
            e1.record()
            e1.synchronize()
            ts[n].append(e0.elapsed_time(e1) / 3)
    fl = 2.0 * T * k * 3 * H * I
    for n, t in ts.items():
        ms = statistics.median(t)
        print(f"T={T} {n:28s} {ms:8.3f} ms  {fl / ms / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
