#!/usr/bin/env python3
"""Can two decode half-batches overlap on MI355X?  (decision probe for
two-stream nano-batched decode)

One Llama-3-8B decode layer at B = 1024 (ctx ~172 tokens), built from the
engine's own ops (tuned hipBLASLt GEMMs, fused rope_kv, paged MFMA decode
attention, act_glu, rmsnorm):

  seq1024   : the layer on the full batch (what the engine runs today)
  seq2x512  : the layer on two 512-row halves, one after the other
  par2x512  : the two halves on two streams (no dependency between them)
  *_graph   : the same, captured in one hipGraph (x `--layers` layers)

Also the pieces: GEMMs only and attention only, at 1024 and 2x512.
Prints median microseconds per layer."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtc_amd import ops  # noqa: E402
from drtc_amd.models import LLAMA3_8B  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--ctx", type=int, default=172)
    a = ap.parse_args()
    dev = torch.device("cuda")
    cfg = LLAMA3_8B
    H, I, D, hq, hkv = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
    B, L = 1024, a.layers
    g = torch.Generator(device=dev).manual_seed(0)

    def w(*s):
        return (torch.randn(*s, device=dev, generator=g) * 0.02).to(torch.bfloat16)

    layers = [dict(qkv=w((hq + 2 * hkv) * D, H), o=w(H, hq * D), gu=w(2 * I, H), dn=w(H, I),
                   ln=torch.ones(H, device=dev, dtype=torch.bfloat16)) for _ in range(L)]
    BS = ops.KV_BLOCK
    nblk = -(-(a.ctx + 1) // BS)
    MB = nblk
    n_blocks = B * nblk + 8
    kc = [torch.zeros(n_blocks, hkv, BS, D, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    vc = [torch.zeros(n_blocks, hkv, D, BS, device=dev, dtype=torch.bfloat16) for _ in range(L)]
    bt = torch.arange(B * nblk, device=dev, dtype=torch.int32).view(B, nblk)
    ctx = torch.full((B,), a.ctx + 1, device=dev, dtype=torch.int32)
    pos = torch.full((B,), a.ctx, device=dev, dtype=torch.int32)
    slots = (bt[:, a.ctx // BS].long() * BS + a.ctx % BS)
    cos_sin = ops.build_rope_cache(4096, D, cfg.rope_theta, cfg.rope_scaling, dev)
    x_full = torch.randn(B, H, device=dev, generator=g).to(torch.bfloat16)

    def make(lo, hi):
        n = hi - lo
        bpp, parts = ops.decode_partitioning(n, hkv, MB)
        ws = ops.DecodeWorkspace(n, hq, D, parts, dev)
        st = dict(x=x_full[lo:hi].clone(), res=torch.zeros(n, H, device=dev, dtype=torch.bfloat16),
                  bt=bt[lo:hi].contiguous(), ctx=ctx[lo:hi].contiguous(), pos=pos[lo:hi].contiguous(),
                  slots=slots[lo:hi].contiguous(), bpp=bpp, ws=ws,
                  out=torch.empty(n, hq, D, device=dev, dtype=torch.bfloat16), n=n)
        return st

    def layer(st, i, gemm=True, attn=True):
        Lw = layers[i]
        n = st["n"]
        x = st["x"]
        if gemm:
            h = ops.rmsnorm(x, Lw["ln"], cfg.rms_eps)
            qkv = ops.linear(h, Lw["qkv"])
        else:
            qkv = st.setdefault("qkv_static", torch.zeros(n, (hq + 2 * hkv) * D, device=dev,
                                                          dtype=torch.bfloat16))
        if attn:
            ops.rope_kv_(qkv, st["pos"], st["slots"], cos_sin, hq, hkv, D, kc[i], vc[i], BS)
            q = qkv.as_strided((n, hq, D), (qkv.stride(0), D, 1))
            att = ops.paged_decode_attention(q, kc[i], vc[i], st["bt"], st["ctx"], cfg.attn_scale,
                                             out=st["out"], blocks_per_part=st["bpp"],
                                             workspace=st["ws"])
        else:
            att = st["out"]
        if gemm:
            o = ops.linear(att.view(n, hq * D), Lw["o"])
            h2 = ops.rmsnorm(o, Lw["ln"], cfg.rms_eps)
            gu = ops.linear(h2, Lw["gu"])
            st["x"] = ops.linear(ops.act_glu(gu, cfg.act), Lw["dn"])

    full = make(0, B)
    halves = [make(0, B // 2), make(B // 2, B)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run_seq(sts, gemm=True, attn=True):
        for i in range(L):
            for st in sts:
                layer(st, i, gemm, attn)

    def run_par(gemm=True, attn=True):
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            for i in range(L):
                layer(halves[0], i, gemm, attn)
        with torch.cuda.stream(s2):
            for i in range(L):
                layer(halves[1], i, gemm, attn)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    arms = {
        "layer_seq1024": lambda: run_seq([full]),
        "layer_seq2x512": lambda: run_seq(halves),
        "layer_par2x512": lambda: run_par(),
        "gemm_seq1024": lambda: run_seq([full], attn=False),
        "gemm_seq2x512": lambda: run_seq(halves, attn=False),
        "gemm_par2x512": lambda: run_par(attn=False),
        "attn_seq1024": lambda: run_seq([full], gemm=False),
        "attn_par2x512": lambda: run_par(gemm=False),
    }
    for fn in arms.values():  # warm-up: lazy hipBLASLt init, workspaces
        fn()
    torch.cuda.synchronize()
    graphs = {}
    for name in ("layer_seq1024", "layer_par2x512", "layer_seq2x512", "gemm_par2x512"):
        gph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gph):
            arms[name]()
        graphs[name + "_graph"] = gph
    torch.cuda.synchronize()
    runs = dict(arms)
    runs.update({k: v.replay for k, v in graphs.items()})
    times = {k: [] for k in runs}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for k, fn in runs.items():
            torch.cuda.synchronize()
            ev0.record()
            fn()
            ev1.record()
            ev1.synchronize()
            times[k].append(ev0.elapsed_time(ev1) * 1e3 / L)
    for k, ts in times.items():
        print(json.dumps({"arm": k, "us_per_layer_med": round(statistics.median(ts), 1),
                          "us_per_layer_min": round(min(ts), 1)}), flush=True)


if __name__ == "__main__":
    main()
