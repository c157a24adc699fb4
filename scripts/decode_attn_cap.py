#!/usr/bin/env python3
"""Decode attention (fused RoPE + KV write, persistent kernel) at the headline shape with its
grid capped at G workgroups (4 waves each): how many CUs does the HBM-bound attention need?
(size a CU-limited attention grid that could run beside the projections.)

Llama-3-8B heads (Hq 32, Hkv 8, D 128), contexts 150-200 tokens (the smart-reply decode),
B = 1024 and 512 (a micro-batch half).  Prints one JSON line per (B, G): us per call and the
K+V bytes read per second.  argv[1]: comma-separated caps (default: the sweep below);
argv[2]: context orders, "random" and / or "sorted" (longest first, as the engine's slots)."""
import json
import math
import random
import sys

import torch

sys.path.insert(0, ".")
from drtc_amd import ops  # noqa: E402


def main():
    caps = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else
                             "0,512,384,256,192,160,128,96,64,32").split(",")]
    dev = torch.device("cuda")
    Hq, Hkv, D, bs = 32, 8, 128, ops.KV_BLOCK
    rng = random.Random(0)
    cos_sin = ops.build_rope_cache(4096, D, 500000.0, None, dev)
    orders = sys.argv[2].split(",") if len(sys.argv) > 2 else ["random"]
    for B, order in [(b, o) for b in (1024, 512) for o in orders]:
        ctxs = [rng.randint(150, 200) for _ in range(B)]
        if order == "sorted":  # the engine's slot order (LLMEngine._sort_slots)
            ctxs.sort(reverse=True)
        maxb = max(math.ceil(c / bs) for c in ctxs)
        nb = sum(math.ceil(c / bs) for c in ctxs) + 1
        kc = torch.randn(nb, Hkv, bs, D, device=dev, dtype=torch.bfloat16)
        vc = torch.randn(nb, Hkv, D, bs, device=dev, dtype=torch.bfloat16)
        perm = torch.randperm(nb - 1) + 1
        bt = torch.zeros(B, maxb, dtype=torch.int32)
        k = 0
        for b, c in enumerate(ctxs):
            n = math.ceil(c / bs)
            bt[b, :n] = perm[k:k + n].to(torch.int32)
            k += n
        bt = bt.to(dev)
        ctx = torch.tensor(ctxs, dtype=torch.int32, device=dev)
        pos = ctx - 1
        # the step's token goes to its slot (rewritten with the same bytes every call)
        slots = torch.tensor([int(bt[b, (c - 1) // bs]) * bs + (c - 1) % bs
                              for b, c in enumerate(ctxs)], dtype=torch.int64, device=dev)
        qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
        out = torch.empty(B, Hq, D, device=dev, dtype=torch.bfloat16)
        bpp, parts = ops.decode_partitioning(B, Hkv, maxb, D=D)
        ws = ops.DecodeWorkspace(B, Hq, D, parts, dev)
        kv_bytes = sum(c - 1 for c in ctxs) * Hkv * D * 2 * 2
        ref = None
        for G in caps:
            def fn():
                ops.paged_decode_attention_rope(qkv, pos, slots, cos_sin, Hq, Hkv, D, kc, vc, bt,
                                                ctx, D ** -0.5, out=out, blocks_per_part=bpp,
                                                workspace=ws, max_wgs=G)
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            same = bool(torch.equal(out, ref))  # the grid size never changes the result
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(20):
                    fn()
            for _ in range(2):
                g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(5):
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / 20)
            us = sorted(ts)[len(ts) // 2]
            print(json.dumps({"B": B, "order": order, "max_wgs": G, "us": round(us, 2),
                              "kv_TBs": round(kv_bytes / us / 1e6, 3), "same_as_full": same}),
                  flush=True)


if __name__ == "__main__":
    main()
