#!/usr/bin/env python3
"""Time the packed varlen prefill attention kernel on chat-shaped batches.

Prints one JSON line per shape: us per call and effective TFLOP/s (causal
FLOPs = 4 * sum(n^2)/2 * Hq * D) for both launch forms - persistent
workgroups and one workgroup per (query tile, head group) - timed in
interleaved rounds in one process, and checks that both forms give bitwise
identical outputs (same per-tile math and order).
"""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from drtc_amd import ops  # noqa: E402

SHAPES = [  # (name, nseq, mean len, Hq, Hkv, D)
    ("llama8b_smart_reply", 1024, 148, 32, 8, 128),
    ("llama8b_smart_reply_16k_chunk", 110, 148, 32, 8, 128),
    ("llama8b_summarize", 512, 432, 32, 8, 128),
    ("llama8b_long", 16, 4096, 32, 8, 128),
    ("gemma2b_smart_reply", 1024, 148, 8, 1, 256),
    ("llama70b_ask", 256, 136, 64, 8, 128),
]


def main():
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    dev = torch.device("cuda")
    rng = random.Random(0)
    for name, nseq, mean, Hq, Hkv, D in SHAPES:
        if only and name != only:
            continue
        lens = [max(8, int(rng.gauss(mean, mean * 0.1))) for _ in range(nseq)]
        cu = [0]
        for n in lens:
            cu.append(cu[-1] + n)
        T = cu[-1]
        qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
        cu_d = torch.tensor(cu, dtype=torch.int32, device=dev)
        ts, tq = ops.prefill_tiles(cu)
        tiles = (torch.tensor(ts, dtype=torch.int32, device=dev),
                 torch.tensor(tq, dtype=torch.int32, device=dev))
        outs = {}
        times = {}
        for form in ("persist", "per_item"):
            outs[form] = torch.empty(T, Hq * D, device=dev, dtype=torch.bfloat16)
            times[form] = []
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        for _ in range(5):
            for form in ("persist", "per_item"):
                ops.set_prefill_persist(form == "persist")
                o = outs[form]
                f = lambda: ops.prefill_attention(qkv, cu_d, Hq, Hkv, D, D ** -0.5, True,
                                                  tiles=tiles, cu_host=cu, out=o)
                f()
                torch.cuda.synchronize()
                e0.record()
                for _ in range(it):
                    f()
                e1.record()
                torch.cuda.synchronize()
                times[form].append(1000 * e0.elapsed_time(e1) / it)
        ops.set_prefill_persist(None)
        same = torch.equal(outs["persist"], outs["per_item"])
        flops = 4 * sum(n * (n + 1) / 2 for n in lens) * Hq * D
        for form, ts in times.items():
            us = sorted(ts)[len(ts) // 2]
            print(json.dumps({"form": form, "shape": name, "tokens": T, "us": round(us, 1),
                              "TFLOPs": round(flops / us / 1e6, 1), "bitwise_equal": same}),
                  flush=True)


if __name__ == "__main__":
    main()
