#!/usr/bin/env python3
"""Measure the best hipBLASLt solution for every decode projection GEMM of a
model (each hipGraph batch bucket x qkv / o / gate_up / down / lm_head) and
write the tuning entries that beat hipBLASLt's heuristic pick.

usage (GPU): python scripts/tune_gemms.py --model llama-3-8b [--tp 8]
             [--ms 256,512,1024] [--out gpurun_out/gemm_tuned.json]
Merge the output into the in-tree table with --merge FILE (CPU side):
             python scripts/tune_gemms.py --merge gpurun_out/gemm_tuned.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from drtc_amd.engine.decode_runner import DEFAULT_BUCKETS  # noqa: E402
from drtc_amd.models import get_config  # noqa: E402
from drtc_amd.models.transformer import ShardInfo  # noqa: E402


def projection_shapes(name: str, tp: int) -> dict[str, tuple[int, int]]:
    """(N, K) of each decode projection of one TP shard."""
    cfg = get_config(name)
    sh = ShardInfo(cfg, SimpleNamespace(tp_size=tp, tp_rank=0, ep_size=1, ep_rank=0))
    H, D = cfg.hidden_size, cfg.head_dim
    shapes = {"qkv": ((sh.hq + 2 * sh.hkv) * D, H), "o": (H, sh.hq * D),
              "lm_head": (sh.vocab, H)}
    if not cfg.is_moe:  # MoE experts run in the fused HIP MoE kernel
        shapes["gate_up"] = (2 * sh.inter, H)
        shapes["down"] = (H, sh.inter)
    return shapes


def merge(src: str) -> None:
    from drtc_amd.ops import gemm

    with open(src) as f:
        new = json.load(f)
    path = gemm.table_path()
    data = gemm.load_table(path)
    for ver, entries in new.items():  # per key: new fields over old (algo / skinny picks)
        cur = data.setdefault(ver, {})
        for k, e in entries.items():
            cur[k] = {**cur.get(k, {}), **e}
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(data, f, indent=1, sort_keys=True)
    print(f"merged {sum(len(e) for e in new.values())} entries into {path}")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--ms", default=None, help="comma list of M (default: every decode bucket)")
    ap.add_argument("--min-gain", type=float, default=0.03,
                    help="keep an entry only if it beats the heuristic pick by this fraction")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="gpurun_out/gemm_tuned.json")
    ap.add_argument("--merge", default=None)
    a = ap.parse_args()
    if a.merge:
        merge(a.merge)
        return
    from drtc_amd.ops import gemm
    from drtc_amd.ops._ext import hipk

    dev = torch.device("cuda", 0)
    ms = [int(m) for m in a.ms.split(",")] if a.ms else list(DEFAULT_BUCKETS)
    ver = str(hipk().lt_version())
    out = {}
    if os.path.exists(a.out):
        with open(a.out) as f:
            out = json.load(f)
    entries = out.setdefault(ver, {})
    shapes = projection_shapes(a.model, a.tp)
    t0 = time.time()
    for M in ms:
        for name, (N, K) in shapes.items():
            if name == "lm_head" and M > 4096:
                continue  # prefill computes logits for the last token of each sequence only
            key = f"{M},{N},{K},{K}"
            r = gemm.tune(M, N, K, dev, iters=a.iters)
            gain = 1.0 - r["us"] / r["heuristic_us"] if r["heuristic_us"] > 0 else 0.0
            r.update(model=a.model, tp=a.tp, gemm=name, gain=round(gain, 3))
            print(json.dumps({"M": M, "N": N, "K": K, **r, "t": round(time.time() - t0, 1)}),
                  flush=True)
            if gain >= a.min_gain and r["algo"] >= 0:
                entries[key] = r
            os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
            with open(a.out, "w") as f:
                json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
