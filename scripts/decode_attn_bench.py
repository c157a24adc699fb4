#!/usr/bin/env python3
"""Paged decode attention micro-benchmark: kernel variant 1 (workgroup per
(seq, kv head) + LDS merge) vs 2 (wave per (seq, kv head)), Llama-3-8B
geometry (Hq 32, Hkv 8, D 128) over several batch / context mixes.
Reports us per call and effective HBM GB/s of K+V bytes read."""
import math
import random
import sys

import torch

sys.path.insert(0, ".")
from drtc_amd import ops  # noqa: E402
from drtc_amd.ops.attention import decode_variant  # noqa: E402


def setup(B, ctxs, Hq=32, Hkv=8, D=128, seed=0):
    bs = ops.KV_BLOCK
    maxb = max(math.ceil(c / bs) for c in ctxs)
    nb = sum(math.ceil(c / bs) for c in ctxs) + 1
    kc = torch.randn(nb, Hkv, bs, D, device="cuda", dtype=torch.bfloat16)
    vc = torch.randn(nb, Hkv, D, bs, device="cuda", dtype=torch.bfloat16)
    perm = torch.randperm(nb - 1) + 1
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    k = 0
    for b, c in enumerate(ctxs):
        n = math.ceil(c / bs)
        bt[b, :n] = perm[k:k + n].to(torch.int32)
        k += n
    q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    return q, kc, vc, bt.cuda(), torch.tensor(ctxs, dtype=torch.int32, device="cuda")


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


VARIANTS = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,2,3").split(","))
# geometry set: (Hq, Hkv, D) and the batch / context mixes of the model's bench configs
GEOMS = {
    "llama8b": ((32, 8, 128), None),
    "gemma": ((8, 1, 256), [("B1024 ctx150-200", 1024, (150, 200)), ("B256 ctx150-200", 256, (150, 200)),
                            ("B256 ctx600-1400", 256, (600, 1400))]),
    "mixtral": ((32, 8, 128), [("B256 ctx175-270", 256, (175, 270)), ("B64 ctx175-270", 64, (175, 270))]),
    "llama70b": ((64, 8, 128), [("B256 ctx136-286", 256, (136, 286)),
                                ("B256 ctx136-436", 256, (136, 436)),  # mid-decode of the ask wave
                                ("B64 ctx136-286", 64, (136, 286))]),
}


def main():
    rng = random.Random(0)
    (Hq, Hkv, D), mixes = GEOMS[sys.argv[2] if len(sys.argv) > 2 else "llama8b"]
    cases = [(n, B, (lambda lo=lo, hi=hi: rng.randint(lo, hi))) for n, B, (lo, hi) in mixes] if mixes else [
        ("B1024 ctx150-200", 1024, lambda: rng.randint(150, 200)),
        ("B1024 ctx150-450", 1024, lambda: rng.randint(150, 450)),  # a suggestions wave mid-decode
        ("B512 ctx150-200", 512, lambda: rng.randint(150, 200)),
        ("B256 ctx600-1400", 256, lambda: rng.randint(600, 1400)),
        ("B64 ctx1500-2000", 64, lambda: rng.randint(1500, 2000)),
        ("B8 ctx4000", 8, lambda: 4000)]
    for name, B, gen in cases:
        ctxs = [gen() for _ in range(B)]
        q, kc, vc, bt, cl = setup(B, ctxs, Hq, Hkv, D)
        kv_bytes = sum(ctxs) * Hkv * D * 2 * 2
        res = []
        outs = []
        maxb = bt.shape[1]
        auto = decode_variant(B, Hkv, D, maxb)
        for v in VARIANTS:
            bpp0, _ = ops.decode_partitioning(B, Hkv, maxb, variant=v, D=D)
            sweep = sorted({bpp0} | {max(4, -(-maxb // n)) for n in (1, 2, 4, 8, 16)})
            for bpp in sweep:
                mp = -(-maxb // bpp)
                ws = ops.DecodeWorkspace(B, Hq, D, mp, "cuda")
                out = torch.empty(B, Hq, D, device="cuda", dtype=torch.bfloat16)
                us = timeit(lambda: ops.paged_decode_attention(
                    q, kc, vc, bt, cl, D ** -0.5, out=out, blocks_per_part=bpp, workspace=ws,
                    variant=v))
                outs.append(out.float())
                tag = "*" if bpp == bpp0 else " "
                res.append(f"v{v}{tag}bpp{bpp:3d}/p{mp:2d} {us:7.1f}us {kv_bytes / us / 1e3:5.0f}GB/s")
        diff = max((o - outs[0]).abs().max().item() for o in outs)
        print(f"{name} Hq{Hq} Hkv{Hkv} D{D} (max diff {diff:.3g}; * = heuristic split; auto variant {auto})",
              flush=True)
        for r in res:
            print("    " + r, flush=True)


if __name__ == "__main__":
    main()
