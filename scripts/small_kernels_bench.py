#!/usr/bin/env python3
"""Decode-step small kernels at Llama-3-8B batch 1024: RoPE + paged KV write
(with / without the dim-major V scatter), RMSNorm(+residual), SiLU-GLU.
Prints us per call and effective GB/s."""
import sys

import torch

sys.path.insert(0, ".")
from drtc_amd import ops  # noqa: E402


def timeit(fn, iters=100):
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


def main():
    B, Hq, Hkv, D, H, I = 1024, 32, 8, 128, 4096, 14336
    dev = "cuda"
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
    cs = ops.build_rope_cache(8192, D, 500000.0, None, device=dev)
    pos = torch.randint(0, 2000, (B,), dtype=torch.int32, device=dev)
    nb = 8192
    kc = torch.zeros(nb, Hkv, 32, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(nb, Hkv, D, 32, device=dev, dtype=torch.bfloat16)
    slots = (torch.randperm(nb - 1, device=dev)[:B] + 1).to(torch.int64) * 32 + \
        torch.randint(0, 32, (B,), device=dev)
    byts = qkv.numel() * 2 * 2 + B * Hkv * D * 2 * 2
    from drtc_amd.ops._ext import hipk
    for variant in (1, 2):  # 1 = 256-thread loop, 2 = one item per thread (default)
        hipk().set_rope_variant(variant)
        for wv in (True, False):
            us = timeit(lambda: ops.rope_kv_(qkv, pos, slots, cs, Hq, Hkv, D, kc, vc, 32, write_v=wv))
            print(f"rope_kv v{variant} B={B} write_v={wv}: {us:7.1f} us  {byts / us / 1e3:6.0f} GB/s",
                  flush=True)
    hipk().set_rope_variant(2)
    x = torch.randn(B, H, device=dev).to(torch.bfloat16)
    r = torch.randn(B, H, device=dev).to(torch.bfloat16)
    w = torch.ones(H, device=dev, dtype=torch.bfloat16)
    us = timeit(lambda: ops.rmsnorm(x, w, 1e-5, False, residual=r))
    print(f"rmsnorm+res B={B}: {us:7.1f} us  {4 * x.numel() * 2 / us / 1e3:6.0f} GB/s", flush=True)
    gu = torch.randn(B, 2 * I, device=dev).to(torch.bfloat16)
    us = timeit(lambda: ops.act_glu(gu, "silu"))
    print(f"act_glu B={B}: {us:7.1f} us  {3 * B * I * 2 / us / 1e3:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
