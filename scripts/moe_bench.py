#!/usr/bin/env python3
"""Micro-benchmark of the fused MoE layer (ops.fused_moe, HIP grouped GEMM)
against a hipBLASLt per-expert path, on Mixtral-8x7B shapes (H 4096,
I 14336, E 8, top-2).  Prints per T: ms, effective TFLOP/s and weight GB/s."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from drtc_amd import ops  # noqa: E402
from drtc_amd.ops import moe as moe_ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    H, I, E, k = 4096, int(sys.argv[1]) if len(sys.argv) > 1 else 14336, 8, 2
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    wgu = (torch.rand(E, 2 * I, H, device=dev, generator=g) * 2 - 1).to(torch.bfloat16) * 0.02
    wdn = (torch.rand(E, H, I, device=dev, generator=g) * 2 - 1).to(torch.bfloat16) * 0.02
    wbytes = (wgu.numel() + wdn.numel()) * 2
    ws = moe_ops.make_workspace(moe_ops.MOE_CHUNK, H, I, E, k, dev)  # + the GEMM workspace
    ts = [int(t) for t in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
        [64, 256, 512, 1024, 2048, 8192]
    for T in ts:
        x = (torch.rand(T, H, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        lg = torch.randn(T, E, device=dev, generator=g).to(torch.bfloat16)
        out = torch.empty_like(x)
        t_v = []
        for v in (0, 1, 2, 3, 4):
            t_v.append(timeit(lambda: ops.fused_moe(x, lg, wgu, wdn, k, workspace=ws, out=out,
                                                    variant=v)))
        # variant 3 with explicit gemm_xd forms (gate_up / down)
        forms = {}
        for gu, dn in ((1281, 1282), (281, 282), (281, 281), (241, 242), (141, 142), (1141, 1142)):
            try:
                forms[f"{gu}/{dn}"] = timeit(lambda: ops.fused_moe(
                    x, lg, wgu, wdn, k, workspace=ws, out=out, variant=3, gu_form=gu, dn_form=dn))
            except RuntimeError:
                pass
        # variant 4 (gemm_w4 grouped gate_up) with down on a 256-row gemm_xd grouped form
        for dn in (282, 1282, 281, 242):
            try:
                forms[f"v4/{dn}"] = timeit(lambda: ops.fused_moe(
                    x, lg, wgu, wdn, k, workspace=ws, out=out, variant=4, dn_form=dn))
            except RuntimeError:
                pass
        t_f = timeit(lambda: ops.fused_moe(x, lg, wgu, wdn, k, workspace=ws, out=out))
        topi, wts = moe_ops.route_ref(lg, k)

        def blaslt():
            o = torch.zeros(T, H, dtype=torch.float32, device=dev)
            for e in range(E):
                tok, slot = torch.nonzero(topi == e, as_tuple=True)
                h = ops.act_glu(F.linear(x.index_select(0, tok), wgu[e]))
                o.index_add_(0, tok, F.linear(h, wdn[e]).float() * wts[tok, slot].unsqueeze(1))
            return o
        t_b = timeit(blaslt, 5)
        flops = 2 * T * k * 3 * H * I
        vs = " ".join(f"v{v}:{flops / t / 1e9:6.0f}" for v, t in enumerate(t_v))
        vs += " | xd " + " ".join(f"{f}:{flops / t / 1e9:6.0f}" for f, t in forms.items())
        print(f"T={T:5d}  fused(auto) {t_f:7.3f} ms {flops / t_f / 1e9:7.1f} TF/s "
              f"{wbytes / t_f / 1e6:7.0f} GB/s [{vs} TF/s] | per-expert hipBLASLt {t_b:7.3f} ms "
              f"{flops / t_b / 1e9:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
