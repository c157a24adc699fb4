"""Worker for test_expert_parallel_gpu.py: one rank of an EP group on device
rank % device_count() (on a one-GPU box every rank shares it; gloo: device
tensors are staged through host memory by parallel/comm.py).  Local experts run
on the fused HIP grouped-MFMA kernel."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtc_amd import ops  # noqa: E402
from drtc_amd.parallel.expert_parallel import (  # noqa: E402
    EpOverflow, ep_combine, ep_gather, ep_moe_forward, ep_plan)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(rank % torch.cuda.device_count())
    g = torch.Generator().manual_seed(11)
    E, H, I, k, T = 8, 256, 256, 2, 48
    router = (torch.randn(E, H, generator=g) * 0.2).to(torch.bfloat16).cuda()
    gu = (torch.randn(E, 2 * I, H, generator=g) * 0.05).to(torch.bfloat16).cuda()
    dn = (torch.randn(E, H, I, generator=g) * 0.05).to(torch.bfloat16).cuda()
    x_all = torch.randn(world * T, H, generator=g).to(torch.bfloat16).cuda()
    el = E // world
    x = x_all[rank * T:(rank + 1) * T].contiguous()
    # the reference routes on the logits each rank computes for its rows (ops.router_logits)
    def logits_by_rank(xa, t):
        return torch.cat([ops.router_logits(xa[r * t:(r + 1) * t].contiguous(), router)
                          for r in range(world)])

    ref = ops.fused_moe_ref(x_all, logits_by_rank(x_all, T), gu, dn, k)
    ref = ref[rank * T:(rank + 1) * T].float()
    gl, dl = gu[rank * el:(rank + 1) * el].contiguous(), dn[rank * el:(rank + 1) * el].contiguous()
    for form in ("exact", "static", "cap"):
        ovf = EpOverflow("cuda")
        y = ep_moe_forward(x, router, gl, dl, k, form=form, overflow=ovf)
        torch.cuda.synchronize()
        err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
        if not err < 2e-2 or int(ovf.count.item()) != 0:
            print(f"rank {rank}: form={form} rel err {err} overflow {ovf.count.item()}", flush=True)
            sys.exit(3)
    # HIP plan / gather / combine == their PyTorch references, bit for bit
    gen = torch.Generator().manual_seed(rank + 5)
    for T2, world2, e_loc, cap in ((48, 4, 2, 24), (4096, 8, 1, 1100), (777, 2, 4, 300)):
        topi = torch.stack([torch.randperm(world2 * e_loc, generator=gen)[:k] for _ in range(T2)])
        o_cpu = torch.zeros(1, dtype=torch.int32)
        o_gpu = torch.zeros(1, dtype=torch.int32, device="cuda")
        ref_plan = ep_plan(topi, e_loc, world2, cap, o_cpu)
        got_plan = ep_plan(topi.cuda(), e_loc, world2, cap, o_gpu)
        for a, b in zip(ref_plan, got_plan):
            if not torch.equal(a, b.cpu()):
                print(f"rank {rank}: ep_plan mismatch T={T2} cap={cap}", flush=True)
                sys.exit(4)
        if int(o_cpu) != int(o_gpu.item()):
            print(f"rank {rank}: ep_plan overflow {int(o_cpu)} vs {o_gpu.item()}", flush=True)
            sys.exit(5)
        xs = torch.randn(T2, 512, generator=gen).to(torch.bfloat16)
        sx_ref = ep_gather(xs, ref_plan[1], k)
        sx = ep_gather(xs.cuda(), got_plan[1], k).cpu()
        real = ref_plan[1] >= 0
        if not torch.equal(sx[real], sx_ref[real]):
            print(f"rank {rank}: ep_gather mismatch T={T2}", flush=True)
            sys.exit(6)
        w = torch.rand(T2, k, generator=gen)
        sx_ref[~real] = 0
        c_ref = ep_combine(sx_ref, ref_plan[0], w, T2, k).float()
        c = ep_combine(sx_ref.cuda(), got_plan[0], w.cuda(), T2, k).cpu().float()
        if (c - c_ref).abs().max().item() > 1e-2 * c_ref.abs().max().item():
            print(f"rank {rank}: ep_combine mismatch T={T2}", flush=True)
            sys.exit(7)
    # prefill-sized shard (T_r k = 8192 pairs, >4096 rows into the experts): the
    # capacity form runs without a host sync and matches the reference
    T3 = 4096
    x3_all = torch.randn(world * T3, H, generator=g).to(torch.bfloat16).cuda()
    ref3 = ops.fused_moe_ref(x3_all, logits_by_rank(x3_all, T3), gu, dn, k)
    ref3 = ref3[rank * T3:(rank + 1) * T3].float()
    ovf = EpOverflow("cuda")
    y3 = ep_moe_forward(x3_all[rank * T3:(rank + 1) * T3].contiguous(), router, gl, dl, k,
                        form="cap", overflow=ovf)
    ovf.reduce(None)
    torch.cuda.synchronize()
    if int(ovf.count.item()) == 0:
        err = (y3.float() - ref3).abs().max().item() / ref3.abs().max().item()
        if not err < 2e-2:
            print(f"rank {rank}: prefill-sized cap form rel err {err}", flush=True)
            sys.exit(8)
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: OK", flush=True)


if __name__ == "__main__":
    main()
