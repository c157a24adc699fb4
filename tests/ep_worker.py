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
from drtc_amd.parallel.expert_parallel import ep_moe_forward  # noqa: E402


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
    ref = ops.fused_moe_ref(x_all, torch.nn.functional.linear(x_all, router), gu, dn, k)
    ref = ref[rank * T:(rank + 1) * T].float()
    for static in (False, True):
        y = ep_moe_forward(x, router, gu[rank * el:(rank + 1) * el].contiguous(),
                           dn[rank * el:(rank + 1) * el].contiguous(), k, static=static)
        torch.cuda.synchronize()
        err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
        if not err < 2e-2:
            print(f"rank {rank}: static={static} rel err {err}", flush=True)
            sys.exit(3)
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank}: OK", flush=True)


if __name__ == "__main__":
    main()
