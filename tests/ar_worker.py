"""Worker for test_custom_allreduce_gpu.py: one rank of a custom all-reduce
group on device rank % device_count().  On a one-GPU box every rank shares
cuda:0 (the IPC handle exchange, flag protocol and reduction are the same code
path as across the GPUs of an xGMI hive); on a box with >= world GPUs each rank
owns its own device, the peer mapping crosses xGMI (hipDeviceCanAccessPeer is
asserted) and the custom sums are also checked against RCCL's all-reduce."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drtc_amd.parallel.custom_allreduce import CustomAllReduce  # noqa: E402


def data(rank, it, n):
    g = torch.Generator().manual_seed(rank * 7919 + it)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def expected(world, it, n):
    acc = torch.zeros(n, dtype=torch.float32)
    for q in range(world):
        acc += data(q, it, n).float()
    return acc.to(torch.bfloat16)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ndev = torch.cuda.device_count()
    dev = rank % ndev
    torch.cuda.set_device(dev)
    distinct = ndev >= world
    if distinct:  # one device per rank: every peer must be reachable over xGMI
        for q in range(world):
            if q != dev:
                assert torch.cuda.can_device_access_peer(dev, q), f"no P2P {dev}->{q}"
    car = CustomAllReduce(dist.group.WORLD, torch.device("cuda", dev), max_bytes=4 << 20)
    it = 0
    for n in (8, 4096, 8 * 1001, 8 * 12345, 1 << 20, 2 << 20):
        for mode in (None, False, True):  # by size / one-shot / two-shot, interleaved
            for _ in range(3):  # consecutive calls alternate the staging halves
                x = data(rank, it, n).cuda()
                y = car.all_reduce(x, two_shot=mode)
                torch.cuda.synchronize()
                if not torch.equal(y.cpu(), expected(world, it, n)):
                    print(f"rank {rank}: mismatch n={n} mode={mode} it={it}", flush=True)
                    sys.exit(3)
                it += 1
    # hipGraph capture + replay with fresh inputs
    n = 4096 * 8
    static = torch.zeros(n, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        car.all_reduce(static)  # warm-up on the capture stream
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        car.all_reduce(static, two_shot=False)
        car.all_reduce(static, two_shot=True)  # the sum, summed again: world * sum
    for _ in range(3):
        static.copy_(data(rank, it, n).cuda())
        gr.replay()
        torch.cuda.synchronize()
        want = (expected(world, it, n).float() * world).to(torch.bfloat16)
        if not torch.equal(static.cpu(), want):
            print(f"rank {rank}: graph mismatch it={it}", flush=True)
            sys.exit(4)
        it += 1
    # fused all-reduce + residual add + RMSNorm (decode sublayer epilogue); H = 5120 does not
    # divide a block's staging chunk, and plain calls interleave with the fused ones
    for rows, H, gemma in ((1, 4096, False), (7, 8192, True), (64, 2048, False),
                           (37, 5120, False), (5, 3072, True), (64, 5120, False)):
        xp = data(rank, it + 500, 8 * 12345).cuda()
        yp = car.all_reduce(xp)
        part = data(rank, it, rows * H).view(rows, H).cuda()
        res0 = data(99, it, rows * H).view(rows, H)
        w = (data(98, it, H) * 0.1 + 1.0).to(torch.bfloat16)
        res = res0.cuda()
        y = car.all_reduce_rmsnorm(part, res, w.cuda(), 1e-5, gemma)
        torch.cuda.synchronize()
        o = expected(world, it, rows * H).view(rows, H).float()
        h = (o + res0.float()).to(torch.bfloat16)
        ww = w.float() + (1.0 if gemma else 0.0)
        ref = (h.float() * torch.rsqrt(h.float().pow(2).mean(-1, keepdim=True) + 1e-5) * ww)
        if not torch.equal(res.cpu(), h):
            print(f"rank {rank}: fused residual mismatch rows={rows}", flush=True)
            sys.exit(6)
        if (y.cpu().float() - ref).abs().max().item() > 0.02 * ref.abs().max().item():
            print(f"rank {rank}: fused norm mismatch rows={rows} H={H}", flush=True)
            sys.exit(7)
        if not torch.equal(yp.cpu(), expected(world, it + 500, 8 * 12345)):
            print(f"rank {rank}: plain all-reduce beside the fused one H={H}", flush=True)
            sys.exit(11)
        ys = [torch.empty_like(y.cpu()) for _ in range(world)]
        dist.all_gather(ys, y.cpu())
        if not all(torch.equal(ys[0], t) for t in ys):
            print(f"rank {rank}: fused norm differs across ranks", flush=True)
            sys.exit(8)
        it += 1
    # back-to-back calls of different sizes and kinds, no host sync in between
    # (fixed per-block partition: parity reuse stays safe across sizes)
    outs, wants = [], []
    for k, n in enumerate((8 * 1001, 1 << 20, 64, 8 * 12345, 4096, 2 << 20, 8 * 3)):
        x = data(rank, it, n).cuda()
        outs.append(car.all_reduce(x, two_shot=(k % 3 == 1) and world > 2))
        wants.append(expected(world, it, n))
        it += 1
    torch.cuda.synchronize()
    for y, want in zip(outs, wants):
        if not torch.equal(y.cpu(), want):
            print(f"rank {rank}: mismatch in the unsynchronised mixed-size sequence", flush=True)
            sys.exit(9)
    # epochs far past the 32-bit range (64-bit counters and flags)
    dist.barrier()
    torch.cuda.synchronize()
    for start in ((1 << 31) - 3, (1 << 32) - 2):
        dist.barrier()
        from drtc_amd.ops._ext import hipk
        assert hipk().ar_set_epoch(car.base, start) == 0
        dist.barrier()
        for _ in range(5):
            x = data(rank, it, 4096).cuda()
            y = car.all_reduce(x)
            torch.cuda.synchronize()
            if not torch.equal(y.cpu(), expected(world, it, 4096)):
                print(f"rank {rank}: mismatch after epoch {start}", flush=True)
                sys.exit(10)
            it += 1
    if distinct:  # RCCL over the same devices: same sums to bf16 rounding of its own order
        grp = dist.new_group(backend="nccl")
        for n in (4096, 1 << 20):
            x = data(rank, it, n).cuda()
            y = car.all_reduce(x.clone())
            dist.all_reduce(x, group=grp)
            torch.cuda.synchronize()
            want = expected(world, it, n)
            if not torch.equal(y.cpu(), want):
                print(f"rank {rank}: custom mismatch on distinct devices n={n}", flush=True)
                sys.exit(12)
            tol = 0.02 * want.float().abs().max().item()
            if (x.cpu().float() - want.float()).abs().max().item() > tol:
                print(f"rank {rank}: RCCL and the reference disagree n={n}", flush=True)
                sys.exit(13)
            it += 1
    if car.error():
        print(f"rank {rank}: flag wait timed out", flush=True)
        sys.exit(5)
    dist.barrier()
    car.close()
    dist.destroy_process_group()
    print(f"rank {rank}: OK", flush=True)


if __name__ == "__main__":
    main()
