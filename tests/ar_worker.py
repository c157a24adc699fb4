"""Worker for test_custom_allreduce_gpu.py: one rank of a custom all-reduce
group.  Every rank runs on cuda:0 (the test box has one GPU) - the IPC
handle exchange, flag protocol and reduction are the same code path as
across the GPUs of an xGMI hive."""
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
    torch.cuda.set_device(0)
    car = CustomAllReduce(dist.group.WORLD, torch.device("cuda", 0), max_bytes=4 << 20)
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
    if car.error():
        print(f"rank {rank}: flag wait timed out", flush=True)
        sys.exit(5)
    dist.barrier()
    car.close()
    dist.destroy_process_group()
    print(f"rank {rank}: OK", flush=True)


if __name__ == "__main__":
    main()
