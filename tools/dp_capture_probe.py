"""Probe: RCCL all-reduce inside a captured HIP graph (torchrun --nproc-per-node N, every rank on its own GPU, or all
on cuda:0 where RCCL allows it).  Prints per rank: eager result, replayed-graph results."""
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", dev))
    x = torch.full((1 << 16,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {rank}: eager {x[0].item()} (want {world * (world + 1) / 2})", flush=True)
    y = torch.zeros(1 << 16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        y.fill_(rank + 1)
        dist.all_reduce(y)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        y.fill_(rank + 1)
        dist.all_reduce(y)
        y.mul_(2)
    for i in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(f"rank {rank}: graph {y[0].item()} (want {world * (world + 1)})", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
