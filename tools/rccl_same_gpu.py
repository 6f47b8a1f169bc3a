"""Rehearsal: can two ranks share one GPU over RCCL (the nccl backend)?  Each rank runs
an all_reduce of a small tensor on cuda:0.  Launched with torch.distributed.run
--nproc-per-node 2; prints the result per rank or the error.
"""
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.full((1024,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize(dev)
    print(f"rank {rank}: all_reduce -> {x[0].item()} (expect 3.0)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
