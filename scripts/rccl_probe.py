#!/usr/bin/env python3
"""Probe: can two ranks share one GPU over the nccl (RCCL) backend?  send/recv + all_reduce."""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1 << 20,), float(rank + 1), device="cuda:0")
if rank == 0:
    dist.send(x, 1)
else:
    y = torch.empty_like(x)
    dist.recv(y, 0)
    print("recv ok", float(y[0]), flush=True)
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {rank} allreduce {float(x[0])}", flush=True)
dist.barrier()
dist.destroy_process_group()
