"""Probe: can two ranks share one GPU over RCCL (torch 'nccl' backend)?"""
import os
import torch
import torch.distributed as dist

dist.init_process_group("nccl")
r = dist.get_rank()
torch.cuda.set_device(0)
x = torch.full((4,), float(r + 1), device="cuda:0")
dist.all_reduce(x)
y = torch.empty(4, device="cuda:0")
ops = [dist.P2POp(dist.isend, x, 1 - r), dist.P2POp(dist.irecv, y, 1 - r)]
for q in dist.batch_isend_irecv(ops):
    q.wait()
torch.cuda.synchronize()
print("rank", r, "allreduce", x.tolist(), "p2p", y.tolist(), flush=True)
dist.destroy_process_group()
