"""Probe: can two ranks on ONE GPU form an RCCL communicator (torch 'nccl' backend)?"""
import os
import torch
import torch.distributed as dist
r = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.full((4,), float(r + 1), device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {r}: all_reduce -> {t.tolist()}", flush=True)
dist.destroy_process_group()
