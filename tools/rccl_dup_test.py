"""Can two RCCL ranks share one GPU on this box? (rehearsal feasibility; prints the outcome)"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((1024,), float(rank + 1), device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce ok, x[0]={x[0].item()}", flush=True)
dist.destroy_process_group()
