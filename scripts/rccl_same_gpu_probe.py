"""Rehearsal probe (not part of the product): can two RCCL ranks share the one GPU of a test box?  Each rank binds
device 0, all-reduces a tensor and barriers.  Run: python -m torch.distributed.run --nproc-per-node 2 --master-addr
127.0.0.1 --master-port 29533 scripts/rccl_same_gpu_probe.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
t = torch.tensor([float(rank + 1)], device="cuda:0")
dist.all_reduce(t)
dist.barrier()
print(f"rank {rank}: all_reduce -> {t.item()}", flush=True)
dist.destroy_process_group()
