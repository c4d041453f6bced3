"""Probe: can two ranks share one GPU under RCCL (torch nccl backend)?"""
import os, torch, torch.distributed as dist
r = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl")
x = torch.full((1 << 20,), float(r + 1), device="cuda:0", dtype=torch.float64)
dist.all_reduce(x)
dist.broadcast(x, 1)
torch.cuda.synchronize()
print("rank", r, "ok", x[0].item(), flush=True)
dist.destroy_process_group()
