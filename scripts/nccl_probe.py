"""Probe: can two ranks share one GPU over the nccl (RCCL) backend on this box?"""
import os
import torch
import torch.distributed as dist

r = int(os.environ["RANK"]); ws = int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", int(os.environ["LOCAL_RANK"]) % torch.cuda.device_count())
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
t = torch.full((4,), float(r + 1), device=dev)
dist.all_reduce(t)
peer = (r + 1) % ws
a = torch.full((1024,), float(r), device=dev); b = torch.empty(1024, device=dev)
ops = [dist.P2POp(dist.isend, a, peer), dist.P2POp(dist.irecv, b, (r - 1) % ws)]
for q in dist.batch_isend_irecv(ops):
    q.wait()
torch.cuda.synchronize()
print(f"rank {r}: allreduce {t.tolist()} recv {b[0].item()}", flush=True)
dist.destroy_process_group()
