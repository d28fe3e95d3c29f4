"""Rehearsal of bench.py's N > 1 collectives (RCCL init bound to a device, barrier, float64 MAX
all-reduce, destroy) with every rank on cuda:0 -- the one-GPU box's only device.  Launch:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 scripts/rccl_two_ranks.py
Prints one line per rank, or RCCL's error (NCCL/RCCL refuse two ranks on one device by default)."""
import os
import time

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
t0 = time.perf_counter()
dist.init_process_group("nccl", device_id=dev)
dist.barrier()
tt = torch.tensor([float(rank + 1)], device=dev, dtype=torch.float64)
dist.all_reduce(tt, op=dist.ReduceOp.MAX)
torch.cuda.synchronize()
print(f"rank {rank}/{dist.get_world_size()}: all_reduce MAX = {tt.item()} "
      f"({time.perf_counter() - t0:.2f} s incl. init)", flush=True)
dist.barrier()
dist.destroy_process_group()
