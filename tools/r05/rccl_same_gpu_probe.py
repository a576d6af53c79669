"""Probe: can two RCCL ranks share one GPU on this pool's one-GPU boxes?  Run under
torch.distributed.run --nproc-per-node 2 (127.0.0.1).  Prints each rank's all-reduce and
all-gather results, or the error RCCL raises."""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((4,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    g = torch.empty(world * 2, device="cuda")
    dist.all_gather_into_tensor(g, torch.full((2,), float(rank), device="cuda"))
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce {x.tolist()} all_gather {g.tolist()}", flush=True)
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001 -- the probe reports whatever RCCL says
    print(f"rank {rank}: {type(e).__name__}: {e}", flush=True)
    sys.exit(3)
