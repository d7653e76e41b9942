"""Probe: can two ranks share one GPU under the nccl (RCCL) backend?"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), rank + 1, dtype=torch.int64, device="cuda")
out = torch.zeros(8, dtype=torch.int64, device="cuda")
dist.all_gather_into_tensor(out, x)
y = torch.arange(4, dtype=torch.int64, device="cuda") + 10 * rank
z = torch.zeros(4, dtype=torch.int64, device="cuda")
dist.all_to_all_single(z, y, [2, 2], [1, 3] if rank == 0 else [3, 1])
torch.cuda.synchronize()
print(rank, out.tolist(), z.tolist(), flush=True)
dist.destroy_process_group()
