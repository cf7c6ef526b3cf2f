"""Can two RCCL ranks share one GPU here? torchrun --nproc-per-node 2 tools/nccl2_probe.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.arange(8, dtype=torch.int64, device="cuda") + 100 * rank
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
torch.cuda.synchronize()
print(rank, y.tolist(), flush=True)
dist.destroy_process_group()
