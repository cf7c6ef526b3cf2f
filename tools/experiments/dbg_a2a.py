"""Check torch.distributed all_to_all_single (RCCL) on large single-peer messages."""
import os
import torch
import torch.distributed as dist
local = int(os.environ.get("LOCAL_RANK", 0))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
for gb in [0.5, 1.0, 2.0, 2.2, 3.2]:
    n = int(gb * 2**30 / 8)
    x = torch.arange(n, dtype=torch.int64, device="cuda")
    y = torch.empty_like(x)
    dist.all_to_all_single(y, x, [n], [n])
    torch.cuda.synchronize()
    bad = (y != x).sum().item()
    print(f"{gb} GiB ({n} int64): mismatches {bad}", flush=True)
dist.destroy_process_group()
