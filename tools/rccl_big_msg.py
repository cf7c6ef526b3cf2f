"""One-rank reproducer for large per-peer messages through torch.distributed (RCCL), beside
tools/rccl_big_msg.cpp (RCCL called directly). DESIGN.md §6: the sharded insert splits every
per-peer message at KH_A2A_CHUNK_MB (512 MiB) since a one-rank self-exchange of 3.2 GB came back
corrupted; this pins the layer and the size at which it happens.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29561 tools/rccl_big_msg.py [GiB ...]

For each size: all_to_all_single (equal split), all_to_all_single with explicit split lists, and
the list form all_to_all (grouped send/recv from views), each checked element by element.
One JSON line per (size, call)."""
import json
import sys
import time

import torch
import torch.distributed as dist


def main():
    sizes = [float(x) for x in sys.argv[1:]] or [1.0, 2.0 - 8 / 2**30, 2.0, 2.0 + 8 / 2**30, 3.2]
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    torch.cuda.set_device(0)
    nccl = ".".join(map(str, torch.cuda.nccl.version()))
    maxw = max(int(g * 2**30) // 8 for g in sizes)
    src = torch.empty(maxw, dtype=torch.int64, device="cuda")
    dst = torch.empty(maxw, dtype=torch.int64, device="cuda")
    mult = -7046029254386353131  # 0x9E3779B97F4A7C15 as int64
    for g in sizes:
        n = int(g * 2**30) // 8
        a, b = src[:n], dst[:n]
        torch.arange(1, n + 1, dtype=torch.int64, device="cuda", out=a)
        a.mul_(mult)
        for call in ("all_to_all_single", "all_to_all_single_splits", "all_to_all_list"):
            b.zero_()
            torch.cuda.synchronize()
            t = time.perf_counter()
            if call == "all_to_all_single":
                dist.all_to_all_single(b, a)
            elif call == "all_to_all_single_splits":
                dist.all_to_all_single(b, a, [n], [n])
            else:
                dist.all_to_all([b], [a])
            torch.cuda.synchronize()
            ms = 1e3 * (time.perf_counter() - t)
            bad = (a != b).nonzero()
            nb = int(bad.numel())
            print(json.dumps({"layer": "torch.distributed " + call, "rccl_version": nccl, "bytes": n * 8,
                              "gib": n * 8 / 2**30, "bad_words": nb,
                              "first_bad": int(bad[0]) if nb else -1, "last_bad": int(bad[-1]) if nb else -1,
                              "ms": round(ms, 3)}), flush=True)
            del bad
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
