"""Where do duplicate inserts come from in the sharded insert at C3/C4 scale? Per-rank n_dup
after the insert only (no walk), several variants."""
import os
import sys
import threading
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

import cs267_hw3_amd as kh  # noqa: E402
from cs267_hw3_amd.dist import DistributedKmerHashMap, GpuShard, ThreadComm  # noqa: E402


def run(n, P, chunks=None, host=False, label="", sync_gen=False, pregen=False, mode=""):
    g = kh.SyntheticKmers(51, n, 8, 200, 0, seed=51)
    comms = ThreadComm.group(P)
    split = (n + P - 1) // P
    res = [None] * P
    hostrecs = g.records() if host else None
    pre = [None] * P
    if pregen:
        for r in range(P):
            b, e = min(r * split, n), min(r * split + split, n)
            pre[r] = g.records_dev(b, e, device=0)
        torch.cuda.synchronize()

    def body(r):
        try:
            torch.cuda.set_device(0)
            b, e = min(r * split, n), min(r * split + split, n)
            sh = GpuShard(51, max(n // P, 1), device=0)
            with torch.cuda.stream(sh.stream):
                if host:
                    mine = torch.from_numpy(np.ascontiguousarray(hostrecs[b:e])).to(sh.dev)
                elif pregen:
                    mine = pre[r]
                else:
                    mine = g.records_dev(b, e, device=0, stream=sh.stream)
                if sync_gen:
                    torch.cuda.synchronize()
                    comms[r].barrier()
                if mode == "streamsync":
                    sh.stream.synchronize()
                if mode == "barrier":
                    comms[r].barrier()
                dm = DistributedKmerHashMap(comms[r], sh)
                if chunks:
                    dm.INSERT_CHUNKS = chunks
                m = dm.insert_all(mine)
                torch.cuda.current_stream().synchronize()
                st = sh.stats()
                res[r] = (m, st["n_dup"], st["n_full"], st["n_inserted"], st["capacity"])
            sh.table.close()
        except BaseException as ex:
            res[r] = repr(ex)
            comms[r].sh.barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    t = time.time()
    for x in th:
        x.start()
    for x in th:
        x.join()
    print(f"{label} n={n} P={P} chunks={chunks} host={host} {time.time() - t:.1f}s:", res, flush=True)


which = sys.argv[1]
if which == "h":
    run(200_000_000, 8, label="E1streamsync", mode="streamsync")
    run(200_000_000, 8, label="E2barrier", mode="barrier")
    run(200_000_000, 8, label="E4chunks2", chunks=2)
    run(200_000_000, 8, label="E5chunks8", chunks=8)
    run(200_000_000, 8, label="A0again")
if which == "g":
    run(200_000_000, 8, label="A0")
    run(200_000_000, 8, label="A1sync", sync_gen=True)
    run(200_000_000, 8, label="A2pregen", pregen=True)
    run(100_000_000, 8, label="S100")
if which == "a":
    run(200_000_000, 8, label="A")
    run(200_000_000, 8, chunks=1, label="B")
    run(200_000_000, 4, label="E4")
    run(200_000_000, 2, label="E2")
    run(40_000_000, 8, label="S40")
    run(100_000_000, 8, label="S100")
elif which == "c":
    os.environ["KH_INSERT"] = "cas"
    run(200_000_000, 8, label="C")
elif which == "f":
    run(200_000_000, 8, host=True, label="F")
