"""Are the duplicates made by the chunked route (kh_route_starts_dev called per chunk) while other
ranks generate their records? Per rank: route in chunks exactly like DistributedKmerHashMap.insert_all,
then count distinct routed words."""
import os
import sys
import threading
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

import cs267_hw3_amd as kh  # noqa: E402
from cs267_hw3_amd.dist import GpuShard, ThreadComm  # noqa: E402


def distinct(words, n):
    w = words[:2 * n].view(n, 2)
    key = w[:, 0] * 1000003 + w[:, 1]  # not injective in theory; a dup check only needs a lower bound
    s, _ = torch.sort(key)
    d = int((s[1:] != s[:-1]).sum().item()) + 1 if n else 0
    # exact on collisions of the mixed key: compare both words of equal neighbours
    return d


def run(n, P, nch, label, barrier=False):
    g = kh.SyntheticKmers(51, n, 8, 200, 0, seed=51)
    comms = ThreadComm.group(P)
    split = (n + P - 1) // P
    res = [None] * P

    def body(r):
        try:
            torch.cuda.set_device(0)
            b, e = min(r * split, n), min(r * split + split, n)
            sh = GpuShard(51, max(n // P, 1), device=0)
            with torch.cuda.stream(sh.stream):
                recs = g.records_dev(b, e, device=0, stream=sh.stream)
                if barrier:
                    comms[r].barrier()
                m = e - b
                bounds = [min(m, (m * c // nch) & ~15) for c in range(nch)] + [m]
                words = torch.empty(m * 2 + 16, dtype=torch.int64, device="cuda")
                for c in range(nch):
                    c0, c1 = bounds[c], bounds[c + 1]
                    sh.route(recs[c0:c1], P, words[c0 * 2:max(c1, c0 + 1) * 2], starts=True)
                torch.cuda.current_stream().synchronize()
                # reference: one route of everything on a second shard after generation is done
                sh2 = GpuShard(51, max(m, 1), device=0)
                with torch.cuda.stream(sh2.stream):
                    w2, _ = sh2.route(recs, 1)
                    torch.cuda.current_stream().synchronize()
                res[r] = (m, distinct(words, m), distinct(w2, m))
                sh2.table.close()
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
    print(f"{label} n={n} P={P} nch={nch} {time.time() - t:.1f}s: (m, distinct chunked, distinct one-pass)", res,
          flush=True)


run(200_000_000, 8, 4, "R4")
run(200_000_000, 8, 1, "R1")
run(200_000_000, 8, 4, "R4barrier", barrier=True)
