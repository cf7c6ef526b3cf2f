"""C4 duplicate-insert hunt: generator validity at 1B (one CAS table) and the sharded path at
several sizes / chunkings."""
import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
import cs267_hw3_amd as kh
from cs267_hw3_amd.dist import run_threaded

def gen(n):
    return kh.SyntheticKmers(51, n, 8, 200, 0, seed=51)

def sharded(n, P, chunks=None):
    g = gen(n)
    info = {}
    t = time.time()
    try:
        run_threaded(51, g, P, info=info, insert_chunks=chunks, check=lambda r, x: None)
        print(f"sharded n={n} P={P} chunks={chunks}: ok {time.time()-t:.1f}s", flush=True)
    except Exception as ex:
        print(f"sharded n={n} P={P} chunks={chunks}: FAIL {ex}", flush=True)

mode = sys.argv[1]
if mode == "gen1b":
    n = 1_000_000_000
    g = gen(n)
    os.environ["KH_INSERT"] = "cas"
    with kh.KmerHashTable(51, n) as t:
        recs = g.records_dev()
        t.insert_dev(recs.data_ptr(), n)
        try:
            t.sync(); print("gen1b: no duplicates", flush=True)
        except Exception as ex:
            print("gen1b:", ex, flush=True)
else:
    for n, P, ch in [(200_000_000, 8, None), (400_000_000, 8, None), (1_000_000_000, 8, 1), (1_000_000_000, 8, None)]:
        sharded(n, P, ch)
