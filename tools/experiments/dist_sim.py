"""Rounds and shard balance of the sharded walk with P logical ranks on one GPU (ThreadComm):
python tools/dist_sim.py [k] [n_total] [P] [protocol] [len_min] [len_max]"""
import sys
import time

sys.path.insert(0, ".")
import cs267_hw3_amd as kh  # noqa: E402
from cs267_hw3_amd.dist import run_threaded  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 51
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
P = int(sys.argv[3]) if len(sys.argv) > 3 else 8
proto = sys.argv[4] if len(sys.argv) > 4 else "migrate"
lmin = int(sys.argv[5]) if len(sys.argv) > 5 else 8
lmax = int(sys.argv[6]) if len(sys.argv) > 6 else 200
g = kh.SyntheticKmers(k, n, lmin, lmax, 0, seed=7)
recs = g.records()
info = {}
t = time.time()
texts = run_threaded(k, recs, P, protocol=proto, info=info)
dt = time.time() - t
ok = all(texts[r] == g.truth(*g.block(P, r)) for r in range(P))
ins = [info["stats"][r]["n_inserted"] for r in range(P)]
print(f"k={k} n={n} P={P} {proto}: rounds={info['rounds']} ok={ok} wall={dt:.2f}s "
      f"shard sizes min/max={min(ins)}/{max(ins)} (imbalance {max(ins) * P / n:.4f})")
