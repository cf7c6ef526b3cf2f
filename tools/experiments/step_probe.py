"""Time the fixed-round kernels in isolation on one GPU (P=1, no communicator):
per-round step/find durations with events, then extra steps once every walker is done
(pure per-round overhead).  python tools/step_probe.py [n_kmers] [len_min] [len_max]"""
import sys
import time

import torch

sys.path.insert(0, ".")
import cs267_hw3_amd as kh  # noqa: E402
from cs267_hw3_amd import _lib  # noqa: E402
from cs267_hw3_amd.dist import GpuShard  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
lmin = int(sys.argv[2]) if len(sys.argv) > 2 else 8
lmax = int(sys.argv[3]) if len(sys.argv) > 3 else 12
k = 51
g = kh.SyntheticKmers(k, n, lmin, lmax, 0, seed=3)
sh = GpuShard(k, n)
S = _lib.SEG_SUBS
with torch.cuda.stream(sh.stream):
    recs = torch.from_numpy(g.records()).to(sh.dev)
    sh.collect_starts(recs)
    words, counts = sh.route(recs, 1)
    sh.insert_words(words, n)
    nw = sh.walk_begin(n)
    C = S * (-(-nw * 5 // (4 * S)) + 8)
    W = sh.W
    L = S + C * W
    send = torch.empty(L, dtype=torch.int64, device=sh.dev)
    reply = torch.empty(C, dtype=torch.uint8, device=sh.dev)
    sh.sync()

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record(sh.stream)
        return e

    prev = None
    st, fd = [], []
    for r in range(lmax + 2):
        a = ev()
        sh.step_fixed(1, C, prev, send)
        b = ev()
        sh.find_ext_fixed(1, C, send, reply)
        c = ev()
        prev = reply
        st.append((a, b))
        fd.append((b, c))
    sh.sync()
    print("walkers", nw, "C", C)
    print("step us", [round(a.elapsed_time(b) * 1e3, 1) for a, b in st])
    print("find us", [round(a.elapsed_time(b) * 1e3, 1) for a, b in fd])
    act = sh.active()
    print("active after", int(act.item()))
    ts = []
    for r in range(20):
        a = ev()
        sh.step_fixed(1, C, prev, send)
        b = ev()
        ts.append((a, b))
    sh.sync()
    print("idle step us", [round(a.elapsed_time(b) * 1e3, 1) for a, b in ts][2:])
    x = torch.empty(nw, dtype=torch.uint8, device=sh.dev)
    a = ev()
    for _ in range(10):
        x.add_(1)
    b = ev()
    sh.sync()
    print("torch add_ over walkers-bytes us", a.elapsed_time(b) * 1e3 / 10)
