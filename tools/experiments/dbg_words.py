import sys, time, torch
sys.path.insert(0, ".")
import cs267_hw3_amd as kh
from cs267_hw3_amd.dist import GpuShard
n = int(sys.argv[1])
g = kh.SyntheticKmers(51, n, 8, 200, 0, seed=51)
host = g.records()
for mode_n in [n]:
    sh = GpuShard(51, int(n * 1.02) + 4096)
    with torch.cuda.stream(sh.stream):
        recs = torch.from_numpy(host).cuda()
        words, counts = sh.route(recs, 1)
        sh.sync()
        print("counts", counts[:2].tolist(), flush=True)
        w2 = words.clone()
        sh.insert_words(w2, n)
        try:
            sh.sync()
        except Exception as e:
            print("ERR", e)
        s = sh.stats(); print("direct words:", s["n_dup"], s["n_inserted"], flush=True)
        # check words vs records-derived words: route via records path on a fresh table
        t2 = kh.KmerHashTable(51, int(n*1.02)+4096)
        t2.insert_dev(recs.data_ptr(), n); 
        try:
            t2.sync(); print("records path ok", t2.stats()["n_dup"])
        except Exception as e:
            print("records ERR", e)
        # compare multiset of words vs a sorted view? check uniqueness of w (hi,lo)
        w = words[: 2 * n].view(-1, 2)
        key = (w[:, 0] >> 6) * 1000003 + w[:, 1]
        print("unique keys in routed words:", torch.unique(w[:, 1]).numel(), "of", n, flush=True)
