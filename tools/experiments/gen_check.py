"""Device vs host generator at C4 size (sample ranges)."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import cs267_hw3_amd as kh
for n in (200_000_000, 1_000_000_000):
    g = kh.SyntheticKmers(51, n, 8, 200, 0, seed=51)
    full = g.records_dev()
    torch.cuda.synchronize()
    for b in (0, n // 3 + 7, n // 2, n - 1_000_000):
        e = min(n, b + 1_000_000)
        h = g.records(b, e)
        d1 = full[b:e].cpu().numpy()
        d2 = g.records_dev(b, e).cpu().numpy()
        print(n, b, "full==host", np.array_equal(d1, h), "range==host", np.array_equal(d2, h),
              "zero rows", int((d1 == 0).all(1).sum()), flush=True)
    del full
    torch.cuda.empty_cache()
