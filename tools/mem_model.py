"""Per-rank peak device allocation of the sharded path (dist.py + libkmerhash_amd), from the
sizing formulas in the code (kh_capi.cpp ensure() calls, dist.py _grow() calls, kh_build.hip
part_* capacities). Used for DESIGN.md §6's C5-at-1B model; no GPU needed.

  python tools/mem_model.py [--P 8] [--n 1e9] [--workload c5|c3] [--ranks-per-gpu 1]
"""
import argparse
import math

GB = 1e9


def model(P, n_total, contigs, starts_rank0, load=0.5, k_words=2, rec=15, splitter_frac=1 / 256,
          long_walkers=0, route_windows=True):
    n = math.ceil(n_total / P)                       # records per rank (block split)
    W8 = 8 * k_words                                  # bytes per partition word / slot
    walkers = contigs + n_total * splitter_frac       # every rank's walkers (starts + splitters)
    out = {}
    # ---- insert (per rank; every rank receives ~n words) ----
    out["records (rank's block)"] = n * rec
    out["route windows (P x n words)" if route_windows else "route (n words)"] = (P if route_windows else 1.25) * n * W8
    out["received words"] = 1.25 * n * W8
    cap = (n * 1.02 + 4096) / load
    out["table slots"] = cap * W8
    nreg = 2 ** 17
    mu = n / nreg
    rc = mu + 7 * math.sqrt(30 * mu) + 16
    mu1 = n / 4096
    cap1 = mu1 + 10 * math.sqrt(mu1 * (1 + 30 / 8)) + 64
    out["partition buf1 + buf2 + overflow list"] = (max(4096 * cap1, n) + max(nreg * rc, n) + n + 65536) * W8
    out["chain head records"] = (cap / nreg / 8 + 32) * nreg * 16
    # ---- walk: worst case = rank 0 (holds every start k-mer under C5's front_starts order) ----
    nseg0 = starts_rank0 + n * splitter_frac
    out["walker init messages (rank's starts)"] = nseg0 * 40
    out["text store (n/32 + 4 per walker of every rank) x2"] = 2 * (n / 32 + 4 * walkers) * 16
    out["grouped text records (= store bound, x1.25)"] = 1.25 * 2 * (n / 32 + 4 * walkers) * 16
    out["held-back messages (2 x every walker)"] = 2 * walkers * 41
    out["round inputs / outputs (first round: rank's walkers)"] = nseg0 * 41
    cap_slot = walkers / P / P * 1.25 + 1024
    out["exchange slots (4 x P x cap, x1.25)"] = 4 * 1.25 * P * (2 + 5 * cap_slot) * 8
    recv_text = n_total / 32 + 2 * walkers if starts_rank0 >= contigs else n / 32 + 2 * walkers / P
    out["received text records (origin, x1.25)"] = 1.25 * recv_text * 16
    out["segment retag records out + in (x1.25)"] = 2 * 1.25 * (recv_text + nseg0) * 24
    text = (n_total if starts_rank0 >= contigs else n) + (starts_rank0 if starts_rank0 else contigs / P) * 51
    out["contig text (sized: 52 per contig + 32 per word record)"] = (
        (starts_rank0 or contigs / P) * 52 + 32 * recv_text)
    return out, text


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--workload", default="c5", choices=["c5", "c3"])
    ap.add_argument("--ranks-per-gpu", type=int, default=1)
    a = ap.parse_args()
    n = int(a.n)
    if a.workload == "c5":  # contigs U[2,16] (mean 9) + 8 chains of 10^6, every start first
        contigs = (n - 8 * 10**6) / 9 + 8
        starts0 = min(contigs, math.ceil(n / a.P))
    else:                   # C3 shape: contigs U[8,200] (mean 104), shuffled
        contigs = n / 104
        starts0 = contigs / a.P
    out, text = model(a.P, n, contigs, starts0)
    tot = sum(out.values())
    print(f"workload {a.workload}, n = {n:.3g}, P = {a.P}: per-rank peak of rank 0 (the start-holding rank)")
    for k, v in out.items():
        print(f"  {k:58s} {v / GB:7.2f} GB")
    print(f"  {'total':58s} {tot / GB:7.2f} GB  (MI355X: 288 GB; {a.ranks_per_gpu} rank(s) per GPU -> "
          f"{'fits' if tot * a.ranks_per_gpu < 288 * GB else 'does NOT fit'} at this rank's size)")


if __name__ == "__main__":
    main()
