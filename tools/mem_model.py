"""Per-rank device memory of the sharded path (dist.py + libkmerhash_amd), from the sizing formulas
in the code: the library's buffers (kh_capi.cpp ensure() calls, kh_build.hip part_* capacities)
and the Python host's torch buffers (dist.py _grow() calls). Checked against what a step really
allocates (kh_device_bytes + torch's allocator) by tests/test_gpu_configs.py::test_mem_model_*;
then used for the C5-at-1B sizing of DESIGN.md §6. No GPU needed:

  python tools/mem_model.py [--P 8] [--n 1e9] [--workload c5|c3]

rank_model() takes the counts a rank sees (records in its block, k-mers it holds, its start and
splitter k-mers, every rank's walkers); workload_ranks() derives them from a BASELINE workload.
"""
import argparse
import math

GB = 1e9
W8 = 16            # bytes per k-mer word / slot at k = 51 (W = 2)
REGION_BITS = 17   # 2^17 placement regions at C3 sizes and above
NW1 = 512 * 8      # pass-1 windows
MSG = 40           # migrating-walker message
REC = 16           # text record
REC_SLOTS = 12     # text records a walker may stage per round (MW_RUN_WORDS + 4)
SLACK = 1.25       # dist.py _grow


def _cap(n_table, load=0.5):
    return math.ceil(n_table / load)


def _split_bits(n_table):
    bits = 1
    while bits < 12 and (n_table >> (20 + bits)) != 0:
        bits += 1
    return max(bits, 4)


def rank_model(P, n_rec, n_ins, n_table, ns, nsp, walkers_all, K=51, routed=True, windows=True,
               text_recs=None, recv_text=None, recv_seg=None, exchange=None, load=0.5, ns_max=None,
               cap_slot=None):
    """Bytes per item {name: (bytes, 'lib'|'torch')} of one rank after a step. n_rec: records in
    its block; n_ins: k-mers in its shard; n_table: the shard's sizing (kh_create / kh_reserve);
    ns / nsp: its start k-mers / the splitters it owns; walkers_all: starts + splitters of all
    ranks; text_recs: text records its walkers stored (default: the bound's estimate); recv_text /
    recv_seg: text / retag records it receives as an origin; ns_max: the largest rank's start
    k-mers (its first round sends them out: the exchange slots are sized by the largest
    per-destination count seen, cap_slot when known)."""
    exchange = (P > 1) if exchange is None else exchange
    out = {}
    cap = _cap(n_table, load)
    R = (K + 3) // 4 + 2
    # ---- records and the route (torch) ----
    out["records (rank's block)"] = (n_rec * R + 16, "torch")
    if routed:
        words = (P * n_rec if windows else n_rec) * W8
        out["routed words (owner windows)" if windows else "routed words"] = (words * (1.0 if windows else SLACK), "torch")
        if exchange:
            out["received words"] = (SLACK * n_ins * W8, "torch")
    # ---- table, partition, chains (library) ----
    out["table slots"] = (cap * W8, "lib")
    nreg = 2 ** REGION_BITS
    mu = n_ins / nreg
    rc = int(mu + 7 * math.sqrt(30 * mu) + 16)
    mu1 = n_ins / NW1
    cap1 = int(mu1 + 10 * math.sqrt(mu1 * (1 + 30 / 8)) + 64)
    out["partition: pass-1 windows"] = (max(NW1 * cap1, n_ins) * W8, "lib")
    out["partition: region windows"] = (max(nreg * rc, n_ins) * W8, "lib")
    out["partition: overflow list"] = ((n_ins + 65536) * W8, "lib")
    hcap = (cap // nreg + 1) // 8 + 32
    out["chain head records"] = (hcap * nreg * 16 + nreg * 4, "lib")
    sb = _split_bits(n_table)
    # the route (and the records pass) reserve a start-list entry for every record of the block
    out["start list"] = (max(1024, n_rec) * W8, "lib")
    out["splitter list"] = (max(1024, (n_table >> max(sb - 3, 0)) + 4096) * W8, "lib")
    out["masks, scans, route tables"] = (2 * (n_rec / 64 + 1) * 8 + 3 * (n_rec / 4096 + 1) * P * 8, "lib")
    # ---- migrating walk (library) ----
    nseg = ns + nsp
    wg = max(walkers_all, nseg)
    store_cap = 2 * (n_ins // 32 + 4 * wg) + 4096
    out["text store"] = (store_cap * REC, "lib")
    if cap_slot is None or cap_slot == 0:
        # the largest per-destination count of a round (+25 %): the busiest rank's first round
        # spreads its walkers over P owners; balanced inputs send walkers / P^2 per pair
        ns_max = ns if ns_max is None else ns_max
        busiest = max(ns_max + nsp, walkers_all / P) / P
        cap_slot = int(busiest * 5 / 4 + 256) if P > 1 else walkers_all + 16
    nb = min(wg, max(nseg, P * cap_slot))
    out["round buffers (messages, staged text, offsets)"] = ((nb + 1) * (2 * MSG + REC_SLOTS * REC + 8 + 2), "lib")
    out["held-back messages"] = (2 * (wg + 1) * (MSG + 1), "lib")
    if nsp or walkers_all > ns:
        cap2 = 64
        while cap2 < 2 * nsp + 64:
            cap2 <<= 1
        stride = nsp  # (the largest rank's count: ~ this one's)
        out["segment state + splitter table"] = ((nseg + 1) * 38 + cap2 * 20, "lib")
        out["pointer jumping buffers"] = ((P * stride + 1) * 34, "lib")
    # ---- the walk's exchange buffers (torch) ----
    sw = 2 + 5 * cap_slot
    out["exchange slots"] = ((2 if exchange else 1) * 2 * SLACK * P * sw * 8, "torch")
    out["grouped text records"] = (SLACK * store_cap * REC, "torch")
    if text_recs is None:
        text_recs = n_ins / 32 + 3 * nseg
    if recv_text is None:
        recv_text = text_recs
    if exchange:
        out["received text records"] = (SLACK * recv_text * REC, "torch")
    if nsp or walkers_all > ns:
        out["segment links"] = (SLACK * nseg * 32, "torch")
        out["retag records"] = (SLACK * (recv_text + nseg) * 24, "torch")
        if exchange:
            out["received retag records"] = (SLACK * (recv_seg if recv_seg is not None else recv_text) * 24, "torch")
        out["predecessor tables"] = (SLACK * (1 + (P if exchange else 0)) * max(nsp, 1) * 16, "torch")
    # ---- the origin's text (library) ----
    seg_recs = recv_seg if recv_seg is not None else 0
    out["contig text"] = (ns * (K + 1) + 32 * (recv_text + seg_recs) + 64, "lib")
    out["contig lengths, offsets, first chunks"] = ((ns + 1) * 12 + ns * 64, "lib")
    return out


def totals(items):
    lib = sum(v for v, k in items.values() if k == "lib")
    tor = sum(v for v, k in items.values() if k == "torch")
    return lib, tor


def workload_ranks(workload, n_total, P):
    """Per-rank model inputs of a BASELINE workload at P ranks (rank 0 first)."""
    n_rec = math.ceil(n_total / P)
    n_table = int(n_rec * 1.02) + 4096
    sb = _split_bits(n_table)
    nsp = n_rec / 2 ** sb                              # splitters each owner collects
    if workload == "c5":   # contigs U[2,16] (mean 9) + 8 chains of 10^6, every start first
        contigs = (n_total - 8 * 10**6) / 9 + 8
        ns = [min(max(contigs - r * n_rec, 0), n_rec) for r in range(P)]
    else:                  # C3 shape: contigs U[8,200] (mean 104), shuffled
        contigs = n_total / 104
        ns = [contigs / P] * P
    walkers_all = contigs + nsp * P
    ranks = []
    for r in range(P):
        # text records an origin receives: its contigs' bases / 32 + partial words and finish records
        kmers_home = ns[r] / contigs * n_total
        recv = kmers_home / 32 + 2 * ns[r] + nsp
        ranks.append(dict(P=P, n_rec=n_rec, n_ins=n_rec, n_table=n_table, ns=int(ns[r]), nsp=int(nsp),
                          walkers_all=int(walkers_all), recv_text=recv, recv_seg=recv / 2, ns_max=int(max(ns))))
    return ranks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--n", type=float, default=1e9)
    ap.add_argument("--workload", default="c5", choices=["c5", "c3"])
    a = ap.parse_args()
    n = int(a.n)
    ranks = workload_ranks(a.workload, n, a.P)
    items = rank_model(**ranks[0])
    lib, tor = totals(items)
    print(f"workload {a.workload}, n = {n:.3g}, P = {a.P}: device memory of rank 0 (the start-holding rank)")
    for k, (v, where) in items.items():
        print(f"  {k:52s} {where:5s} {v / GB:7.2f} GB")
    print(f"  {'total':52s}       {(lib + tor) / GB:7.2f} GB  (library {lib / GB:.2f}, torch {tor / GB:.2f}; "
          f"MI355X: 288 GB -> {'fits' if lib + tor < 288 * GB else 'does NOT fit'})")


if __name__ == "__main__":
    main()
