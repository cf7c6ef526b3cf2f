"""Benchmark: k-mer inserts+lookups/s (k=51) on MI355X — BASELINE.json metric.

One step = one full pass of the hot path over the synthetic dataset already resident in HBM:
clear the table, bulk-insert every record (+ start-node collection), walk every contig and
materialise the contig text (test_<rank>.dat bytes) in HBM. Inputs are generated on the host and
copied to HBM before timing; the D2H of the contigs is outside the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2] [--n N]
  N > 1: one rank per GPU; the table is sharded by a hash of each k-mer's minimizer, routed
         words and migrating walkers move with RCCL all-to-all (cs267_hw3_amd.dist); weak
         scaling (n k-mers per GPU). Under an outer torch.distributed.run the ranks are its
         processes; without one (no WORLD_SIZE) bench.py starts N ranks itself as a
         torch.distributed.run child before any GPU call. A world size other than --gpus fails.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # BASELINE.json configs[2]: k=51, 200M synthetic k-mers, single MI355X, table at 50% load
    "c3": dict(k=51, n=200_000_000, len_min=8, len_max=200, single=0, seed=51,
               desc="C3: k=51, 200M synthetic k-mers per GPU, contigs U[8,200] k-mers "
                    "(human-chr14-like mean 104), table load 0.5"),
    # BASELINE.json configs[1]: k=19, 10M synthetic k-mers
    "c2": dict(k=19, n=10_000_000, len_min=200, len_max=1374, single=0, seed=19,
               desc="C2: k=19, 10M synthetic k-mers per GPU, contigs U[200,1374] k-mers "
                    "(test.txt-like mean 787), table load 0.5"),
    # BASELINE.json configs[3]: k=51, 1B k-mers sharded across the GPUs (strong scaling: the
    # block split of read_kmers.hpp:55-58 over the ranks; at one rank the whole 1B on one GPU)
    "c4": dict(k=51, n=1_000_000_000, len_min=8, len_max=200, single=0, seed=5101, strong=True,
               desc="C4: k=51, 1B synthetic k-mers in all, block split over the GPUs, contigs U[8,200] "
                    "k-mers"),
    # BASELINE.json configs[4]: skewed set, 8 chains of 10^6 k-mers among
    # short contigs U[2,16], every start k-mer first in record order (the block split hands all
    # walkers to the first rank)
    "c5": dict(k=51, n=200_000_000, len_min=2, len_max=16, single=0, seed=5199,
               gen=dict(n_long=8, long_len=1_000_000, front_starts=True),
               desc="C5: k=51, 200M synthetic k-mers per GPU, 8 chains of 10^6 k-mers + contigs "
                    "U[2,16], start k-mers first in record order"),
    # BASELINE.json configs[4] hot-bucket half: 30% of the contigs carry one of 8 shared 16-mer
    # motifs in every k-mer (the motifs are their minimizers: 60M k-mers share 8 minimizer
    # windows, i.e. 8 placement regions / shard owners before the table remaps them)
    "c5h": dict(k=51, n=200_000_000, len_min=8, len_max=200, single=0, seed=5198,
                gen=dict(hot_permille=300, n_motifs=8),
                desc="C5 hot-bucket: k=51, 200M synthetic k-mers per GPU, contigs U[8,200], 30% of "
                     "them built around one of 8 shared minimizer motifs"),
    # the hot-bucket half's worst case for the remap: a fixed flank before every motif (the
    # families share the minimizer's neighbour window too: a 32-base repeat)
    "c5f": dict(k=51, n=200_000_000, len_min=8, len_max=200, single=0, seed=5197,
                gen=dict(hot_permille=300, n_motifs=8, hot_flank=True),
                desc="C5 hot-bucket, flank: as c5h, every motif preceded by a fixed 16-mer (families "
                     "share the minimizer and its neighbour window)"),
}
RANDOM_REQ_CEILING = 49e9
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
BEST_PUBLISHED_OPS = 72.6e6    # k=51, 4 nodes x 128 ranks (512 CPU ranks)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """Threads for the parallel CPU baseline: this process's CPU share (OMP_NUM_THREADS on the GPU
    box, else the affinity mask) — os.cpu_count() reports the whole machine there."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(avail, int(env))) if env and env.isdigit() else avail


def cpu_baseline(w, host_recs, truth, sample_n):
    """CPU restatements of the reference path on this host (oracle/, test infrastructure):
    (1) the thread-parallel DistributedHashMap restatement (oracle/kmer_oracle_par.c: threads =
        ranks, block split, owner-batched insert_all, each rank walks its own start nodes) on the
        FULL workload, all cores of this process's share -> `value`;
    (2) the serial stock-semantics oracle (oracle/kmer_oracle.c, 1 core) on a bounded sample of
        the same generator/config -> `serial`.
    Both time the reference's boundary (records packed in host memory -> contigs in host memory,
    kmer_hash.cpp:129-137), file I/O excluded."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_bind as ob
    import cs267_hw3_amd as kh
    k, n = w["k"], len(host_recs)
    P = host_threads()
    rc, text, nc, nl, ti, tw = ob.assemble_par(k, host_recs, P)
    if rc != 0:
        raise RuntimeError(f"parallel oracle failed rc={rc}")
    ok_par = text == truth
    del text
    par_ops = (n + nl) / (ti + tw)
    serial = None
    if sample_n:
        g = kh.SyntheticKmers(k, sample_n, w["len_min"], w["len_max"], w["single"],
                              seed=w["seed"], **w.get("gen", {}))
        rc, text, snc, snl, sti, stw = ob.assemble(k, g.records())
        if rc != 0:
            raise RuntimeError(f"oracle failed rc={rc}")
        serial = {"value": (sample_n + snl) / (sti + stw), "unit": "ops/s", "cores": 1, "kind": "port",
                  "sample": f"{sample_n} k-mers of the same generator/config, {snc} contigs; insert "
                            f"{sti:.2f}s + walk {stw:.2f}s; oracle/kmer_oracle.c serial stock semantics "
                            f"(djb2, linear probing, load 0.5); output == ground truth: {text == g.truth()}"}
    return {"value": par_ops, "unit": "ops/s", "cores": P, "kind": "port",
            "nproc": os.cpu_count(), "host_cpu": host_cpu_model(),
            "sample": f"the full workload: {n} k-mers, {nc} contigs; {P} threads as {P} ranks "
                      f"(oracle/kmer_oracle_par.c: block split read_kmers.hpp:55-58, owner-batched "
                      f"insert_all hash_map.hpp:55-80 into stock open-addressing shards at load 0.5, "
                      f"each rank walks its own start nodes kmer_hash.cpp:38-55); insert {ti:.2f}s + "
                      f"walk {tw:.2f}s; output == ground truth: {ok_par}",
            "serial": serial}


def load_traffic(workload, n_per_gpu):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (workload key: e.g. "c3", or "c3_dist" for the sharded path at one rank)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    e = d.get(workload)
    if not e or e.get("n") != n_per_gpu:
        return None, None
    return e, os.path.relpath(path, ROOT)


def end_to_end(table, host, n, nl, truth, steps):
    """The reference's timed boundary (kmer_hash.cpp:129-137): records packed in host memory ->
    contigs in host memory. One step = kh_insert of the host records (H2D from pinned memory +
    the insert pipeline), assemble, D2H of the contig text into pinned memory."""
    import ctypes
    import numpy as np
    import torch
    import cs267_hw3_amd as kh
    L = kh._lib.lib()
    pin = torch.empty(host.nbytes, dtype=torch.uint8, pin_memory=True)
    pin.numpy()[:] = host.reshape(-1).view(np.uint8)
    tb = len(truth)
    tpin = torch.empty(tb + 64, dtype=torch.uint8, pin_memory=True)
    nb = ctypes.c_uint64(0)
    nco = ctypes.c_uint64(0)

    def step(ph=None):
        t0 = time.perf_counter()
        table.clear()
        kh._lib.check(L.kh_insert(table._h, ctypes.c_void_p(pin.data_ptr()), n))
        t1 = time.perf_counter()
        kh._lib.check(L.kh_assemble(table._h, ctypes.byref(nco), ctypes.byref(nb)))
        t2 = time.perf_counter()
        kh._lib.check(L.kh_contigs_text(table._h, ctypes.c_void_p(tpin.data_ptr()), tb + 64))
        t3 = time.perf_counter()
        if ph is not None:
            ph.append(((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3))

    step()
    times, ph = [], []
    for _ in range(steps):
        t = time.perf_counter()
        step(ph)
        times.append((time.perf_counter() - t) * 1e3)
    ok = nb.value == tb and bytes(tpin.numpy()[:tb]) == truth
    med = sorted(times)[len(times) // 2]
    # the PCIe floor of the same bytes: the pinned records alone up, the text alone down
    dev = torch.empty(host.nbytes, dtype=torch.uint8, device="cuda")
    dtext = torch.empty(tb, dtype=torch.uint8, device="cuda")
    h2d, d2h = [], []
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        dev.copy_(pin, non_blocking=True)
        torch.cuda.synchronize()
        h2d.append((time.perf_counter() - t) * 1e3)
        t = time.perf_counter()
        tpin[:tb].copy_(dtext, non_blocking=True)
        torch.cuda.synchronize()
        d2h.append((time.perf_counter() - t) * 1e3)
    del dev, dtext
    hot = table.stats()["n_hot_regions"]
    h2d_ms, d2h_ms = min(h2d), min(d2h)
    return {"value": (n + nl) / (med / 1e3), "unit": "ops/s", "ms_per_step_median": med, "step_ms": times,
            "phases_ms_median": {k: sorted(p[i] for p in ph)[len(ph) // 2]
                                 for i, k in enumerate(("kh_insert", "kh_assemble", "kh_contigs_text"))},
            "pcie_floor_ms": {"h2d_records": h2d_ms, "d2h_text": d2h_ms, "sum": h2d_ms + d2h_ms,
                              "h2d_GBs": host.nbytes / h2d_ms / 1e6, "d2h_GBs": tb / d2h_ms / 1e6},
            "h2d_bytes": int(host.nbytes), "d2h_bytes": tb, "verified_vs_truth": ok, "hot_regions": hot,
            "note": "reference boundary (kmer_hash.cpp:129-137): kh_insert from pinned host records "
                    "(H2D + insert), kh_assemble, kh_contigs_text D2H into pinned host memory"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` without an outer torchrun: start N ranks (one process per GPU) as a
    torch.distributed.run CHILD of this process and exit with its status. This parent has not
    touched the GPU (nothing above imports torch or the library), and it never execs: the ranks
    are children. Rank 0 prints the JSON line; its stdout is passed through unchanged."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, KH_BENCH_LAUNCHED="1")
    log(f"bench: --gpus {n} without WORLD_SIZE: launching {n} ranks via torch.distributed.run")
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--n", "--kmers", dest="n", type=int, default=0,
                    help="override k-mers per GPU (--kmers under torchrun: its argparse takes --n "
                         "for an abbreviation of its own options)")
    ap.add_argument("--load", type=float, default=0.5,
                    help="table load factor (kmer_hash.cpp:109 uses 0.5; SURVEY C5 names a 0.85 variant)")
    ap.add_argument("--cpu-sample", type=int, default=20_000_000,
                    help="k-mers for the serial CPU baseline sample (0 = skip the serial leg)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--e2e-steps", type=int, default=3,
                    help="steps of the reference-boundary (host records -> host contigs) figure")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-routed", action="store_true",
                    help="forced one-rank sharded line: skip the routed-step measurement")
    args = ap.parse_args()

    w = dict(WORKLOADS[args.workload])
    w["name"] = args.workload
    if args.n:
        w["n"] = args.n
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if os.environ.get("KH_BENCH_LAUNCHED"):
            raise SystemExit("bench: launched ranks see no WORLD_SIZE")
        return launch_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        # never report an N-GPU run measured on another number of ranks
        log(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
        return 2
    if world > 1 or os.environ.get("KH_BENCH_FORCE_DIST") == "1":
        # sharded path (also forced at one rank to exercise it on a 1-GPU box)
        from cs267_hw3_amd import dist
        return dist.bench_main(args, w, world, rank, cpu_baseline=cpu_baseline, load_traffic=load_traffic)

    import numpy as np
    import cs267_hw3_amd as kh

    k, n = w["k"], w["n"]
    t = time.time()
    g = kh.SyntheticKmers(k, n, w["len_min"], w["len_max"], w["single"], seed=w["seed"], **w.get("gen", {}))
    if w.get("strong"):
        log("note: a strong-scaling workload on one GPU: the whole set on this GPU")
    host = g.records()
    log(f"generated {n} records ({host.nbytes / 1e9:.2f} GB) in {time.time() - t:.1f}s")
    L = kh._lib.lib()
    import ctypes
    dptr = ctypes.c_void_p()
    kh._lib.check(L.kh_dev_malloc(ctypes.byref(dptr), host.nbytes, 0))
    kh._lib.check(L.kh_memcpy_htod(dptr, ctypes.c_void_p(host.ctypes.data), host.nbytes))
    table = kh.KmerHashTable(k, n, args.load, device=0)

    def step():
        table.clear()
        table.insert_dev(dptr.value, n)
        table.assemble_dev()
        table.sync()
        return table.stats()

    for _ in range(args.warmup):
        step()
    table.sync()
    phases, step_ms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ts = time.perf_counter()
        phases.append(step())           # step() ends with a stream sync: per-step wall time
        step_ms.append((time.perf_counter() - ts) * 1e3)
    t1 = time.perf_counter()
    ms = (t1 - t0) * 1e3 / args.steps
    s = phases[-1]
    nc, nl = s["n_contigs"], s["n_lookups"]
    assert s["n_inserted"] == n and nl == n - nc, s
    truth = g.truth()
    ok = None
    if not args.no_verify:
        ok = table.contigs_text() == truth
        if not ok:
            raise SystemExit("bench: contig text differs from the generator ground truth")
    e2e = end_to_end(table, host, n, nl, truth, args.e2e_steps) if args.e2e_steps else None
    ops = n + nl
    value = ops / (ms / 1e3)
    avg = lambda key: sum(p[key] for p in phases) / len(phases)  # noqa: E731
    ins_ms, walk_ms = avg("ms_insert_kernel"), avg("ms_walk")
    build_ms, walkk_ms = avg("ms_build"), avg("ms_walk_kernel")
    rec_bytes = kh.record_size(k)
    b_alg = 2 * rec_bytes      # read+write one kmer_pair per insert / lookup
    traffic, tsrc = load_traffic(args.workload, n)

    def kernel_roof(name, units, ms, tkey, what):
        t = traffic.get(tkey) if traffic else None
        return {"bound": "hbm", "kernel": name, "achieved": units * b_alg / (ms / 1e3) / 1e9, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": units * b_alg / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": t,
                "alg_bytes_per_unit": b_alg, "units_per_launch": units, "avg_launch_ms": ms,
                "traffic_GBs": (t / (ms / 1e3) / 1e9) if t else None,
                "note": f"achieved = {what} x 2*sizeof(kmer_pair) / HIP-event duration of the kernel"
                        + (f"; traffic = PMC HBM bytes per launch from {tsrc}" if tsrc and t else "")}

    # region build (k_part_build_pf: LDS build of every region + chain links + head records, then
    # the overflow inserts), HIP events around it on the table's stream; its inherent traffic is a
    # 16-B word in and two 16-B slots out per k-mer (load 0.5), 48 B
    kb = kernel_roof("k_part_build_pf (region build + chains)", n, build_ms, "k_part_build", "inserts")
    kb["inherent_bytes_per_unit"] = 48
    # contig walk: one lookup per k-mer but, with chains, ~1 random request per run of ~19 k-mers
    # (the record of the next run, named by k_rec_succ beside the walk: both in the HIP-event bracket
    # and in the PMC sums)
    kw = kernel_roof("k_walk_q + k_rec_succ (contig walk, chain hops)", nl, walkk_ms, "k_walk", "lookups")
    rq = ((traffic or {}).get("requests") or {}).get("TCC_EA0_RDREQ_sum", {}).get("k_walk")
    kw["requests_per_lookup"] = rq / nl if rq else None  # 64-B HBM read requests (PMC) per lookup
    # the walk in what it moves: PMC bytes (traffic_GBs above) and random 64-B requests per second
    # against the measured random-request ceiling (tools/membench.hip: ~49 G random 16-B loads/s
    # = 64-B requests/s at a 6.4 GB table, profiles/r01/membench.jsonl)
    kw["requests_per_s"] = rq / (walkk_ms / 1e3) if rq else None
    kw["request_ceiling_per_s"] = RANDOM_REQ_CEILING
    kw["request_frac"] = kw["requests_per_s"] / RANDOM_REQ_CEILING if rq else None
    roof = dict(kb if build_ms >= walkk_ms else kw)
    roof["kernels"] = {"k_part_build_pf": kb, "k_walk_q": kw}
    insert_pipe = {"kernels": "k_win1_rec (records -> parse + minimizer + bucket sort), k_win2, k_part_build_pf, "
                              "k_insert_overflow" if k in (51, 19) else
                              "k_part1_convert (records -> words + minimizer), k_win1, k_win2, k_part_build_pf, "
                              "k_insert_overflow",
                   "ms": ins_ms, "achieved_alg_GBs": n * b_alg / (ins_ms / 1e3) / 1e9,
                   "inserts_per_s": n / (ins_ms / 1e3),
                   "traffic": traffic.get("insert_pipeline") if traffic else None}
    if insert_pipe["traffic"]:
        # PMC-measured HBM bytes of the pipeline's kernels / their HIP-event time, against peak
        insert_pipe["traffic_GBs"] = insert_pipe["traffic"] / (ins_ms / 1e3) / 1e9
        insert_pipe["traffic_frac"] = insert_pipe["traffic_GBs"] / HBM_PEAK_GBS
    cpu = None
    if not args.no_cpu:
        t = time.time()
        cpu = cpu_baseline(w, host, truth, min(args.cpu_sample, n))
        log(f"cpu baseline took {time.time() - t:.1f}s")
    out = {
        "metric": "k-mer inserts+lookups/sec (k=51)" if k == 51 else f"k-mer inserts+lookups/sec (k={k})",
        "value": value, "unit": "ops/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms,
        "ms_per_step_median": sorted(step_ms)[len(step_ms) // 2], "step_ms": step_ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": value / BEST_PUBLISHED_OPS, "dtype": "u64", "data": "synthetic",
        "config": {"workload": w["desc"], "k": k, "n_kmers_per_gpu": n, "contigs": nc,
                   "lookups": nl, "parallelism": "1 GPU", "load_factor": args.load,
                   "hot_regions": s["n_hot_regions"], "spread_regions": s["n_spread_regions"],
                   "overflow_cas_keys": s["n_overflow"],
                   "vs_baseline_ref": "72.6e6 ops/s: reference best, k=51 human-chr14, "
                                      "4 nodes x 128 CPU ranks (BASELINE.md)"},
        "inserts_per_s": n / (ms / 1e3), "lookups_per_s": nl / (ms / 1e3),
        "contigs_per_s": nc / (ms / 1e3),
        "phases_ms": {"insert_total": avg("ms_insert"), "k_insert": ins_ms, "build": build_ms,
                      "k_walk": walk_ms, "walk_kernel": walkk_ms, "materialize": avg("ms_materialize")},
        "verified_vs_truth": ok,
        "roofline": roof, "insert_pipeline": insert_pipe, "end_to_end": e2e, "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    table.close()
    L.kh_dev_free(dptr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
