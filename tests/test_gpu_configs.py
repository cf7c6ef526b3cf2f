"""Every BASELINE.json config at the size it names, on the GPU:

  C2  k=19, 10M k-mers, one GPU                 -> byte-compared to the oracle (device and host
      inserts); test_gpu_parity.py (generator truth, 10M)
  C3  k=51, 200M k-mers, one GPU, load 0.5      -> byte-compared to the generator's ground truth;
      a C3-shape 20M sample byte-compared to the oracle (oracle/kmer_oracle.c, ~7 s)
  C4  k=51, 1B k-mers sharded over 8 ranks      -> 8 logical ranks on one GPU (ThreadComm): each
      rank's text == the truth of its block (read_kmers.hpp:55-58); the exchange protocol is the
      one RCCL runs at 8 GPUs, only the transport differs
  C5  k=51, 200M skewed k-mers over 8 ranks     -> same, with the C5 generator (8 chains of 10^6
      k-mers, every start k-mer first: rank 0 owns every walker)

Inputs are generated on the GPU (kh_gen_records_dev) so a 1B set takes seconds; the truth is
built on the host by the same generator (kh_gen_truth) and compared per rank.
"""
import os
import sys

import pytest
import torch

import cs267_hw3_amd as kh

pytestmark = pytest.mark.gpu

C3 = dict(k=51, len_min=8, len_max=200, single=0, seed=51)
C5 = dict(k=51, len_min=2, len_max=16, single=0, seed=5199, n_long=8, long_len=1_000_000, front_starts=True)
# C5's hot-bucket half: 30 % of the contigs carry one of 8 shared minimizer motifs (60M k-mers in
# 8 minimizer windows: each window alone is ~2,500 region slices' worth of keys)
C5H = dict(k=51, len_min=8, len_max=200, single=0, seed=5198, hot_permille=300, n_motifs=8)
# its worst case for the remap: a fixed flank before every motif, so ~40 % of each family shares the
# neighbour window too (one remap target region per family before the level-2 spread)
C5F = dict(C5H, seed=5197, hot_flank=True)


def _gen(cfg, n):
    c = dict(cfg)
    return kh.SyntheticKmers(c.pop("k"), n, c.pop("len_min"), c.pop("len_max"), c.pop("single"),
                             seed=c.pop("seed"), **c)


def _single_gpu(g, n, load=0.5):
    """One table, records generated in HBM, one insert + assemble; returns the contig text."""
    with kh.KmerHashTable(g.k, n, load) as t:
        s = torch.cuda.Stream()
        t.set_stream(s.cuda_stream)
        recs = g.records_dev(stream=s)
        t.insert_dev(recs.data_ptr(), n)
        t.sync()
        del recs
        t.assemble()
        st = t.stats()
        assert st["n_dup"] == 0 and st["n_full"] == 0 and st["n_missing"] == 0
        return t.contigs_text(), st


def test_device_generator_matches_host():
    """kh_gen_records_dev == kh_gen_records (plain and C5 orders, unaligned ranges)."""
    import numpy as np
    for cfg, n in ((C3, 3_000_000), (C5, 1_500_000), (dict(C3, k=19, seed=19, len_min=200, len_max=1374), 2_000_000)):
        g = _gen(dict(cfg, long_len=100_000) if "long_len" in cfg else cfg, n)
        for b, e in ((0, n), (12345, 1_234_567), (n - 77, n)):
            got = g.records_dev(b, e).cpu().numpy()
            assert np.array_equal(got, g.records(b, e))


def test_c3_full_size_vs_truth():
    """BASELINE configs[2] at full size: 200M k-mers, k=51, load 0.5."""
    n = 200_000_000
    g = _gen(C3, n)
    text, st = _single_gpu(g, n)
    assert st["n_contigs"] == g.num_contigs
    assert text == g.truth()


def test_c3_shape_20m_vs_oracle():
    """The oracle (serial stock open addressing + the reference walk) on a 20M C3-shape set."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_bind as ob
    n = 20_000_000
    g = _gen(C3, n)
    rc, want, nc, _, _, _ = ob.assemble(51, g.records())
    assert rc == 0
    text, st = _single_gpu(g, n)
    assert st["n_contigs"] == nc
    assert text == want


def _host_insert(g, recs, n, load=0.5):
    """The reference boundary: records in host memory through kh_insert (>= 2^24 records into an
    empty table: the chunked upload, H2D overlapped with the partition passes)."""
    with kh.KmerHashTable(g.k, n, load) as t:
        t.insert_all(recs)
        t.assemble()
        st = t.stats()
        assert st["n_dup"] == 0 and st["n_full"] == 0 and st["n_missing"] == 0
        return t.contigs_text(), st


@pytest.mark.parametrize("load", [0.5, 0.85])
def test_c3_shape_20m_host_insert_vs_oracle(load):
    """kh_insert from host records (chunked upload) == the oracle on the 20M C3-shape set."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_bind as ob
    n = 20_000_000
    g = _gen(C3, n)
    recs = g.records()
    rc, want, nc, _, _, _ = ob.assemble(51, recs)
    assert rc == 0
    text, st = _host_insert(g, recs, n, load)
    assert st["n_contigs"] == nc and text == want


def test_c2_10m_vs_oracle():
    """BASELINE configs[1] (k=19, 10M) byte-compared to the oracle, device and host inserts."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_bind as ob
    n = 10_000_000
    g = _gen(dict(C3, k=19, seed=19, len_min=200, len_max=1374), n)
    recs = g.records()
    rc, want, nc, _, _, _ = ob.assemble(19, recs)
    assert rc == 0
    text, st = _single_gpu(g, n)
    assert st["n_contigs"] == nc and text == want
    text, st = _host_insert(g, recs, n)
    assert st["n_contigs"] == nc and text == want


def test_chunked_upload_hot_bucket_vs_truth():
    """The chunked upload samples hot regions from its first chunk only: the C5 hot-bucket set at
    40M through kh_insert still assembles to the truth with the hot regions found."""
    n = 40_000_000
    g = _gen(C5H, n)
    text, st = _host_insert(g, g.records(), n)
    assert st["n_contigs"] == g.num_contigs and st["n_hot_regions"] >= 8
    assert text == g.truth()


@pytest.mark.parametrize("load", [0.5, 0.85])
def test_c5_hot_bucket_200m_one_gpu(load):
    """BASELINE configs[4] hot-bucket half at 200M on one GPU, at load 0.5 and SURVEY's 0.85."""
    n = 200_000_000
    g = _gen(C5H, n)
    text, st = _single_gpu(g, n, load)
    assert st["n_contigs"] == g.num_contigs and st["n_hot_regions"] >= 8
    assert text == g.truth()


@pytest.mark.parametrize("load", [0.5, 0.85])
def test_c5_hot_flank_200m_one_gpu(load):
    """Hot families that also share the neighbour window (a 32-base repeat): the remap's target
    regions overfill, the sampled level-2 mark spreads their remapped keys by key hash before pass
    1, so the global CAS list (list B) stays under 1 % of n and the text equals the truth."""
    n = 200_000_000
    g = _gen(C5F, n)
    text, st = _single_gpu(g, n, load)
    assert st["n_contigs"] == g.num_contigs and st["n_hot_regions"] >= 8
    assert st["n_spread_regions"] >= 8, st
    assert st["n_overflow"] < n // 100, st
    assert text == g.truth()


def test_c5_hot_flank_20m_vs_oracle_and_8_ranks():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_bind as ob
    n = 20_000_000
    g = _gen(C5F, n)
    rc, want, nc, _, _, _ = ob.assemble(51, g.records())
    assert rc == 0 and want == g.truth()
    text, st = _single_gpu(g, n)
    assert st["n_contigs"] == nc and text == want
    assert st["n_spread_regions"] > 0 and st["n_overflow"] < n // 100, st
    # the owners of the shared minimizers receive whole families; their shards spread them too
    info = _sharded(g, 8)
    assert sum(s["n_inserted"] for s in info["stats"].values()) == n
    assert max(s["n_overflow"] for s in info["stats"].values()) < n // 100


def test_c5_hot_bucket_20m_vs_oracle():
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import oracle_bind as ob
    n = 20_000_000
    g = _gen(C5H, n)
    rc, want, nc, _, _, _ = ob.assemble(51, g.records())
    assert rc == 0
    text, st = _single_gpu(g, n)
    assert st["n_contigs"] == nc and text == want


def _sharded(g, P, **kw):
    from cs267_hw3_amd.dist import run_threaded
    bad = []

    def check(r, text):
        b, e = g.block(P, r)
        if text != g.truth(b, e):
            bad.append(r)

    info = {}
    run_threaded(g.k, g, P, check=check, info=info, **kw)
    assert not bad, f"ranks {bad} differ from the truth of their blocks"
    return info


def test_c4_1b_kmers_8_ranks():
    """BASELINE configs[3]: 1B k-mers, k=51, sharded over 8 ranks (logical, one GPU)."""
    n = 1_000_000_000
    info = _sharded(_gen(C3, n), 8)
    assert sum(s["n_inserted"] for s in info["stats"].values()) == n


def test_c5_skewed_200m_8_ranks():
    """BASELINE configs[4]: the skewed set at 200M over 8 ranks (logical, one GPU)."""
    info = _sharded(_gen(C5, 200_000_000), 8)
    assert sum(s["n_inserted"] for s in info["stats"].values()) == 200_000_000


@pytest.mark.parametrize("load", [0.5, 0.85])
def test_c5_hot_bucket_200m_8_ranks(load):
    """The hot-bucket set over 8 ranks (logical, one GPU): the owner of a shared minimizer window
    receives its whole family (the all-to-all imbalance the config names)."""
    info = _sharded(_gen(C5H, 200_000_000), 8, load_factor=load)
    assert sum(s["n_inserted"] for s in info["stats"].values()) == 200_000_000


@pytest.mark.parametrize("load", [0.5, 0.85])
def test_c5_hot_bucket_1b_8_ranks(load):
    """BASELINE configs[4] at SURVEY §8(d)'s size: the hot-bucket set (30 % of the contigs on 8
    shared minimizers, so 8 owners each receive a whole 37.5M-k-mer family) at 1B k-mers over 8
    ranks (logical, one GPU), loads 0.5 and 0.85; every rank's text equals its block's truth."""
    info = _sharded(_gen(C5H, 1_000_000_000), 8, load_factor=load)
    assert sum(s["n_inserted"] for s in info["stats"].values()) == 1_000_000_000


def _mem_model():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "mem_model", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "mem_model.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _dev_bytes():
    """Device bytes held now: the library's buffers (every table) + torch's allocated tensors."""
    import ctypes
    from cs267_hw3_amd import _lib
    now = ctypes.c_uint64(0)
    _lib.lib().kh_device_bytes(ctypes.byref(now), None, 0)
    torch.cuda.synchronize()
    return now.value, torch.cuda.memory_allocated()


def test_mem_model_matches_measured_c3_routed_one_rank():
    """tools/mem_model.py (the sizing formulas of the library's buffers and the Python host's)
    against what the sharded step holds after a step: C3 200M through the one-pass route at one
    rank (the step P > 1 runs), the model fed with the step's own counts. Within 15 %."""
    import gc
    from cs267_hw3_amd.dist import DistributedKmerHashMap, GpuShard, ThreadComm
    gc.collect()
    torch.cuda.empty_cache()
    lib0, tor0 = _dev_bytes()
    n = 200_000_000
    g = _gen(C3, n)
    recs = g.records_dev(0, n, device=0)
    shard = GpuShard(51, int(n * 1.02) + 4096, device=0)
    with torch.cuda.stream(shard.stream):
        dm = DistributedKmerHashMap(ThreadComm.group(1)[0], shard)
        dm.ROUTE_ONE_RANK = True
        for step in range(2):
            if step:
                shard.clear()
            dm.insert_all(recs)
            dm.assemble(n)
    lib1, tor1 = _dev_bytes()
    assert dm.contigs_text() == g.truth(0, n)
    mm = _mem_model()
    items = mm.rank_model(P=1, n_rec=n, n_ins=n, n_table=int(n * 1.02) + 4096, ns=dm._ns, nsp=dm._nsp,
                          walkers_all=dm._walkers, routed=True, windows=True, exchange=False,
                          recv_text=dm.text_records, recv_seg=dm.seg_records)
    lib_m, tor_m = mm.totals(items)
    got_lib, got_tor = lib1 - lib0, tor1 - tor0
    print(f"model lib {lib_m / 1e9:.2f} torch {tor_m / 1e9:.2f} GB; measured lib {got_lib / 1e9:.2f} "
          f"torch {got_tor / 1e9:.2f} GB", file=sys.stderr)
    assert abs(lib_m + tor_m - got_lib - got_tor) <= 0.15 * (got_lib + got_tor)
    assert abs(lib_m - got_lib) <= 0.15 * got_lib
    shard.table.close()
    del recs, dm, shard


def test_mem_model_matches_measured_c5_8_ranks():
    """The same for C5 (walker skew: rank 0 holds every start k-mer) at 200M over 8 logical ranks
    on one GPU: the model fed with each rank's own counts, and the model fed with the counts
    workload_ranks() derives from the generator's parameters (as the 1B claim of DESIGN.md §6 is):
    both totals over the 8 ranks within 15 % of what the ranks hold after the step."""
    import gc
    import threading
    from cs267_hw3_amd.dist import run_threaded
    gc.collect()
    torch.cuda.empty_cache()
    lib0, tor0 = _dev_bytes()
    n, P = 200_000_000, 8
    g = _gen(C5, n)
    seen = {}
    bar = threading.Barrier(P)

    def check(r, text):
        bar.wait()          # every rank's walk is done, no shard closed yet
        if r == 0:
            seen["bytes"] = _dev_bytes()
        bar.wait()
        b, e = g.block(P, r)
        assert text == g.truth(b, e)

    info = {}
    run_threaded(51, g, P, check=check, info=info, shard_kmers=int(n / P * 1.02) + 4096)
    lib1, tor1 = seen["bytes"]
    got = (lib1 - lib0) + (tor1 - tor0)
    mm = _mem_model()
    exact = 0
    for r in range(P):
        b, e = g.block(P, r)
        exact += sum(mm.totals(mm.rank_model(P=P, n_rec=e - b, **info["counts"][r])))
    derived = sum(sum(mm.totals(mm.rank_model(**rk))) for rk in mm.workload_ranks("c5", n, P))
    print(f"model {exact / 1e9:.2f} GB (rank counts), {derived / 1e9:.2f} GB (workload counts); measured "
          f"{got / 1e9:.2f} GB (library {(lib1 - lib0) / 1e9:.2f})", file=sys.stderr)
    assert abs(exact - got) <= 0.15 * got
    assert abs(derived - got) <= 0.15 * got
