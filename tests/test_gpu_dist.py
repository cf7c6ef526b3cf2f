"""GPU: the sharded path's kernels (route / insert words / migrating walker rounds / splitter
segments) with P logical ranks on one GPU (ThreadComm). Each rank's text == ground truth of its block; the union
== the reference-harness output / the oracle."""
import json
import os

import numpy as np
import pytest

import cs267_hw3_amd as kh
import oracle_bind as ob

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))


def check_ranks(g, texts, P):
    for r, got in enumerate(texts):
        b, e = g.block(P, r)
        assert got == g.truth(b, e), f"rank {r}"


@pytest.mark.parametrize("name", ["mixed19", "small51", "singles51", "k30", "k60", "tiny19"])
@pytest.mark.parametrize("P", [1, 2, 3, 4, 8])
def test_sharded_golden(name, P):
    from cs267_hw3_amd.dist import run_threaded
    m = MANIFEST[name]
    recs = kh.pack_text(m["k"], open(os.path.join(GOLDEN, f"{name}.txt"), "rb").read())
    texts = run_threaded(m["k"], recs, P)
    g = kh.SyntheticKmers(m["k"], m["n"], m["len_min"], m["len_max"], m["single_permille"],
                          seed=m["seed"])
    check_ranks(g, texts, P)
    want = open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()
    assert sorted(b"".join(texts).splitlines()) == sorted(want.splitlines())


@pytest.mark.parametrize("k,n,P", [(51, 2_000_000, 8), (19, 1_000_000, 4)])
def test_sharded_generated(k, n, P):
    from cs267_hw3_amd.dist import run_threaded
    g = kh.SyntheticKmers(k, n, 8, 400, 10, seed=k + P)
    texts = run_threaded(k, g.records(), P)
    check_ranks(g, texts, P)


def test_sharded_missing_kmer_raises():
    from cs267_hw3_amd.dist import run_threaded
    m = MANIFEST["tiny19"]
    recs = kh.pack_text(19, open(os.path.join(GOLDEN, "tiny19.txt"), "rb").read())
    P = (19 + 3) // 4
    interior = np.where((recs[:, P] != ord("F")) & (recs[:, P + 1] != ord("F")))[0][5]
    with pytest.raises(kh.KmerHashError):
        run_threaded(19, np.delete(recs, interior, axis=0), 2)


@pytest.mark.parametrize("mode", ["cas", "part"])
@pytest.mark.parametrize("P", [1, 2, 5])
def test_sharded_large_both_insert_paths(monkeypatch, mode, P):
    """>= 1M routed words per rank: the partitioned build consumes words, not records."""
    from cs267_hw3_amd.dist import run_threaded
    monkeypatch.setenv("KH_INSERT", mode)
    g = kh.SyntheticKmers(51, 2_500_000 * P, 8, 200, 0, seed=77 + P)
    texts = run_threaded(51, g.records(), P)
    check_ranks(g, texts, P)


@pytest.mark.parametrize("mode", ["cas", "part"])
def test_insert_words_direct(monkeypatch, mode):
    import torch
    from cs267_hw3_amd.dist import GpuShard
    monkeypatch.setenv("KH_INSERT", mode)
    g = kh.SyntheticKmers(51, 3_000_000, 8, 200, 0, seed=5)
    sh = GpuShard(51, 3_000_000)
    with torch.cuda.stream(sh.stream):
        recs = torch.from_numpy(g.records()).cuda()
        words, counts = sh.route(recs, 1)
        sh.insert_words(words, recs.shape[0])
        sh.sync()
    s = sh.stats()
    assert s["n_dup"] == 0 and s["n_inserted"] == 3_000_000


def test_sharded_long_contigs_migrate():
    """C2-like chains (hundreds of k-mers): many self-migrations (run word budget) and
    cross-rank hops per walker."""
    from cs267_hw3_amd.dist import run_threaded
    g = kh.SyntheticKmers(19, 2_000_000, 200, 1374, 0, seed=11)
    for P in (1, 3):
        check_ranks(g, run_threaded(19, g.records(), P), P)


def test_sharded_hash_owner(monkeypatch):
    """SURVEY §8(e)'s owner (hash bits) instead of the minimizer owner: same outputs."""
    from cs267_hw3_amd.dist import run_threaded
    monkeypatch.setenv("KH_OWNER", "hash")
    g = kh.SyntheticKmers(51, 500_000, 8, 200, 10, seed=123)
    check_ranks(g, run_threaded(51, g.records(), 4), 4)


@pytest.mark.parametrize("chunks", [2, 5])
def test_sharded_pipelined_insert(chunks):
    """Chunked route + one count exchange + chunked transfers of the insert, P=4 logical ranks."""
    from cs267_hw3_amd.dist import run_threaded
    g = kh.SyntheticKmers(51, 6_000_000, 8, 200, 10, seed=321)
    check_ranks(g, run_threaded(51, g.records(), 4, insert_chunks=chunks), 4)


@pytest.mark.parametrize("mode", ["auto", "cas"])
@pytest.mark.parametrize("k,n,chunks", [(51, 3_000_000, 4), (19, 2_000_000, 3), (51, 200_000, 2)])
def test_staged_insert_words(monkeypatch, mode, k, n, chunks):
    """kh_insert_words_stage_dev per chunk (an empty one included) + kh_insert_words_finish ==
    one insert: the walk reproduces the ground truth; staging past the build's size fails."""
    import torch
    from cs267_hw3_amd import _lib
    from cs267_hw3_amd.dist import GpuShard
    if mode != "auto":
        monkeypatch.setenv("KH_INSERT", mode)
    g = kh.SyntheticKmers(k, n, 8, 300, 10, seed=k + chunks)
    sh = GpuShard(k, n + 5)
    with torch.cuda.stream(sh.stream):
        recs = torch.from_numpy(g.records()).cuda()
        sh.collect_starts(recs)
        words, _ = sh.route(recs, 1)
        W = sh.W
        bounds = [n * c // chunks for c in range(chunks + 1)]
        for c in range(chunks):
            a, b = bounds[c], bounds[c + 1]
            sh.stage_words(words[a * W:b * W], b - a, n + 5)
            if c == 0:
                sh.stage_words(words[:0], 0, n + 5)
        sh.finish_words()
        sh.table.assemble()
        assert sh.table.contigs_text() == g.truth()
        s = sh.stats()
        assert s["n_dup"] == 0 and s["n_inserted"] == n
        sh.clear()
        sh.stage_words(words[:W * 10], 10, 10)
        with pytest.raises(kh.KmerHashError) as e:
            sh.stage_words(words[:W * 10], 10, 10)
        assert e.value.code == _lib.KH_ERR_FULL
        sh.finish_words()


@pytest.mark.parametrize("P", [1, 4])
def test_sharded_skewed_c5(P):
    """C5 skew at small scale: long chains (hundreds of migrations each) among short contigs,
    every start k-mer in the first records (rank 0 owns all walkers)."""
    from cs267_hw3_amd.dist import run_threaded
    g = kh.SyntheticKmers(51, 600_000, 2, 16, 0, seed=55, n_long=4, long_len=20_000, front_starts=True)
    info = {}
    check_ranks(g, run_threaded(51, g.records(), P, info=info), P)


def test_sharded_stats_leave_no_hip_error():
    """The migrating walk records no walk-kernel event; stats() must not leave a failed event
    query as the thread's HIP last-error (torch's next launch check would raise it)."""
    import torch
    from cs267_hw3_amd.dist import DistributedKmerHashMap, GpuShard, ThreadComm
    g = kh.SyntheticKmers(51, 200_000, 8, 200, 0, seed=9)
    sh = GpuShard(51, 200_000)
    dm = DistributedKmerHashMap(ThreadComm.group(1)[0], sh)
    with torch.cuda.stream(sh.stream):
        dm.insert_all(torch.from_numpy(g.records()).cuda())
        dm.assemble(200_000)
    sh.sync()
    s = sh.stats()
    assert s["ms_walk"] >= 0 and s["ms_walk_kernel"] == 0
    assert dm.contigs_text() == g.truth()
    assert torch.ones(64, device="cuda").sum().item() == 64  # raises on a stale HIP error
    sh.table.close()
    assert torch.ones(64, device="cuda").sum().item() == 64


@pytest.mark.parametrize("P", [2, 8])
def test_sharded_host_syncs_per_step(P):
    """Device-resident rounds: fixed-size exchange slots (no host read per walk round), the
    splitter chains ranked on the device from an all-gathered predecessor table (no jump rounds),
    the walk's end checked where the last step ended. C3 shape (k=51, contigs U[8,200]) over P
    logical ranks, second step (buffers sized by the first): at most 8 blocking host reads per
    rank and step, this host's and the library's (kh_host_syncs), output == ground truth."""
    from cs267_hw3_amd.dist import run_threaded
    g = kh.SyntheticKmers(51, 4_000_000, 8, 200, 0, seed=51)
    info = {}
    check_ranks(g, run_threaded(51, g.records(), P, info=info, steps=2), P)
    assert max(info["syncs"].values()) <= 8, info["syncs"]
    assert max(info["checks"].values()) == 1, info["checks"]


@pytest.mark.parametrize("P", [1, 3, 4])
def test_sharded_tiny_slots_hold_messages_back(monkeypatch, P):
    """Slots of 256 messages: most walkers are held back on their sender and go out in later
    rounds (and at one rank, resent to itself); the walk still ends with every contig exact."""
    from cs267_hw3_amd import dist
    monkeypatch.setattr(dist.DistributedKmerHashMap, "SLOT_CAP_MAX", 256)
    g = kh.SyntheticKmers(51, 60_000, 8, 200, 0, seed=7 + P)
    check_ranks(g, dist.run_threaded(51, g.records(), P, steps=2), P)


@pytest.mark.parametrize("P", [2, 4])
def test_sharded_small_then_large_input(P):
    """Slot capacities are learnt per input: a map that walked a small set, cleared and given a
    C3-shape set 100x larger, sizes its first rounds from the new walker count (not the small
    walk's slots of a few hundred), so the walk ends in a normal number of rounds with every
    contig exact; then the small set again."""
    from cs267_hw3_amd.dist import run_threaded
    gs = kh.SyntheticKmers(51, 30_000, 8, 200, 0, seed=3)
    gl = kh.SyntheticKmers(51, 3_000_000, 8, 200, 0, seed=4)
    info = {}
    texts = run_threaded(51, [gs.records(), gl.records(), gs.records()], P, info=info)
    check_ranks(gs, texts[0], P)
    check_ranks(gl, texts[1], P)
    check_ranks(gs, texts[2], P)


@pytest.mark.parametrize("k,L,every,P", [(19, 3000, 1, 2), (51, 1500, 3, 2), (19, 2000, 2, 3)])
def test_sharded_overlapping_walks(k, L, every, P):
    """Walks that run into each other (malformed input: a k-mer with several predecessors, every
    start walking the shared tail again, kmer_hash.cpp:41-53) make a splitter segment two walks'
    successor: the segmented walk reports the overlap with its retag count exchange and every rank
    walks again without splitter segments (then once more with the text store the first redo
    needed). The ranks' texts, concatenated in rank order, equal the oracle's byte for byte (as the
    single-GPU kh_assemble's redo does, test_overlapping_walks_redo)."""
    from cs267_hw3_amd.dist import run_threaded
    from test_gpu_parity import dirty_device_memory, merging_walks
    recs = merging_walks(k, L, seed=26 + k, every=every)
    rc, want, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0 and len(want) > 4 * len(recs)
    dirty_device_memory()
    texts = run_threaded(k, recs, P)
    assert b"".join(texts) == want


@pytest.mark.parametrize("P", [1, 3])
@pytest.mark.parametrize("n_long", [0, 2])
def test_sharded_short_walk_first(P, n_long):
    """Short walk first (dist.py assemble): contigs shorter than the splitter spacing walk without
    splitter segments; two long chains make every rank walk again segmented (and keep doing so for
    this input: the second step goes straight to the segmented walk). Ground truth either way."""
    from cs267_hw3_amd.dist import run_threaded
    g = kh.SyntheticKmers(51, 1_500_000, 2, 12, 0, seed=71 + n_long, n_long=n_long, long_len=40_000)
    info = {}
    texts = run_threaded(51, [g.records(), g.records()], P, info=info)
    for t in texts:
        check_ranks(g, t, P)
    assert all(v == bool(n_long) for v in info["segmented"].values())

