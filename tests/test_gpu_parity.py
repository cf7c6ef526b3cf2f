"""GPU parity: the HIP path (through the C ABI) against the reference-harness golden files, the
oracle, and the generator's ground truth. Integer/byte work -> every comparison is bit-exact."""
import json
import os

import numpy as np
import pytest

import cs267_hw3_amd as kh
from cs267_hw3_amd import _lib
import oracle_bind as ob
from cases import merging_walks_text

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))


def golden(name):
    m = MANIFEST[name]
    recs = kh.pack_text(m["k"], open(os.path.join(GOLDEN, f"{name}.txt"), "rb").read())
    want = open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()
    return m["k"], recs, want


def run(k, recs, batches=1, load=0.5, n_kmers=None):
    t = kh.KmerHashTable(k, n_kmers if n_kmers is not None else max(len(recs), 1), load)
    for part in np.array_split(recs, batches):
        t.insert_all(part)
    nc, nb = t.assemble()
    text = t.contigs_text()
    assert len(text) == nb
    return t, text, nc


def test_device_present():
    assert kh.device_count() >= 1


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_golden_byte_identical(name):
    k, recs, want = golden(name)
    t, got, nc = run(k, recs)
    assert got == want                          # test_0.dat bytes, start-node order
    s = t.stats()
    assert nc == MANIFEST[name]["contigs"] == s["n_contigs"] == s["n_starts"]
    assert s["n_lookups"] == len(recs) - nc
    assert s["n_inserted"] == len(recs)
    assert s["n_dup"] == s["n_missing"] == s["n_full"] == s["n_bad_ext"] == 0


@pytest.mark.parametrize("name", ["mixed19", "small51", "k32"])
@pytest.mark.parametrize("batches", [2, 7])
def test_multi_batch_insert_keeps_start_order(name, batches):
    k, recs, want = golden(name)
    _, got, _ = run(k, recs, batches=batches)
    assert got == want


@pytest.mark.parametrize("load", [0.25, 0.7, 0.95])
def test_load_factor_does_not_change_output(load):
    k, recs, want = golden("small51")
    _, got, _ = run(k, recs, load=load)
    assert got == want


@pytest.mark.parametrize("name", ["mixed19", "small51", "k29", "k30", "k60"])
def test_find_matches_oracle(name):
    k, recs, _ = golden(name)
    t = kh.KmerHashTable(k, len(recs))
    t.insert_all(recs)
    P = (k + 3) // 4
    rng = np.random.default_rng(5)
    present = recs[rng.choice(len(recs), 500, replace=False)]
    got, found = t.find(present[:, :P])
    assert found.all() and np.array_equal(got, present)
    # absent keys: random k-mers checked against the oracle's stock table
    ot = ob.Table(k, 2 * len(recs))
    for r in recs:
        ot.insert(r)
    bases = "ACGT"
    absent = np.stack([kh.pack_kmer(k, "".join(bases[x] for x in rng.integers(0, 4, k)))
                       for _ in range(300)])
    got, found = t.find(absent)
    for i in range(len(absent)):
        ok, rec = ot.find(absent[i])
        assert found[i] == ok
        if ok:
            assert np.array_equal(got[i], rec)
    assert np.all(got[~found] == 0)


def test_explicit_start_list():
    # assemble_contigs(hashmap, start_nodes) with a caller-supplied start list (kmer_hash.cpp:38)
    k, recs, want = golden("mixed19")
    t = kh.KmerHashTable(k, len(recs))
    t.insert_all(recs)
    starts = recs[recs[:, (k + 3) // 4] == ord("F")]
    t.set_starts(starts[::-1])
    t.assemble()
    assert t.contigs_text().splitlines() == want.splitlines()[::-1]


def merging_walks(k, L, seed, every=1):
    """Packed records of cases.merging_walks_text (overlapping start walks, malformed input)."""
    return kh.pack_text(k, merging_walks_text(k, L, seed, every))


def dirty_device_memory(gib=4):
    """Fill free device memory with 0xFF bytes and hand it back to the driver, so buffers the next
    step allocates start as garbage (a fresh box hands out zeros, which hid round 6's store-overflow
    bug: text records past the store's end read as rank 255)."""
    import torch
    t = torch.empty(gib << 30, dtype=torch.uint8, device="cuda")
    t.fill_(0xFF)
    torch.cuda.synchronize()
    del t
    torch.cuda.empty_cache()


@pytest.mark.parametrize("k,L,every", [(19, 3000, 1), (51, 2000, 3)])
def test_overlapping_walks_redo(k, L, every):
    """Walks that overlap (malformed input) pass the pre-walk text bound and exhaust the walker
    chunk pool: kh_assemble redoes the walk sized from the scanned total with the pool the first
    attempt asked for, and the text equals the oracle's (each start walked on its own)."""
    recs = merging_walks(k, L, seed=7 + k, every=every)
    rc, want, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0 and len(want) > 4 * len(recs)
    dirty_device_memory()
    _, got, got_nc = run(k, recs)
    assert got_nc == nc and got == want


def _split_hash(kmer):
    """kh_codec.hpp split_hash of a k-mer string (V = 2-bit bases, first base most significant)."""
    v = 0
    for ch in kmer:
        v = (v << 2) | "ACGT".index(ch)
    lo = v & ((1 << 62) - 1)
    return (((lo & 0xFFFFFFFF) ^ (lo >> 32)) * 0x9E3779B1) & 0xFFFFFFFF


@pytest.mark.parametrize("k", [19, 51])
def test_walk_into_start_that_passes_split_test(monkeypatch, k):
    """Malformed input: a chain k-mer C_j that passes split_test (so the segmented walk stops
    before it) also carries bwd 'F' (so it is a start, not a collected splitter). The reference
    walks C_0's contig on through C_j (kmer_hash.cpp:44 checks only the forward extension) and
    walks C_j's own contig too. The segmented walk cannot link to C_j; it reports an overlap and
    kh_assemble redoes the walk unsegmented: the text equals the oracle's."""
    monkeypatch.setenv("KH_SPLIT_BITS", "4")  # splitters 1 in 16, and walked at that density
    rng = np.random.default_rng(31 + k)
    L = 300
    seq = "".join("ACGT"[x] for x in rng.integers(0, 4, L + k - 1))
    chain = [seq[i:i + k] for i in range(L)]
    js = [j for j in range(2, L - 2) if _split_hash(chain[j]) < (1 << 28)]
    assert js, "no chain k-mer passes split_test at 4 bits"
    j = js[len(js) // 2]
    lines = []
    for i in range(L):
        bwd = "F" if i in (0, j) else seq[i - 1]
        fwd = "F" if i == L - 1 else seq[i + k]
        lines.append(f"{chain[i]} {bwd}{fwd}\n")
    lines += [f"{x} FF\n" for x in ("".join("ACGT"[b] for b in rng.integers(0, 4, k)) for _ in range(5))]
    order = rng.permutation(len(lines))
    recs = kh.pack_text(k, "".join(lines[i] for i in order).encode())
    rc, want, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0 and nc == 7
    dirty_device_memory()
    _, got, got_nc = run(k, recs)
    assert got_nc == nc and got == want


def test_empty_table():
    t = kh.KmerHashTable(19, 0)
    assert t.assemble() == (0, 0)
    assert t.contigs_text() == b""
    t.insert_all(np.zeros((0, 7), np.uint8))
    assert t.assemble() == (0, 0)


def test_clear_and_reuse():
    k, recs, want = golden("small51")
    t = kh.KmerHashTable(k, len(recs))
    for _ in range(3):
        t.clear()
        t.insert_all(recs)
        t.assemble()
        assert t.contigs_text() == want


def test_missing_kmer_raises():
    k, recs, _ = golden("tiny19")
    P = (k + 3) // 4
    interior = np.where((recs[:, P] != ord("F")) & (recs[:, P + 1] != ord("F")))[0][10]
    t = kh.KmerHashTable(k, len(recs))
    t.insert_all(np.delete(recs, interior, axis=0))
    with pytest.raises(kh.KmerHashError) as e:
        t.assemble()
    assert e.value.code == _lib.KH_ERR_NOT_FOUND


def test_duplicate_insert_is_reported():
    k, recs, _ = golden("small51")
    t = kh.KmerHashTable(k, 2 * len(recs))
    t.insert_all(recs)
    with pytest.raises(kh.KmerHashError) as e:
        t.insert_all(recs[:10])
    assert e.value.code == _lib.KH_ERR_DUPLICATE


def test_overfill_is_reported():
    k, recs, _ = golden("small51")
    t = kh.KmerHashTable(k, len(recs) - 1)
    with pytest.raises(kh.KmerHashError) as e:
        t.insert_all(recs)
    assert e.value.code == _lib.KH_ERR_FULL


def test_bad_extension_is_reported():
    k, recs, _ = golden("mixed19")
    recs = recs.copy()
    recs[3, (k + 3) // 4 + 1] = ord("N")
    t = kh.KmerHashTable(k, len(recs))
    with pytest.raises(kh.KmerHashError) as e:
        t.insert_all(recs)
    assert e.value.code == _lib.KH_ERR_BAD_BASE


@pytest.mark.parametrize("bad", [b"N", b"a", b"\x00", b"\x87", b"\xc1"])
def test_bad_extension_is_reported_partitioned(bad):
    """The records pass (batches >= 2^20 records) decodes both extension bytes with a byte table
    (ext_codes2): a byte outside {A,C,G,T,F} is EXT_BAD as in base_code, including bytes whose low 3
    bits index a valid character (0x87 -> 'G''s slot, 0xC1 -> 'A''s)."""
    k = 51
    g = kh.SyntheticKmers(k, 1_200_000, 8, 200, 10, seed=77)
    recs = g.records().copy()
    P = (k + 3) // 4
    interior = np.where((recs[:, P] != ord("F")) & (recs[:, P + 1] != ord("F")))[0][1000]
    recs[interior, P + 1] = bad[0]
    with pytest.raises(kh.KmerHashError) as e:
        with kh.KmerHashTable(k, len(recs), device=0) as t:
            t.insert_all(recs)
            t.assemble()
    assert e.value.code == _lib.KH_ERR_BAD_BASE


@pytest.mark.parametrize("k,n,lmin,lmax,single,seed", [
    (19, 1_000_000, 200, 1374, 0, 19),        # C2-like length mix, reduced n
    (51, 1_000_000, 8, 200, 10, 51),          # C3-like length mix, reduced n
    (31, 300_000, 1, 500, 50, 31),
    (45, 300_000, 1, 500, 50, 45),
])
def test_generated_vs_oracle(k, n, lmin, lmax, single, seed):
    g = kh.SyntheticKmers(k, n, lmin, lmax, single, seed=seed)
    recs = g.records()
    rc, want, nc, nl, _, _ = ob.assemble(k, recs)
    assert rc == 0
    _, got, gnc = run(k, recs)
    assert got == want and gnc == nc


@pytest.mark.parametrize("k", [19, 31, 40, 51])
def test_record_successors(k):
    """Head records name the record of the run after their tail (k_rec_succ): resolved beside the
    walk where a torn read is harmless (records read before their successor is resolved still say
    0 and the walker probes), before it otherwise (16-B slots at k <= 40); the text is the
    oracle's in every case, and a second walk of the same table reads resolved records only."""
    g = kh.SyntheticKmers(k, 1_000_000, 8, 400, 10, seed=k + 7)
    recs = g.records()
    rc, want, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0
    with kh.KmerHashTable(k, len(recs), device=0) as t:
        t.insert_all(recs)
        for _ in range(2):
            got_nc, _ = t.assemble()
            assert got_nc == nc and t.contigs_text() == want


def test_c2_full_size_vs_truth():
    # BASELINE configs[1]: k=19, 10M synthetic k-mers, bit-exact (vs generator ground truth,
    # which the oracle matches at every smaller size above)
    g = kh.SyntheticKmers(19, 10_000_000, 200, 1374, 0, seed=19)
    recs = g.records()
    t, got, nc = run(19, recs)
    assert nc == g.num_contigs
    assert got == g.truth()
    s = t.stats()
    assert s["n_lookups"] == 10_000_000 - nc


def test_c3_shape_vs_truth_30m():
    # configs[2] shape (k=51, U[8,200]) at 30M k-mers: byte-identical to the ground truth
    g = kh.SyntheticKmers(51, 30_000_000, 8, 200, 0, seed=51)
    recs = g.records()
    _, got, nc = run(51, recs)
    assert nc == g.num_contigs
    assert got == g.truth()


# ---- both insert strategies (KH_INSERT=cas: global CAS per key; part: partitioned LDS build) ----
@pytest.fixture(params=["cas", "part"])
def insert_mode(request, monkeypatch):
    monkeypatch.setenv("KH_INSERT", request.param)
    return request.param


@pytest.mark.parametrize("name", ["mixed19", "small51", "k29", "k30", "k60", "singles51"])
@pytest.mark.parametrize("batches", [1, 3])
def test_golden_both_insert_paths(insert_mode, name, batches):
    k, recs, want = golden(name)
    t, got, _ = run(k, recs, batches=batches)
    assert got == want
    assert t.stats()["n_dup"] == 0


@pytest.mark.parametrize("k,n,batches", [(51, 3_000_000, 1), (51, 3_000_000, 2), (19, 2_000_000, 1),
                                         (31, 2_000_000, 3)])
def test_generated_both_insert_paths(insert_mode, k, n, batches):
    g = kh.SyntheticKmers(k, n, 8, 300, 10, seed=k * 7 + batches)
    t, got, nc = run(k, g.records(), batches=batches)
    assert got == g.truth() and nc == g.num_contigs
    assert t.stats()["n_dup"] == 0


def test_part_build_detects_duplicates(monkeypatch):
    monkeypatch.setenv("KH_INSERT", "part")
    g = kh.SyntheticKmers(51, 2_000_000, 8, 200, 0, seed=3)
    recs = g.records()
    dup = np.concatenate([recs, recs[:1000]])
    t = kh.KmerHashTable(51, len(dup))
    with pytest.raises(kh.KmerHashError) as e:
        t.insert_all(dup)
    assert e.value.code == _lib.KH_ERR_DUPLICATE
    assert t.stats()["n_dup"] == 1000


# ---- §8(f)2: the text parser on the GPU ---------------------------------------------------------
@pytest.mark.parametrize("name", ["mixed19", "small51", "k30", "k60", "tiny19"])
def test_gpu_pack_text_golden(name):
    """kh_pack_text_dev == the host codec (pinned by the reference KATs) on the golden text."""
    import torch
    m = MANIFEST[name]
    raw = open(os.path.join(GOLDEN, f"{name}.txt"), "rb").read()
    want = kh.pack_text(m["k"], raw)
    t = kh.KmerHashTable(m["k"], 16)
    R = kh.record_size(m["k"])
    for off in (0, 1, 7):  # unaligned text starts
        buf = torch.zeros(len(raw) + 16, dtype=torch.uint8)
        buf[off:off + len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
        d = buf.cuda()
        recs = torch.empty(len(want) * R + 16, dtype=torch.uint8, device="cuda")
        n = t.pack_text_dev(d.data_ptr() + off, len(raw), recs.data_ptr())
        t.sync()
        assert n == len(want)
        assert bytes(recs[:n * R].cpu().numpy()) == want.tobytes()


@pytest.mark.parametrize("k", [19, 51])
def test_gpu_pack_text_large_and_bad_base(k):
    import torch
    g = kh.SyntheticKmers(k, 300_001, 8, 200, 10, seed=3)
    recs = g.records()
    line = k + 4
    text = np.empty((len(recs), line), np.uint8)
    # text from records through the host codec (unpack) -- vectorised per base
    P = (k + 3) // 4
    packed = recs[:, :P]
    bits = np.unpackbits(packed, axis=1)[:, :2 * k].reshape(len(recs), k, 2)
    codes = bits[:, :, 0] * 2 + bits[:, :, 1]
    text[:, :k] = np.frombuffer(b"ACGT", np.uint8)[codes]
    text[:, k] = ord(" ")
    text[:, k + 1] = recs[:, P]
    text[:, k + 2] = recs[:, P + 1]
    text[:, k + 3] = ord("\n")
    t = kh.KmerHashTable(k, 16)
    d = torch.from_numpy(text.reshape(-1)).cuda()
    out = torch.empty(len(recs) * (P + 2) + 16, dtype=torch.uint8, device="cuda")
    n = t.pack_text_dev(d.data_ptr(), d.numel(), out.data_ptr())
    t.sync()
    assert n == len(recs)
    assert np.array_equal(out[:n * (P + 2)].cpu().numpy().reshape(n, P + 2), recs)
    text[12345, 3] = ord("N")
    d = torch.from_numpy(text.reshape(-1)).cuda()
    t.pack_text_dev(d.data_ptr(), d.numel(), out.data_ptr())
    with pytest.raises(kh.KmerHashError):
        t.sync()


# ---- long chains: splitter segments (SURVEY §8(d) C5 / §8(e) long-tail strategy) --------------
@pytest.mark.parametrize("k,n,lmin,lmax,bits", [
    (51, 3_000_000, 200_000, 1_000_000, None),   # C5-like: a handful of very long chains
    (51, 3_000_000, 200_000, 1_000_000, "4"),    # dense splitters: many segments per contig
    (19, 2_000_000, 200, 1374, None),            # C2-like chain lengths
    (29, 1_000_000, 1, 3000, "3"),               # W=1 keys, single-k-mer contigs, dense splitters
    (60, 1_000_000, 1, 400, None),
])
def test_gpu_splitter_segments_vs_truth(monkeypatch, k, n, lmin, lmax, bits):
    if bits is not None:
        monkeypatch.setenv("KH_SPLIT_BITS", bits)
    g = kh.SyntheticKmers(k, n, lmin, lmax, 5, seed=k * 7 + lmin)
    with kh.KmerHashTable(k, n) as t:
        t.insert_all(g.records())
        t.assemble()
        assert t.contigs_text() == g.truth()


def test_gpu_splitters_off_equals_on(monkeypatch):
    g = kh.SyntheticKmers(51, 1_000_000, 50, 5000, 0, seed=99)
    texts = []
    for bits in ("0", "6"):
        monkeypatch.setenv("KH_SPLIT_BITS", bits)
        with kh.KmerHashTable(51, 1_000_000) as t:
            t.insert_all(g.records())
            t.assemble()
            texts.append(t.contigs_text())
    assert texts[0] == texts[1] == g.truth()


# ---- the line writer (k_write_lines, K >= 16; K < 16 keeps the heads writer) ------------------
# 1 KiB of text per wave: the shortest contigs (single k-mers, K + 1 bytes) put the most contig
# starts in one KiB (62 at K = 16) and a contig boundary in most 16-B lanes; contigs past their first
# 256-base chunk leave bytes to the chunk writer (splitters off: extra chunks; dense splitters:
# splitter segments as well); the text's last vector is partial.
@pytest.mark.parametrize("k,n,lmin,lmax,single", [
    (15, 200_000, 1, 40, 40), (16, 200_000, 1, 40, 40), (17, 200_000, 1, 4, 60),
    (16, 300_000, 200, 900, 0), (51, 300_000, 1, 3, 50), (60, 400_000, 250, 700, 5),
])
@pytest.mark.parametrize("bits", ["0", "3", None])
def test_gpu_line_writer_vs_oracle(monkeypatch, k, n, lmin, lmax, single, bits):
    if bits is not None:
        monkeypatch.setenv("KH_SPLIT_BITS", bits)
    g = kh.SyntheticKmers(k, n, lmin, lmax, single, seed=k * 11 + lmin)
    recs = g.records()
    rc, want, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0 and want == g.truth()
    _, got, gnc = run(k, recs)
    assert gnc == nc and got == want


# ---- the region build's two kernels: prefetching (default) and one-region-at-a-time (windows
# above 12 words per thread, > ~760M k-mers per table; forced here with KH_DEBUG=plain_build) ----
@pytest.mark.parametrize("build", ["plain_build", ""])
@pytest.mark.parametrize("k,n,load", [(51, 3_000_000, 0.5), (19, 2_000_000, 0.5), (31, 1_500_000, 0.9),
                                      (60, 1_200_000, 0.25)])
def test_gpu_build_kernels(monkeypatch, build, k, n, load):
    monkeypatch.setenv("KH_INSERT", "part")
    monkeypatch.setenv("KH_DEBUG", build)
    g = kh.SyntheticKmers(k, n, 8, 300, 10, seed=k + n % 97)
    with kh.KmerHashTable(k, n, load) as t:
        t.insert_all(g.records())
        t.assemble()
        assert t.contigs_text() == g.truth()
        s = t.stats()
        assert s["n_dup"] == 0 and s["n_full"] == 0


# ---- C5 skew on one GPU ---------------------------------------------------------------------------
@pytest.mark.parametrize("k,n,n_long,long_len", [(51, 4_000_000, 4, 600_000), (19, 2_000_000, 3, 300_000)])
def test_gpu_skewed_c5(k, n, n_long, long_len):
    """C5 skew on one GPU: splitter segments walk the long chains; starts first in record order."""
    g = kh.SyntheticKmers(k, n, 2, 16, 0, seed=k + n_long, n_long=n_long, long_len=long_len, front_starts=True)
    t, got, nc = run(k, g.records())
    assert nc == g.num_contigs and got == g.truth()


@pytest.mark.parametrize("k,long_last", [(51, True), (51, False), (19, True)])
def test_deferred_splitter_segments(monkeypatch, k, long_last):
    """Deferred splitter segments (k_walk_q, wb.split_min): contigs mostly shorter than the splitter
    spacing, so the walkers reaching the splitter walkers in the queue defer them, plus a few long
    chains that do stop at splitters. long_last puts the long chains' start records after every
    other record (their walkers start last: the splitter walkers are deferred first and walked by
    the second launch); otherwise they sit anywhere among the starts. Byte-equal to the oracle, and
    to the eager walk (KH_DEBUG=seg_eager: every walker stops at every walked splitter)."""
    # contigs of 2-16 k-mers (mean 9: below the walk's splitter spacing, 16 at this size)
    g = kh.SyntheticKmers(k, 2_000_000, 2, 16, 0, seed=61 + k, n_long=3, long_len=60_000)
    recs = g.records()
    if long_last:
        P = kh.packed_size(k)
        heads = {kh.pack_kmer(k, line[:k]).tobytes() for line in g.truth().split(b"\n") if len(line) > 10_000}
        rows = recs[:, :P]
        is_long = np.array([rows[i].tobytes() in heads for i in range(len(recs))])
        assert is_long.sum() == 3
        recs = np.concatenate([recs[~is_long], recs[is_long]])
    rc, want, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0
    _, got, got_nc = run(k, recs)
    assert got_nc == nc and got == want
    monkeypatch.setenv("KH_DEBUG", "seg_eager")
    _, got2, _ = run(k, recs)
    assert got2 == want


# ---- C5 hot-bucket half: many k-mers sharing a few minimizer windows (BASELINE configs[4]) -------
# kh_gen_create_hot plants one of a few shared M-mers in every k-mer of the hot contigs, so their
# k-mers share one minimizer window: one placement region before the table remaps it (k_hot_mark).
@pytest.mark.parametrize("mode", ["part", "cas"])
@pytest.mark.parametrize("k,n,lmax,hot,motifs,load,batches", [
    (51, 2_000_000, 200, 300, 4, 0.5, 1),     # 30 % of contigs on 4 motifs
    (51, 2_000_000, 200, 1000, 1, 0.5, 1),    # every k-mer shares ONE minimizer window
    (51, 1_500_000, 200, 300, 8, 0.85, 1),    # SURVEY C5's 0.85-load variant
    (51, 2_000_000, 200, 500, 2, 0.5, 3),     # later batches place keys with the first batch's remap
    # k=19, M=12: a hot k-mer has 7 free bases (8 phases x 4^7 = 131K distinct per motif), so a
    # family of ~5K k-mers (2x a region) in short contigs is what stays unique
    (19, 1_200_000, 20, 20, 1, 0.5, 1),
    (31, 1_000_000, 200, 500, 2, 0.7, 1),
])
def test_gpu_hot_minimizers_vs_oracle(monkeypatch, mode, k, n, lmax, hot, motifs, load, batches):
    monkeypatch.setenv("KH_INSERT", mode)
    g = kh.SyntheticKmers(k, n, 8, lmax, 10, seed=k * 31 + hot + motifs, hot_permille=hot, n_motifs=motifs)
    recs = g.records()
    rc, want, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0 and want == g.truth()
    t, got, gnc = run(k, recs, batches=batches, load=load)
    assert gnc == nc and got == want
    s = t.stats()
    assert s["n_full"] == s["n_dup"] == s["n_missing"] == 0
    if hot >= 300:
        assert s["n_hot_regions"] > 0      # the shared windows were remapped
    # find agrees with the oracle table on present keys of the hot contigs too
    P = (k + 3) // 4
    sel = recs[np.random.default_rng(k).choice(len(recs), 2000, replace=False)]
    out, found = t.find(sel[:, :P])
    assert found.all() and np.array_equal(out, sel)


@pytest.mark.parametrize("mode", ["part", "cas"])
@pytest.mark.parametrize("batches", [1, 3])
def test_gpu_hot_flank_vs_oracle(monkeypatch, mode, batches):
    """Families sharing the minimizer and its neighbour window (generator flank mode): level 2 of
    the remap spreads them; both insert paths and multi-batch inserts agree with the oracle, and
    find returns the exact records."""
    monkeypatch.setenv("KH_INSERT", mode)
    k, n = 51, 2_000_000
    g = kh.SyntheticKmers(k, n, 8, 200, 10, seed=77 + batches, hot_permille=300, n_motifs=4, hot_flank=True)
    recs = g.records()
    rc, want, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0 and want == g.truth()
    t, got, gnc = run(k, recs, batches=batches)
    assert gnc == nc and got == want
    s = t.stats()
    assert s["n_full"] == s["n_dup"] == s["n_missing"] == 0
    assert s["n_hot_regions"] > 0 and s["n_spread_regions"] > 0, s
    if mode == "part" and batches == 1:
        assert s["n_overflow"] < n // 100, s
    P = (k + 3) // 4
    sel = recs[np.random.default_rng(3).choice(len(recs), 2000, replace=False)]
    out, found = t.find(sel[:, :P])
    assert found.all() and np.array_equal(out, sel)


def test_gpu_hot_remap_off_is_not_needed_for_random_sets():
    """Random (non-repetitive) C3-shape input: no region is remapped; only probe runs that leave
    their slice near its end take the CAS path (a few per 10^4 keys at this table size)."""
    g = kh.SyntheticKmers(51, 4_000_000, 8, 200, 0, seed=51)
    t, got, _ = run(51, g.records())
    assert got == g.truth()
    s = t.stats()
    assert s["n_hot_regions"] == 0 and s["n_overflow"] < len(g.records()) // 1000
