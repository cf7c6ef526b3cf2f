"""CPU tests of the product library's host side (no kernels launched): C-ABI symbol surface,
host codec vs the reference KATs, text packing vs the oracle, and the synthetic generator."""
import hashlib
import json
import os

import numpy as np
import pytest

import cs267_hw3_amd as kh
from cs267_hw3_amd import _lib
import oracle_bind as ob

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT = json.load(open(os.path.join(GOLDEN, "kat.json")))
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    declared = _lib.declared_symbols()
    assert len(declared) >= 30
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    # every declared symbol is also bound with a signature in the Python stub
    assert sorted(_lib._SIGS) == declared
    assert L.kh_abi_version() == 3
    hdr = open(os.path.join(os.path.dirname(GOLDEN), "..", "include", "kmer_hash_amd.h")).read()
    for name in ("MSG_WORDS", "TEXT_REC_WORDS", "LINK_WORDS", "PRED_WORDS", "SEG_REC_WORDS"):
        assert f"#define KH_{name} {getattr(_lib, name)}" in hdr


@pytest.mark.parametrize("k", [1, 19, 29, 30, 31, 32, 51, 60])
def test_sizes(k):
    L = _lib.lib()
    assert L.kh_packed_size(k) == (k + 3) // 4          # packing.hpp:9
    assert L.kh_record_size(k) == (k + 3) // 4 + 2      # sizeof(kmer_pair), align 1
    assert L.kh_packed_size(61) < 0 and L.kh_record_size(0) < 0


@pytest.mark.parametrize("v", KAT, ids=[f"k{v['k']}-{v['kmer'][:8]}-{v['fb']}" for v in KAT])
def test_host_codec_kat(v):
    k = v["k"]
    p = kh.pack_kmer(k, v["kmer"])
    assert p.tobytes().hex() == v["packed"]
    assert kh.unpack_kmer(k, p) == v["kmer"]
    assert kh.djb2(k, p) == v["djb2"]
    if v["next"] is not None:
        rec = np.concatenate([p, np.frombuffer(v["fb"].encode(), np.uint8)])
        assert kh.next_kmer(k, rec).tobytes().hex() == v["next"]


def test_pack_rejects_non_acgt():
    with pytest.raises(kh.KmerHashError):
        kh.pack_kmer(19, "ACGTACGTACGTACGTACN")


def test_pack_every_byte_value():
    # the branch-free base decode (kh_codec.hpp base_code) against all 256 byte values: exactly
    # A C G T pack (to codes 0..3), anything else is rejected
    head = b"ACGTACGTACGTACGTAC"
    for b in range(256):
        s = head + bytes([b])
        if b in b"ACGT":
            got = kh.pack_kmer(19, s)
            # base i sits in byte i/4 at bits 7-2(i%4)..6-2(i%4) (packing.hpp:50-75): base 18 -> bits 3..2
            assert (got[-1] >> 2) & 3 == b"ACGT".index(b), b
        else:
            with pytest.raises(kh.KmerHashError):
                kh.pack_kmer(19, s)


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_pack_text_matches_oracle(name):
    k = MANIFEST[name]["k"]
    text = open(os.path.join(GOLDEN, f"{name}.txt"), "rb").read()
    assert np.array_equal(kh.pack_text(k, text), ob.parse_text(k, text))


def test_read_kmers_block_split(tmp_path):
    # read_kmers.hpp:55-58: rank r reads lines [r*ceil(n/P), ...)
    src = os.path.join(GOLDEN, "mixed19.txt")
    full = kh.read_kmers(src, 19)
    for P in (1, 2, 3, 7):
        parts = [kh.read_kmers(src, 19, P, r) for r in range(P)]
        assert np.array_equal(np.concatenate(parts), full)
    assert kh.kmer_size(src) == 19


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_generator_reproduces_committed_inputs(name):
    m = MANIFEST[name]
    g = kh.SyntheticKmers(m["k"], m["n"], m["len_min"], m["len_max"], m["single_permille"],
                          seed=m["seed"], shuffle=m["shuffle"])
    text = open(os.path.join(GOLDEN, f"{name}.txt"), "rb").read()
    assert hashlib.sha256(text).hexdigest() == m["input_sha256"]
    assert np.array_equal(g.records(), kh.pack_text(m["k"], text))
    # generator ground truth == reference-harness solution
    assert g.truth() == open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()
    assert g.num_contigs == m["contigs"]


def test_generator_ranges_and_truth_split():
    g = kh.SyntheticKmers(19, 50000, 5, 300, 30, seed=7)
    full = g.records()
    for P in (2, 3, 8):
        blocks = [g.block(P, r) for r in range(P)]
        assert np.array_equal(np.concatenate([g.records(b, e) for b, e in blocks]), full)
        # per-rank truth files concatenate to the same multiset (check_it.sh sorts)
        parts = b"".join(g.truth(b, e) for b, e in blocks)
        assert sorted(parts.splitlines()) == sorted(g.truth().splitlines())


def test_generator_unique_kmers_k19():
    # 200k random 19-mers would repeat ~0.07 times by chance; contigs holding a repeat are re-drawn
    g = kh.SyntheticKmers(19, 200000, 50, 400, 0, seed=11)
    keys = g.records()[:, :5]
    v = np.zeros(len(keys), np.uint64)
    for j in range(5):
        v = (v << np.uint64(8)) | keys[:, j].astype(np.uint64)
    assert len(np.unique(v)) == len(v)


def test_generator_matches_oracle_assembly():
    g = kh.SyntheticKmers(51, 40000, 8, 200, 10, seed=99)
    rc, text, nc, nl, _, _ = ob.assemble(51, g.records())
    assert rc == 0 and text == g.truth() and nc == g.num_contigs


def test_generator_unshuffled_is_contig_major():
    g = kh.SyntheticKmers(19, 1000, 10, 10, 0, seed=3, shuffle=False)
    r = g.records()
    assert all(r[i * 10, 5] == ord("F") for i in range(100))          # starts every 10 records
    assert all(r[i * 10 + 9, 6] == ord("F") for i in range(100))      # ends


@pytest.mark.parametrize("k,front", [(19, True), (51, True), (31, False)])
def test_skewed_generator_c5(k, front):
    """C5 skew (BASELINE configs[4]): long chains among short contigs, start k-mers first in
    record order; the oracle's assembly == the generator's truth, every block split included."""
    g = kh.SyntheticKmers(k, 150_000, 2, 16, 0, seed=k + 5, n_long=3, long_len=20_000, front_starts=front)
    recs = g.records()
    rc, text, nc, _, _, _ = ob.assemble(k, recs)
    assert rc == 0 and nc == g.num_contigs and text == g.truth()
    P = (k + 3) // 4
    starts = np.nonzero(recs[:, P] == ord("F"))[0]
    if front:
        assert starts.max() == g.num_contigs - 1      # all walkers in the first records
    assert b"".join(g.truth(*g.block(4, r)) for r in range(4)) == g.truth()
