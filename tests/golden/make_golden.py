"""Regenerates the committed golden vectors in tests/golden/ (run in the build container only).

Expected outputs come from the REFERENCE's own codec and I/O code: oracle/_ref/ref_harness_<K> is
compiled from /root/reference/{packing,pkmer_t,kmer_t,read_kmers}.hpp in place (oracle/Makefile),
with the world_size==1 driver loop of kmer_hash.cpp:21-55 restated around them.

  kat.json                  pack / djb2 / next_kmer vectors (reference codec)
  <name>.txt                inputs in the reference's fixed-width format (read_kmers.hpp:62-76),
                            drawn by the product generator (kh_gen_*) with the params in
                            manifest.json
  <name>_test_0.dat         reference-codec harness output for that input at one rank
                            (= test_0.dat of `kmer_hash_<K> <name>.txt test`, kmer_hash.cpp:60-68)

Usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import cs267_hw3_amd as kh  # noqa: E402

REF_DIR = os.path.join(ROOT, "oracle", "_ref")

# name: (k, n, len_min, len_max, single_permille, seed)
DATASETS = {
    "tiny19": (19, 3580, 3580, 3580, 0, 1),           # tiny.txt-like: one contig
    "verysmall19": (19, 20464, 1700, 2400, 0, 2),     # verysmall.txt-like: ~10 contigs
    "mixed19": (19, 8000, 1, 60, 100, 19),            # many short contigs + 10% single k-mers
    "small51": (51, 6000, 8, 200, 20, 51),            # human-chr14-like length mix
    "singles51": (51, 300, 1, 1, 1000, 5),            # every contig one k-mer ("FF")
    "k29": (29, 3000, 1, 120, 50, 29),                # last 8-byte-slot k
    "k30": (30, 3000, 1, 120, 50, 30),                # first 16-byte-slot k
    "k31": (31, 3000, 1, 120, 50, 31),
    "k32": (32, 3000, 1, 120, 50, 32),
    "k60": (60, 3000, 1, 120, 50, 60),                # largest supported k
}

KAT_KMERS = {
    19: [("AAAAAAAAAAAAAAAAAAA", "FC"), ("TTTTTTTTTTTTTTTTTTT", "AF"),
         ("ACGTACGTACGTACGTACG", "TA"), ("GATTACAGATTACAGATTA", "CG"),
         ("CCCCCCCCCCCCCCCCCCG", "GT"), ("TGCATGCATGCATGCATGC", "FF")],
    29: [("ACGTACGTACGTACGTACGTACGTACGTA", "CT"), ("T" * 29, "GA")],
    30: [("ACGTACGTACGTACGTACGTACGTACGTAC", "CT"), ("T" * 30, "GA")],
    31: [("GATTACA" * 4 + "GAT", "AC"), ("T" * 31, "GG")],
    32: [("GATTACA" * 4 + "GATT", "AC"), ("T" * 32, "CC")],
    51: [("A" * 51, "FC"), ("T" * 51, "AF"), ("ACGT" * 12 + "ACG", "TA"),
         ("GATTACA" * 7 + "GA", "CG"), ("C" * 50 + "G", "GT")],
    60: [("ACGT" * 15, "TA"), ("T" * 60, "AG"), ("GATTACA" * 8 + "GATT", "CF")],
}


def records_to_text(k, recs):
    lines = []
    P = (k + 3) // 4
    for r in recs:
        lines.append(kh.unpack_kmer(k, r[:P]) + " " + bytes(r[P:P + 2]).decode() + "\n")
    return "".join(lines).encode()


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    kat = []
    for k, items in KAT_KMERS.items():
        for kmer, fb in items:
            out = subprocess.run([os.path.join(REF_DIR, f"ref_harness_{k}"), "kat", kmer, fb],
                                 check=True, capture_output=True, text=True).stdout.split()
            kat.append({"k": k, "kmer": kmer, "fb": fb, "packed": out[0], "djb2": int(out[1]),
                        "next": None if out[2] == "-" else out[2]})
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    manifest = {}
    for name, (k, n, lmin, lmax, single, seed) in DATASETS.items():
        g = kh.SyntheticKmers(k, n, lmin, lmax, single, seed=seed)
        text = records_to_text(k, g.records())
        path = os.path.join(HERE, f"{name}.txt")
        with open(path, "wb") as f:
            f.write(text)
        sol = subprocess.run([os.path.join(REF_DIR, f"ref_harness_{k}"), "assemble", path],
                             check=True, capture_output=True).stdout
        with open(os.path.join(HERE, f"{name}_test_0.dat"), "wb") as f:
            f.write(sol)
        manifest[name] = {"k": k, "n": n, "len_min": lmin, "len_max": lmax,
                          "single_permille": single, "seed": seed, "shuffle": True,
                          "contigs": sol.count(b"\n"),
                          "input_sha256": hashlib.sha256(text).hexdigest(),
                          "solution_sha256": hashlib.sha256(sol).hexdigest()}
        print(name, manifest[name]["contigs"], "contigs", len(text), "bytes")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
