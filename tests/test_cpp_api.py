"""The C++ host surface (include/cs267_hw3_amd/*.hpp) on the GPU:
  * the stock single-key HashMap (README.md:95,99): insert / find / size / full,
  * the reference's own initialize_kmers + assemble_contigs + output_results loop
    (kmer_hash.cpp:21-68, one DistributedHashMap::find per step) at P = 1, 2, 3, 8 ranks,
  * the multi-rank DistributedHashMap through the drop-in driver (KH_RANKS=P ranks as threads on
    one GPU, kh::ThreadComm) and over a one-rank RCCL communicator,
  * the driver's stdout contract (kmer_hash.cpp:71-78, 143-145).
Each rank's <prefix>_<rank>.dat == the ground truth of its block (read_kmers.hpp:55-58) and the
sorted union == the reference-harness solution (scripts/check_it.sh semantics)."""
import json
import os
import re
import subprocess

import pytest

import cs267_hw3_amd as kh

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))
pytestmark = pytest.mark.gpu


def _exe(kind, k):
    return os.path.join(ROOT, "tools", f"kmer_hash_{k}") if kind == "driver" else \
        os.path.join(ROOT, "tests", "cpp", f"test_hash_map_{k}")


def _check_ranks(tmp_path, name, P, prefix="out"):
    m = MANIFEST[name]
    g = kh.SyntheticKmers(m["k"], m["n"], m["len_min"], m["len_max"], m["single_permille"], seed=m["seed"])
    parts = []
    for r in range(P):
        got = open(tmp_path / f"{prefix}_{r}.dat", "rb").read()
        b, e = g.block(P, r)
        assert got == g.truth(b, e), f"rank {r}"
        parts.append(got)
    want = open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()
    assert sorted(b"".join(parts).splitlines()) == sorted(want.splitlines())


@pytest.mark.parametrize("name,k", [("tiny19", 19), ("small51", 51)])
def test_stock_hashmap_surface(name, k):
    r = subprocess.run([_exe("test", k), "stock", os.path.join(GOLDEN, f"{name}.txt")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "stock ok" in r.stdout


@pytest.mark.parametrize("P", [1, 2, 3, 8])
@pytest.mark.parametrize("name,k", [("tiny19", 19), ("small51", 51)])
def test_reference_find_loop(tmp_path, name, k, P):
    """kmer_hash.cpp:38-55 as written: one find() per walk step, answered by the owner's table."""
    r = subprocess.run([_exe("test", k), "refloop", os.path.join(GOLDEN, f"{name}.txt"), str(P), "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    _check_ranks(tmp_path, name, P)


@pytest.mark.parametrize("P", [1, 2, 3, 8])
@pytest.mark.parametrize("name,k", [("tiny19", 19), ("small51", 51)])
def test_reference_find_loop_collective(tmp_path, name, k, P):
    """kmer_hash.cpp:38-55 without a peer group (the one-process-per-GPU protocol: every find() a
    collective round, process_requests() answering until all ranks are done) and without the
    caller's barriers: a find() right after insert_all relies on insert_all's own barrier."""
    r = subprocess.run([_exe("test", k), "refloopc", os.path.join(GOLDEN, f"{name}.txt"), str(P), "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    _check_ranks(tmp_path, name, P)


@pytest.mark.parametrize("name,k", [("tiny19", 19), ("small51", 51)])
def test_reference_find_loop_over_rccl(tmp_path, name, k):
    """The reference's find loop over RcclComm without a peer group, one rank (one process per GPU)."""
    r = subprocess.run([_exe("test", k), "rccl1loop", os.path.join(GOLDEN, f"{name}.txt"), "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert open(tmp_path / "out_0.dat", "rb").read() == \
        open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()


@pytest.mark.parametrize("P", [2, 3, 8])
@pytest.mark.parametrize("name,k", [("mixed19", 19), ("small51", 51), ("singles51", 51), ("k60", 60)])
def test_driver_multirank_threads(tmp_path, name, k, P):
    if not os.path.exists(_exe("driver", k)):
        pytest.skip(f"driver for k={k} not built")
    env = dict(os.environ, KH_RANKS=str(P), KH_COMM="thread")
    r = subprocess.run([_exe("driver", k), os.path.join(GOLDEN, f"{name}.txt"), "test", "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    _check_ranks(tmp_path, name, P)
    lines = r.stdout.splitlines()
    assert len(lines) == 1                       # BUtil::print: rank 0 only
    assert re.fullmatch(r"Rank 0 reconstructed \d+ contigs with \d+ nodes from 0 start nodes\. "
                        r"\(\d+\.\d{6} read, \d+\.\d{6} insert, \d+\.\d{6} total\)", lines[0])


@pytest.mark.parametrize("name,k", [("small51", 51), ("mixed19", 19)])
def test_sharded_over_rccl_one_rank(tmp_path, name, k):
    r = subprocess.run([_exe("test", k), "rccl1", os.path.join(GOLDEN, f"{name}.txt"), "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert open(tmp_path / "out_0.dat", "rb").read() == \
        open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()


def test_driver_summary_line(tmp_path):
    """kmer_hash.cpp:71-78: contigs = lines of test_0.dat, nodes = k-mers over all contigs."""
    name, k = "small51", 51
    r = subprocess.run([_exe("driver", k), os.path.join(GOLDEN, f"{name}.txt"), "test", "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    text = open(tmp_path / "out_0.dat", "rb").read()
    nc = text.count(b"\n")
    m = re.fullmatch(r"Rank 0 reconstructed (\d+) contigs with (\d+) nodes from 0 start nodes\. "
                     r"\((\S+) read, (\S+) insert, (\S+) total\)", r.stdout.strip())
    assert m and int(m.group(1)) == nc and int(m.group(2)) == MANIFEST[name]["n"]


@pytest.mark.parametrize("k,n,P,lmin,lmax", [(51, 64_000_000, 8, 8, 200), (51, 12_000_000, 3, 200, 1374),
                                             (19, 20_000_000, 5, 8, 400)])
def test_sharded_table_generated(k, n, P, lmin, lmax):
    """kh::ShardedTable at P ranks on generated data: per rank >= 4M records, so the insert takes
    the chunked path (transfers on the exchange stream, staged partitioning on the table's)."""
    r = subprocess.run([_exe("test", k), "gen", str(n), str(P), str(lmin), str(lmax)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gen ok" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("P", [2, 4])
def test_cpp_sharded_small_then_large(P):
    """kh::ShardedTable walks a small set, is cleared, walks one 100x larger, then the small one
    again on the same maps: slot capacities are learnt per input (walker count), every text
    equals its block's truth."""
    r = subprocess.run([_exe("test", 51), "gen2", "30000", "3000000", str(P)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gen2 ok" in r.stdout


@pytest.mark.parametrize("P", [1, 8])
def test_cpp_host_sharded_step_syncs(P):
    """The C++ host's sharded step (tools/kh_bench_cpp: clear + insert_all_dev + assemble) over P
    logical ranks on one GPU, C3 shape at 500K k-mers per rank: verified against the generator's
    truth, at most 8 blocking device reads per rank and step (count exchanges, the walk's end
    check, the library's own; ThreadComm's transport waits are not the protocol's), one check."""
    exe = os.path.join(ROOT, "tools", "kh_bench_cpp")
    if not os.path.exists(exe):
        pytest.skip("kh_bench_cpp not built")
    r = subprocess.run([exe, "--ranks", str(P), "--comm", "thread", "--n", "500000", "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["verified_vs_truth"] is True
    assert d["host_syncs_per_step_max"] <= 8, d
    assert d["walk_checks"] == 1, d
