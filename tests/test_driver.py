"""The drop-in C++ driver (tools/kmer_hash_<K>) reproduces the reference's test_<rank>.dat and
stdout contract (kmer_hash.cpp:60-79,143-148), and check_it.sh's sort-and-diff passes."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.mark.gpu
@pytest.mark.parametrize("name,k", [("tiny19", 19), ("verysmall19", 19), ("small51", 51)])
def test_driver_test_mode(tmp_path, name, k):
    exe = os.path.join(ROOT, "tools", f"kmer_hash_{k}")
    r = subprocess.run([exe, os.path.join(GOLDEN, f"{name}.txt"), "test", "out"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = open(tmp_path / "out_0.dat", "rb").read()
    want = open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()
    assert got == want
    assert sorted(got.splitlines()) == sorted(want.splitlines())  # check_it.sh semantics


@pytest.mark.gpu
def test_driver_timing_lines(tmp_path):
    exe = os.path.join(ROOT, "tools", "kmer_hash_19")
    r = subprocess.run([exe, os.path.join(GOLDEN, "mixed19.txt")], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0].startswith("Finished inserting in ") and lines[0].endswith(" sec")
    assert lines[1].startswith("Assembled in ") and lines[1].endswith(" total")


def test_driver_rejects_wrong_k(tmp_path):
    exe = os.path.join(ROOT, "tools", "kmer_hash_51")
    if not os.path.exists(exe):
        pytest.skip("driver not built")
    r = subprocess.run([exe, os.path.join(GOLDEN, "tiny19.txt")], cwd=tmp_path,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "19-mers" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["plain", "self_exchange", "self_exchange_pipelined"])
def test_dist_launcher_one_rank(tmp_path, mode):
    """cs267_hw3_amd.kmer_hash_dist under torchrun (1 rank, RCCL): same test_0.dat. The
    self-exchange modes run every exchange through RCCL anyway (the per-peer window views of the
    one-pass route, count exchanges, walker rounds; pipelined: chunked async all-to-alls)."""
    import sys
    env = dict(os.environ, PYTHONPATH=ROOT)
    if mode != "plain":
        env["KH_DIST_SELF_EXCHANGE"] = "1"
    if mode == "self_exchange_pipelined":
        env["KH_PIPELINE_MIN"] = "0"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
                        "--nproc-per-node", "1", "--master-addr", "127.0.0.1", "--master-port",
                        "29533", "-m", "cs267_hw3_amd.kmer_hash_dist",
                        os.path.join(GOLDEN, "small51.txt"), "test", "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    got = open(tmp_path / "out_0.dat", "rb").read()
    assert got == open(os.path.join(GOLDEN, "small51_test_0.dat"), "rb").read()
