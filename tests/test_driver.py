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
        env["KH_DIST_SELF_EXCHANGE"] = "pipelined" if mode == "self_exchange_pipelined" else "1"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
                        "--nproc-per-node", "1", "--master-addr", "127.0.0.1", "--master-port",
                        "29533", "-m", "cs267_hw3_amd.kmer_hash_dist",
                        os.path.join(GOLDEN, "small51.txt"), "test", "out"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    got = open(tmp_path / "out_0.dat", "rb").read()
    assert got == open(os.path.join(GOLDEN, "small51_test_0.dat"), "rb").read()


def _torchrun(P, port, args, cwd, env, timeout=300):
    import sys
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1",
                           "--nproc-per-node", str(P), "--master-addr", "127.0.0.1", "--master-port",
                           str(port)] + args, cwd=cwd, capture_output=True, text=True, timeout=timeout,
                          env=env)


def _shared_gpu_env():
    """P processes on the one GPU of the test box (KH_DIST_DEVICE=0), exchanging over gloo: RCCL
    refuses two ranks on one device, everything else (kernels, SPMD protocol, collectives, the
    launcher and bench's timing bracket) is the multi-GPU code path."""
    return dict(os.environ, PYTHONPATH=ROOT, KH_DIST_BACKEND="gloo", KH_DIST_DEVICE="0")


@pytest.mark.gpu
@pytest.mark.parametrize("name,P", [("small51", 2), ("small51", 4), ("verysmall19", 3)])
def test_dist_launcher_multiprocess(tmp_path, name, P):
    """P real processes (torchrun), one shard each: every rank writes its block's contigs in its
    start-node order (kmer_hash.cpp:60-68), so out_0.dat + ... + out_{P-1}.dat is the one-rank
    solution byte for byte (read_kmers.hpp:55-58 block split)."""
    r = _torchrun(P, 29541 + P, ["-m", "cs267_hw3_amd.kmer_hash_dist", os.path.join(GOLDEN, f"{name}.txt"),
                                 "test", "out"], tmp_path, _shared_gpu_env())
    assert r.returncode == 0, r.stderr[-3000:]
    got = b"".join(open(tmp_path / f"out_{q}.dat", "rb").read() for q in range(P))
    assert got == open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()
    assert f"Rank 0 reconstructed" in r.stdout


@pytest.mark.gpu
def test_bench_multiprocess(tmp_path):
    """bench.py's N > 1 line from 2 real processes: barrier + sync bracket, max over ranks, the
    ground-truth check on every rank, roofline and phases from rank 0."""
    import json
    r = _torchrun(2, 29551, [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--kmers", "2000000", "--steps", "2",
                             "--warmup", "1", "--no-cpu", "--e2e-steps", "0"], tmp_path, _shared_gpu_env())
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert line["n_gpus"] == 2 and line["verified_vs_truth"] is True
    assert line["config"]["n_kmers_total"] == 4_000_000 and line["value"] > 0


@pytest.mark.gpu
def test_bench_self_launch(tmp_path):
    """`python bench.py --gpus 2` with no outer torchrun (the way the driver calls --gpus 1):
    bench.py starts the 2 ranks itself as a torch.distributed.run child before any GPU call, and
    the line reports the communicator's world size."""
    import json
    import sys
    env = _shared_gpu_env()
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--kmers", "2000000",
                        "--steps", "2", "--warmup", "1", "--no-cpu", "--e2e-steps", "0"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert line["n_gpus"] == 2 and line["verified_vs_truth"] is True
    assert line["config"]["n_kmers_total"] == 4_000_000
    # the diagnosable N > 1 line: per-rank phase times (max / min over ranks), bytes sent to other
    # ranks per step, host syncs per step
    ph = line["rank_phases_ms"]
    # (a 2M-record block goes in one chunk: its partition and build are one phase)
    for name in ("route", "counts", "exchange_wait", "partition_build", "walk_rounds", "walk_exchange",
                 "text_group", "text_exchange", "materialize"):
        assert name in ph and ph[name]["max"] >= ph[name]["min"] >= 0, (name, ph)
    assert line["exchange_bytes_per_step"]["min"] > 0
    assert 1 <= line["host_syncs_per_step"]["max"] <= 12
    assert line["rank_step_ms"]["max"] > 0


def test_bench_world_size_mismatch_fails(tmp_path):
    """--gpus N under a launcher whose world size differs is an error, never a 1-GPU line
    (checked before anything touches a GPU)."""
    import sys
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


@pytest.mark.gpu
def test_bench_forced_one_rank_routed(tmp_path):
    """The forced one-rank sharded line (KH_BENCH_FORCE_DIST=1) also times the routed step
    (records through the one-pass route and the receiver's re-partition, as at P > 1) and checks
    its text against the ground truth."""
    import json
    r = _torchrun(1, 29553, [os.path.join(ROOT, "bench.py"), "--gpus", "1", "--kmers", "2000000", "--steps", "2",
                             "--warmup", "1", "--no-cpu", "--e2e-steps", "0"], tmp_path,
                  dict(os.environ, PYTHONPATH=ROOT, KH_BENCH_FORCE_DIST="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert line["n_gpus"] == 1 and line["verified_vs_truth"] is True
    ro = line["routed_one_rank"]
    assert ro["verified_vs_truth"] is True and ro["ms_per_step"] > 0
