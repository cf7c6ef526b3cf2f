"""The sharded SPMD driver (cs267_hw3_amd.dist) over a real torch.distributed gloo group on CPU,
with the oracle-backed test double shard: per-rank test_<rank>.dat == the ground truth of that
rank's block, and the union sorted == the reference harness output (scripts/check_it.sh)."""
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
MANIFEST = json.load(open(os.path.join(GOLDEN, "manifest.json")))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, name, outdir, chunk_bytes=None, insert_chunks=None, max_kmers=None,
               windows=False, slot_cap=None, steps=1):
    import sys
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import torch
    import torch.distributed as dist
    import cs267_hw3_amd as kh
    from cs267_hw3_amd.dist import DistributedKmerHashMap, TorchComm
    from dist_fake_shard import FakeShard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    k = MANIFEST[name]["k"]
    recs = kh.read_kmers(os.path.join(GOLDEN, f"{name}.txt"), k, world, rank)
    shard = FakeShard(k) if max_kmers is None else FakeShard(k, max_kmers=max_kmers if rank == 0 else 1 << 24)
    shard.route_windows = windows          # the one-pass route's owner-window layout
    dm = DistributedKmerHashMap(TorchComm(), shard)
    if insert_chunks:                      # pipelined insert: chunked route/exchange + staged build
        dm.INSERT_CHUNKS = insert_chunks
        dm.PIPELINE_MIN = 0
    if chunk_bytes:
        dm.A2A_CHUNK_BYTES = chunk_bytes   # force the chunked all-to-all path
    if slot_cap:
        dm.SLOT_CAP_MAX = slot_cap         # tiny exchange slots: walkers held back on their sender
    try:
        for step in range(steps):          # later steps size slots from the previous walk
            if step:
                shard.clear()
            dm.insert_all(torch.from_numpy(recs))
            rounds = dm.assemble(MANIFEST[name]["n"])
    except Exception as ex:                # every rank must fail together (no rank left waiting)
        with open(os.path.join(outdir, f"err_{rank}"), "w") as f:
            f.write(str(ex))
        dist.destroy_process_group()
        return
    with open(os.path.join(outdir, f"test_{rank}.dat"), "wb") as f:
        f.write(dm.contigs_text())
    with open(os.path.join(outdir, f"rounds_{rank}"), "w") as f:
        f.write(str(rounds))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world,chunk", [
    ("mixed19", 2, None), ("small51", 2, None), ("singles51", 2, None), ("small51", 3, None),
    ("small51", 3, 64), ("mixed19", 3, 1000), ("small51", 4, None)])
def test_sharded_driver_gloo(tmp_path, name, world, chunk):
    mp.start_processes(_rank_main, args=(world, _free_port(), name, str(tmp_path), chunk),
                       nprocs=world, join=True, start_method="spawn")
    import cs267_hw3_amd as kh
    m = MANIFEST[name]
    g = kh.SyntheticKmers(m["k"], m["n"], m["len_min"], m["len_max"], m["single_permille"],
                          seed=m["seed"])
    want = open(os.path.join(GOLDEN, f"{name}_test_0.dat"), "rb").read()
    parts = []
    for r in range(world):
        got = open(tmp_path / f"test_{r}.dat", "rb").read()
        b, e = g.block(world, r)
        assert got == g.truth(b, e)            # rank r walks the start k-mers of its block
        parts.append(got)
    assert sorted(b"".join(parts).splitlines()) == sorted(want.splitlines())
    rounds = {open(tmp_path / f"rounds_{r}").read() for r in range(world)}
    assert len(rounds) == 1                    # every rank ran the same number of rounds


@pytest.mark.parametrize("name,world,chunks", [("small51", 2, 3), ("mixed19", 3, 4), ("singles51", 2, 2)])
def test_sharded_pipelined_insert_gloo(tmp_path, name, world, chunks):
    """Pipelined insert over gloo: every chunk routed, the count matrix exchanged once, async
    all-to-alls, each received chunk staged while the next is in flight, one build at the end."""
    mp.start_processes(_rank_main, args=(world, _free_port(), name, str(tmp_path), None, chunks),
                       nprocs=world, join=True, start_method="spawn")
    import cs267_hw3_amd as kh
    m = MANIFEST[name]
    g = kh.SyntheticKmers(m["k"], m["n"], m["len_min"], m["len_max"], m["single_permille"],
                          seed=m["seed"])
    for r in range(world):
        b, e = g.block(world, r)
        assert open(tmp_path / f"test_{r}.dat", "rb").read() == g.truth(b, e)


def test_sharded_shard_full_fails_on_every_rank(tmp_path):
    """A shard that cannot hold what it is routed (rank 0 here) makes EVERY rank raise at the
    walk's first check (it still takes part in every exchange before it), instead of leaving the
    others blocked in the next collective."""
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), "small51", str(tmp_path), None, None, 3),
                       nprocs=world, join=True, start_method="spawn")
    errs = [open(tmp_path / f"err_{r}").read() for r in range(world)]
    assert "cannot hold" in errs[0]
    assert "another rank" in errs[1]


@pytest.mark.parametrize("name,world,chunk,chunks", [("small51", 2, None, None), ("mixed19", 3, 1000, None),
                                                     ("small51", 3, None, 3), ("mixed19", 2, None, 4)])
def test_sharded_route_windows_gloo(tmp_path, name, world, chunk, chunks):
    """The one-pass route's layout (each owner's words in its own window, not back to back):
    single and chunked all-to-all, and the pipelined insert, over gloo."""
    mp.start_processes(_rank_main, args=(world, _free_port(), name, str(tmp_path), chunk, chunks, None, True),
                       nprocs=world, join=True, start_method="spawn")
    import cs267_hw3_amd as kh
    m = MANIFEST[name]
    g = kh.SyntheticKmers(m["k"], m["n"], m["len_min"], m["len_max"], m["single_permille"],
                          seed=m["seed"])
    for r in range(world):
        b, e = g.block(world, r)
        assert open(tmp_path / f"test_{r}.dat", "rb").read() == g.truth(b, e)


@pytest.mark.parametrize("name,world,cap", [("small51", 3, 2), ("mixed19", 2, 5), ("small51", 4, 64)])
def test_sharded_tiny_slots_gloo(tmp_path, name, world, cap):
    """Exchange slots of a few messages: walkers past a slot's capacity are held back on their
    sender and go out in later rounds; two steps (the second sizes its slots from the first walk's
    per-round counts, still capped); every rank's text equals its block's truth."""
    mp.start_processes(_rank_main, args=(world, _free_port(), name, str(tmp_path), None, None, None, False, cap, 2),
                       nprocs=world, join=True, start_method="spawn")
    import cs267_hw3_amd as kh
    m = MANIFEST[name]
    g = kh.SyntheticKmers(m["k"], m["n"], m["len_min"], m["len_max"], m["single_permille"],
                          seed=m["seed"])
    for r in range(world):
        b, e = g.block(world, r)
        assert open(tmp_path / f"test_{r}.dat", "rb").read() == g.truth(b, e)


_HANG_SCRIPT = r"""
import os, sys, datetime
sys.path.insert(0, {tests!r}); sys.path.insert(0, {root!r})
import torch, torch.distributed as dist
import cs267_hw3_amd as kh
from cs267_hw3_amd.dist import DistributedKmerHashMap, TorchComm, StepWatchdog, guarded_step
from dist_fake_shard import FakeShard
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                        timeout=datetime.timedelta(seconds={pg_timeout}))
recs = torch.from_numpy(kh.read_kmers({path!r}, {k}, world, rank))
dm = DistributedKmerHashMap(TorchComm(), FakeShard({k}))
dm.HANG_AT = ({phase!r}, 1)
dog = StepWatchdog({step_timeout}, rank, lambda: dm.phase)
guarded_step(dm, dog, lambda: (dm.insert_all(recs), dm.assemble({n})))
print("finished", flush=True)
"""


@pytest.mark.parametrize("phase", ["walk_rounds", "counts"])
def test_sharded_hang_exits_nonzero(tmp_path, phase):
    """A rank that never reaches the next collective (stalled at the start of `phase`): the peer's
    collective times out with the process group (gloo, 4 s) and the stalled rank's StepWatchdog
    (8 s) ends it; both exit with StepWatchdog.EXIT_CODE within the limits, each naming the phase
    it was in — the behaviour an 8-GPU run needs when a collective hangs."""
    import subprocess
    import sys
    import time
    name = "small51"
    m = MANIFEST[name]
    script = _HANG_SCRIPT.format(tests=HERE, root=os.path.dirname(HERE), port=_free_port(), pg_timeout=4,
                                 path=os.path.join(GOLDEN, f"{name}.txt"), k=m["k"], n=m["n"], phase=phase,
                                 step_timeout=8)
    t0 = time.time()
    procs = [subprocess.Popen([sys.executable, "-c", script], env=dict(os.environ, RANK=str(r), WORLD_SIZE="2"),
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    elapsed = time.time() - t0
    from cs267_hw3_amd.dist import StepWatchdog
    for r, (p, (out, err)) in enumerate(zip(procs, outs)):
        assert p.returncode == StepWatchdog.EXIT_CODE, (r, p.returncode, err[-2000:])
        assert "finished" not in out
        assert f"[rank {r}]" in err and "phase '" in err, err[-2000:]
    assert f"phase '{phase}'" in outs[1][1]       # the stalled rank names where it stopped
    assert elapsed < 60
