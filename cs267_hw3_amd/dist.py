"""Sharded multi-GPU k-mer table + migrating-walker contig walk (one rank per GPU), Python host.

MI355X-native replacement of the reference's DistributedHashMap (hash_map.hpp:12-114) and its
UPC++ transport:
  owner = std::hash<string>(key) % P, one blocking RPC per target   hash_map.hpp:28-30,38-46,64-77
    -> owner = hash of the k-mer's minimizer (consecutive k-mers of a contig share it for ~19
       steps), ONE all-to-all of 8/16-B routed words, each shard sized from what it receives
  find(): one blocking RPC round trip per remote walk step           hash_map.hpp:83-107
    -> migrating walkers: a walker walks the local shard until its next k-mer is owned by another
       rank, then the walker itself (a 40-B message) moves there in the round's all-to-all;
       ~19 rounds at P=8 for C3 contigs. Appended bases go home in one more all-to-all.
    -> splitter segments (1 per ~256 k-mers) cut long chains (C2, C5) into segments walked in
       parallel and stitched by distributed pointer jumping (kh_mseg.hip)
  barrier() between phases                                           hash_map.hpp:79
Each rank's contig text is exactly its test_<rank>.dat: the contigs of the start k-mers in its
block (kmer_hash.cpp:41), in start-node order.

The SPMD driver below is written against two small interfaces so that the same code runs
  * on GPUs: GpuShard (C ABI kernels on torch device tensors) + TorchComm (torch.distributed;
    backend "nccl" is RCCL over xGMI),
  * on one GPU with P logical ranks: GpuShard + ThreadComm (tests, smoke),
  * on CPUs: a test double shard + TorchComm over gloo (tests/test_dist_cpu.py).
The C++ host of the same protocol is include/cs267_hw3_amd/dist_hash_map.hpp.
"""
import ctypes
import datetime
import faulthandler
import os
import sys
import threading
import time

import torch  # before the C ABI library is loaded: one HIP runtime for both

from . import _lib
from ._lib import check


# --------------------------------------------------------------------------------------------
# Communicators
# A collective that never completes (a rank that died or took another branch) must end the job,
# naming where it stopped: the process group times out after KH_DIST_TIMEOUT seconds (RCCL: torch's
# watchdog tears the communicator down, TORCH_NCCL_ASYNC_ERROR_HANDLING=1), and StepWatchdog ends a
# rank whose step outlives its limit, printing the phase it was in and every thread's stack.
DIST_TIMEOUT_S = float(os.environ.get("KH_DIST_TIMEOUT", "300"))


def init_rank_process_group(timeout_s=None):
    """One process per GPU: LOCAL_RANK's device, RCCL (backend "nccl") over xGMI. Returns the
    device index. Rehearsal of the multi-process path on a box with fewer GPUs than ranks:
    KH_DIST_DEVICE=<d> puts every local rank on device d and KH_DIST_BACKEND=gloo moves the
    exchanges through gloo (RCCL refuses two ranks on one GPU); the kernels, the SPMD protocol
    and its collectives are the same."""
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    shared = os.environ.get("KH_DIST_DEVICE")
    dev = int(shared) if shared else local
    torch.cuda.set_device(dev)
    backend = os.environ.get("KH_DIST_BACKEND", "nccl")
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    to = datetime.timedelta(seconds=timeout_s if timeout_s is not None else DIST_TIMEOUT_S)
    dist.init_process_group(backend, timeout=to,
                            device_id=torch.device("cuda", dev) if backend == "nccl" else None)
    return dev


class StepWatchdog:
    """Ends this rank (exit status 3) when a step outlives `limit_s`, after printing the phase the
    driver was in (DistributedKmerHashMap.phase) and every thread's Python stack: a stuck
    collective then names itself instead of hanging the job. faulthandler's own timer (which
    needs no GIL) backs it up 30 s later."""

    EXIT_CODE = 3

    def __init__(self, limit_s, rank, phase_of):
        self.limit_s = float(limit_s)
        self.rank = rank
        self.phase_of = phase_of
        self._timer = None

    def _fire(self):
        print(f"[rank {self.rank}] step exceeded {self.limit_s:.0f} s in phase "
              f"'{self.phase_of()}': exiting", file=sys.stderr, flush=True)
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        sys.stderr.flush()
        os._exit(self.EXIT_CODE)

    def arm(self):
        self.disarm()
        self._timer = threading.Timer(self.limit_s, self._fire)
        self._timer.daemon = True
        self._timer.start()
        faulthandler.dump_traceback_later(self.limit_s + 30, exit=True)

    def disarm(self):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
            faulthandler.cancel_dump_traceback_later()


def guarded_step(dm, dog, body):
    """Run one SPMD step under the watchdog; any exception (a collective that timed out, a peer's
    failure) ends this rank with StepWatchdog.EXIT_CODE after naming the driver's phase."""
    dog.arm()
    try:
        body()
    except Exception as ex:
        print(f"[rank {dog.rank}] step failed in phase '{dm.phase}': {ex!r}", file=sys.stderr, flush=True)
        sys.stderr.flush()
        os._exit(StepWatchdog.EXIT_CODE)
    dog.disarm()


class PhaseTimer:
    """Time of each driver phase on this rank's stream: mark(name) ends the interval named `name`
    (HIP events on the current stream, read after the step's synchronize; host clock on CPU)."""

    def __init__(self, cuda):
        self.cuda = cuda
        self.marks = []

    def reset(self):
        self.marks = []

    def mark(self, name):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append((name, e))
        else:
            self.marks.append((name, time.perf_counter()))

    def totals(self):
        """{phase: ms} summed over the step's intervals (call after synchronize)."""
        out, prev = {}, None
        for name, e in self.marks:
            if prev is not None:
                dt = prev.elapsed_time(e) if self.cuda else 1e3 * (e - prev)
                out[name] = out.get(name, 0.0) + dt
            prev = e
        return out


class TorchComm:
    """torch.distributed process group (nccl = RCCL over xGMI on MI355X, or gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        # processes sharing one GPU (KH_DIST_DEVICE rehearsals) split its free memory
        self.ranks_per_device = int(os.environ.get("LOCAL_WORLD_SIZE", "1")) if os.environ.get(
            "KH_DIST_DEVICE") else 1

    def all_to_all_async(self, out, inp, out_splits, in_splits):
        return self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group, async_op=True)

    def all_to_all(self, out, inp, out_splits, in_splits):
        self.dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def all_to_all_list(self, outs, inps):
        """Per-peer views in and out (no packing copies); RCCL runs it as grouped send/recv."""
        if self.backend != "nccl":
            raise NotImplementedError
        self.dist.all_to_all(outs, inps, group=self.group)

    def all_to_all_views_async(self, outs, inps):
        """Per-peer input views (not back to back: the one-pass route's owner windows) into
        per-peer output views. RCCL: grouped send/recv straight from the views; other backends:
        packed through one all_to_all_single, unpacked at wait()."""
        if self.backend == "nccl":
            return self.dist.all_to_all(outs, inps, group=self.group, async_op=True)
        send, recv = _pack_views(inps, outs)
        w = self.dist.all_to_all_single(recv, send, [o.numel() for o in outs], [i.numel() for i in inps],
                                        group=self.group, async_op=True)
        return _UnpackOnWait(w, recv, outs)

    def barrier(self):
        self.dist.barrier(group=self.group)

    def all_gather(self, out, inp):
        """Equal-size blocks: rank q's inp lands at out[q * inp.numel() ...]."""
        if self.backend == "nccl":
            self.dist.all_gather_into_tensor(out, inp, group=self.group)
        else:
            self.dist.all_gather(list(out.view(self.world, -1).unbind(0)), inp, group=self.group)

    def max_to_host(self, t):
        """Element-wise max over ranks of a small int64 tensor, read on the host (ONE device read)."""
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return t.cpu()

    def all_reduce_max(self, x):
        t = torch.tensor([float(x)], dtype=torch.float64)
        if self.dist.get_backend(self.group) == "nccl":
            t = t.cuda()
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return float(t.item())


def _pack_views(inps, outs):
    like = inps[0] if inps else outs[0]
    send = torch.cat(list(inps)) if len(inps) > 1 else inps[0].contiguous()
    recv = torch.empty(sum(o.numel() for o in outs), dtype=like.dtype, device=like.device)
    return send, recv


class _UnpackOnWait:
    def __init__(self, work, recv, outs):
        self.work, self.recv, self.outs = work, recv, outs

    def wait(self):
        if self.work is not None:
            self.work.wait()
        pos = 0
        for o in self.outs:
            if o.numel():
                o.copy_(self.recv[pos:pos + o.numel()])
            pos += o.numel()


class ThreadComm:
    """P logical ranks as P threads of one process (one GPU): all_to_all through shared memory."""

    class _Shared:
        def __init__(self, world):
            self.world = world
            self.barrier = threading.Barrier(world)
            self.slots = [None] * world

    @classmethod
    def group(cls, world):
        sh = cls._Shared(world)
        return [cls(sh, r) for r in range(world)]

    def __init__(self, shared, rank):
        self.sh = shared
        self.rank = rank
        self.world = shared.world
        self.ranks_per_device = shared.world  # every logical rank shares the one GPU

    class _Done:
        def wait(self):
            pass

    def all_to_all_async(self, out, inp, out_splits, in_splits):
        self.all_to_all(out, inp, out_splits, in_splits)
        return ThreadComm._Done()

    def _sync(self, t):
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()

    def all_to_all_views_async(self, outs, inps):
        send, recv = _pack_views(inps, outs)
        self.all_to_all(recv, send, [o.numel() for o in outs], [i.numel() for i in inps])
        _UnpackOnWait(None, recv, outs).wait()
        return ThreadComm._Done()

    def all_to_all(self, out, inp, out_splits, in_splits):
        self._sync(inp)
        self.sh.slots[self.rank] = (inp, list(in_splits))
        self.sh.barrier.wait()
        parts = []
        for q in range(self.world):
            src, splits = self.sh.slots[q]
            a = sum(splits[:self.rank])
            parts.append(src[a:a + splits[self.rank]])
        if parts:
            got = torch.cat(parts) if len(parts) > 1 else parts[0]
            out.copy_(got)
        self._sync(out)
        self.sh.barrier.wait()

    def barrier(self):
        self.sh.barrier.wait()

    def all_gather(self, out, inp):
        self._sync(inp)
        self.sh.slots[self.rank] = inp
        self.sh.barrier.wait()
        n = inp.numel()
        for q in range(self.world):
            out[q * n:(q + 1) * n].copy_(self.sh.slots[q])
        self._sync(out)
        self.sh.barrier.wait()

    def max_to_host(self, t):
        h = t.cpu()
        self.sh.slots[self.rank] = h
        self.sh.barrier.wait()
        m = torch.stack(list(self.sh.slots)).max(0).values
        self.sh.barrier.wait()
        return m

    def all_reduce_max(self, x):
        self.sh.slots[self.rank] = x
        self.sh.barrier.wait()
        m = max(self.sh.slots)
        self.sh.barrier.wait()
        return m


# --------------------------------------------------------------------------------------------
# Local shard on this rank's GPU (C ABI kernels)
class GpuShard:
    """This rank's table + walker state on its GPU; buffers are torch device tensors."""

    def __init__(self, k, n_kmers, device=0, load_factor=0.5):
        from .hashmap import KmerHashTable, record_size
        self.k = k
        self.R = record_size(k)
        self.dev = torch.device("cuda", device)
        self.table = KmerHashTable(k, n_kmers, load_factor, device=device)
        self.L = _lib.lib()
        self.W = self.L.kh_word_count(k)
        self.h = self.table._h
        self.n_kmers = n_kmers
        self.n_table = n_kmers  # the table's sizing (kh_create, grown by reserve)
        self.stream = torch.cuda.Stream(device=self.dev)
        self.table.set_stream(self.stream.cuda_stream)
        self.inserted = 0  # k-mers the shard holds since the last clear

    @staticmethod
    def _p(t):
        return ctypes.c_void_p(t.data_ptr())

    def zeros(self, n, dtype):
        return torch.empty(max(int(n), 1), dtype=dtype, device=self.dev)

    def clear(self):
        self.table.clear()
        self.inserted = 0

    def collect_starts(self, recs):
        check(self.L.kh_collect_starts_dev(self.h, self._p(recs), recs.shape[0]))

    def route(self, recs, nranks, words=None, starts=False):
        """Records -> owner-grouped words (+ counts); starts=True also collects this block's
        start k-mers in the same pass (kh_route_starts_dev)."""
        n = recs.shape[0]
        if words is None:
            words = self.zeros(n * self.W, torch.int64)
        counts = self.zeros(nranks + 1, torch.int64)
        f = self.L.kh_route_starts_dev if starts else self.L.kh_route_dev
        check(f(self.h, self._p(recs), n, nranks, self._p(words), self._p(counts)))
        return words, counts

    @property
    def route_windows(self):  # route_win: one pass over records of <= 15 bytes into owner windows
        return self.R <= 15

    def route_win(self, recs, nranks, words, win):
        """Records -> owner q's words at words[q * win * W ...] (one pass, kh_route_starts_win_dev;
        win >= the records routed) + this block's start k-mers; returns the [P+1] counts."""
        counts = self.zeros(nranks + 1, torch.int64)
        check(self.L.kh_route_starts_win_dev(self.h, self._p(recs), recs.shape[0], nranks, self._p(words), int(win),
                                             self._p(counts)))
        return counts

    def reserve(self, m):
        """Room for m more k-mers: an empty shard grows to them (kh_reserve); a non-empty one must
        already have the room (kh_reserve fails otherwise: the caller's ranks agree on it)."""
        check(self.L.kh_reserve(self.h, int(self.inserted + m)))
        self.n_table = max(self.n_table, int(self.inserted + m))

    def insert_records(self, recs):
        """One rank: the route is the identity, so the block's records go straight through the
        single-GPU records pass (kh_insert_dev: start k-mers and splitters in the same pass)."""
        n = recs.shape[0]
        check(self.L.kh_insert_dev(self.h, self._p(recs), n))
        self.inserted += n

    def insert_words(self, words, m):
        check(self.L.kh_insert_words_dev(self.h, self._p(words), m))
        self.inserted += m

    def stage_words(self, words, m, total):
        """Partition m received words toward one build of <= total (kh_insert_words_stage_dev)."""
        check(self.L.kh_insert_words_stage_dev(self.h, self._p(words), m, total))
        self.inserted += m

    def finish_words(self):
        check(self.L.kh_insert_words_finish(self.h))

    def counters(self):
        """[start k-mers, splitter k-mers] collected so far (device int64[2], async)."""
        out = self.zeros(2, torch.int64)
        check(self.L.kh_counters_dev(self.h, self._p(out)))
        return out

    def counters_host(self):
        """[start k-mers, splitter k-mers] on the host (blocking; after insert_records it waits for
        the copy made beside the build, not for the build)."""
        v = (ctypes.c_uint64 * 2)()
        check(self.L.kh_counters(self.h, v))
        return [int(v[0]), int(v[1])]

    def route_splitters(self, nranks):
        """Splitter k-mers this rank's routes sent to each owner (device int64[P], async)."""
        out = self.zeros(nranks, torch.int64)
        check(self.L.kh_route_splitters_dev(self.h, self._p(out), nranks))
        return out

    def host_syncs(self):
        v = ctypes.c_uint64(0)
        check(self.L.kh_host_syncs(self.h, ctypes.byref(v)))
        return v.value

    # migrating-walker rounds (fixed-size exchange slots: no device read per round)
    MSG_WORDS = _lib.MSG_WORDS
    TEXT_REC_WORDS = _lib.TEXT_REC_WORDS

    def mw_begin(self, nranks, rank, total_kmers, n_starts, n_splitters, total_walkers):
        nw = ctypes.c_uint64(0)
        check(self.L.kh_mwalk_begin(self.h, nranks, rank, total_kmers, n_starts, n_splitters, total_walkers,
                                    ctypes.byref(nw)))
        self.nranks = nranks
        return nw.value

    def mw_round(self, inp, cap_in, out, cap_out, live):
        """inp: the received slots (None: the first round); out: P slots of cap_out; live: int64[2]."""
        check(self.L.kh_mwalk_round_dev(self.h, self._p(inp) if inp is not None else None, cap_in, self._p(out),
                                        cap_out, self._p(live)))

    def mw_text_bound(self):
        v = ctypes.c_uint64(0)
        check(self.L.kh_mwalk_text_bound(self.h, ctypes.byref(v)))
        return v.value

    def mw_text(self, out):
        counts = self.zeros(self.nranks + 1, torch.int64)
        check(self.L.kh_mwalk_text_dev(self.h, self._p(out), self._p(counts)))
        return counts

    def mw_end(self, recs, n):
        check(self.L.kh_mwalk_end_dev(self.h, self._p(recs), n))

    def mw_flags(self):
        """Device int64[2] (async): [overlap / overflow reports of this walk, store records needed]."""
        out = self.zeros(2, torch.int64)
        check(self.L.kh_mwalk_flags_dev(self.h, self._p(out)))
        return out

    def mw_redo(self, store_records):
        check(self.L.kh_mwalk_redo(self.h, int(store_records)))

    def mw_short(self, total_kmers, total_starts):
        """Arm the next walk as a short walk (no splitter segments, long contigs reported) where the
        mean contig is shorter than the splitter spacing; True when armed."""
        if not hasattr(self.L, "kh_mwalk_short"):
            return False
        armed = ctypes.c_int(0)
        check(self.L.kh_mwalk_short(self.h, int(total_kmers), int(total_starts), ctypes.byref(armed)))
        return bool(armed.value)

    def mw_abandon(self):
        check(self.L.kh_mwalk_abandon(self.h))

    # splitter segments of the migrating walk (kh_mseg.hip)
    LINK_WORDS = _lib.LINK_WORDS
    PRED_WORDS = _lib.PRED_WORDS
    SEG_REC_WORDS = _lib.SEG_REC_WORDS

    def mw_segments(self):
        v = ctypes.c_uint64(0)
        check(self.L.kh_mwalk_segments(self.h, ctypes.byref(v)))
        return v.value

    def mw_link(self, recs, n, out):
        counts = self.zeros(self.nranks + 1, torch.int64)
        check(self.L.kh_mwalk_link_dev(self.h, self._p(recs), n, self._p(out), self._p(counts)))
        return counts

    def mw_pred(self, links, m, preds, stride):
        check(self.L.kh_mwalk_pred_dev(self.h, self._p(links), m, self._p(preds), stride))

    def mw_resolve(self, all_preds, stride):
        check(self.L.kh_mwalk_resolve_dev(self.h, self._p(all_preds), stride))

    def mw_retag(self, recs, n, out):
        counts = self.zeros(self.nranks + 1, torch.int64)
        check(self.L.kh_mwalk_retag_dev(self.h, self._p(recs), n, self._p(out), self._p(counts)))
        return counts

    def mw_end_seg(self, recs, n, seg, m):
        check(self.L.kh_mwalk_end_seg_dev(self.h, self._p(recs), n, self._p(seg), m))

    def sync(self):
        self.table.sync()

    def contigs_text(self):
        return self.table.contigs_text()

    def stats(self):
        return self.table.stats()


# --------------------------------------------------------------------------------------------
class DistributedKmerHashMap:
    """hash_map.hpp DistributedHashMap + kmer_hash.cpp assemble_contigs across ranks (SPMD).

    insert_all(recs): recs = this rank's block of kmer_pair records (read_kmers.hpp:55-58),
                      collective (hash_map.hpp:55-80 ends in a barrier too).
    assemble(total):  walk this rank's start k-mers; returns this rank's contig text
                      (= test_<rank>.dat bytes); collective.
    """

    def __init__(self, comm, shard):
        self.comm = comm
        self.shard = shard
        self.P = comm.world
        self.rounds = 0
        self.checks = 0
        self.syncs = 0          # host reads of device data by this host since the last reset
        self._caps = []         # per-round slot capacities learnt from the last assemble
        self._caps_walkers = 0  # ... whose walker count (another count: another input, not used)
        self._cap_floor = 0     # this assemble: the demand of rounds that held messages back
        self._rounds_hint = 0   # its round count (the next assemble checks for the end there first)
        self.phase = "idle"     # the driver phase running now (StepWatchdog names it on a hang)
        self._cur = None
        self.timer = None       # a PhaseTimer: per-phase stream time of the step (bench)
        self.xbytes = 0         # bytes this rank sent to other ranks in the step (all exchanges)
        self.text_records = self.seg_records = 0  # text / retag records received by the last walk

    # tests: stall this rank when it begins phase HANG_AT[0] (HANG_AT[1] = the rank) — a rank that
    # never reaches the next collective, as a crashed or diverged peer would look to the others
    HANG_AT = None

    def _begin(self, name):
        """Phase `name` begins (and the one before it ends: the timer labels the interval)."""
        if self.timer is not None:
            self.timer.mark(self._cur)
        self._cur = name
        self.phase = name
        if self.HANG_AT is not None and tuple(self.HANG_AT) == (name, self.comm.rank):
            time.sleep(3600)

    def _end(self):
        if self.timer is not None and self._cur is not None:
            self.timer.mark(self._cur)
        self._cur = None
        self.phase = "idle"

    def _sent(self, splits, elem_bytes):
        """Count the bytes of an exchange's splits that leave this rank (not its own block)."""
        self.xbytes += sum(int(x) for q, x in enumerate(splits) if q != self.comm.rank) * elem_bytes

    def close(self):
        pass

    def host_syncs(self):
        """Blocking device reads so far: this host's plus the shard library's own (kh_host_syncs)."""
        lib = self.shard.host_syncs() if hasattr(self.shard, "host_syncs") else 0
        return self.syncs + lib

    def _host(self, t):
        """A device tensor read on the host: one blocking round trip (counted)."""
        self.syncs += 1
        return t.cpu()

    def _int64(self, like, n):
        return torch.empty(max(int(n), 1), dtype=torch.int64, device=like.device)

    # One-rank self send/recv through RCCL loses everything past the first half of a message of
    # >= 2 GiB - 8 B (tools/rccl_big_msg.cpp and .py; profiles/r04/rccl_big_msg: RCCL 2.27.7 and
    # torch's 2.26.6, equal and split all_to_all and grouped send/recv alike; exact at 1 GiB), so
    # no single call moves more than A2A_CHUNK_BYTES per peer.
    A2A_CHUNK_BYTES = 512 << 20
    # one rank: exchanges are skipped (KH_DIST_SELF_EXCHANGE=1 runs them anyway, for tests;
    # =pipelined also in chunks at any size), and the records go straight into the records pass
    # (KH_DIST_ROUTE_ONE_RANK=1 routes them anyway)
    SELF_EXCHANGE = os.environ.get("KH_DIST_SELF_EXCHANGE", "0") in ("1", "pipelined")
    ROUTE_ONE_RANK = os.environ.get("KH_DIST_ROUTE_ONE_RANK") == "1"

    def _exchange_counts(self, counts, extra=None):
        """counts: [P+1] int64 (per-destination, total) -> (send_splits, recv_splits, totals,
        global max per-peer split, extras). One small all-to-all and ONE host read; each rank also
        learns every rank's total and largest split (chunk count), and `extra` (a device int64
        scalar of this rank, e.g. its splitter count) of every rank."""
        P = self.P
        if P == 1 and not self.SELF_EXCHANGE:
            # one rank: the exchange is the identity; read the counts (and extra) as they are
            h = self._host(counts[:2] if extra is None else torch.cat([counts[:2], extra.reshape(1)])).tolist()
            return [h[0]], [h[0]], [h[1]], h[0], [h[2] if extra is not None else 0]
        mx = counts[:P].max().reshape(1)
        ex = extra.reshape(1) if extra is not None else mx.new_zeros(1)
        send = torch.stack([counts[:P], counts[P:P + 1].expand(P), mx.expand(P), ex.expand(P)], 1)
        send = send.contiguous().view(-1)
        recv = torch.empty_like(send)
        self._sent([4] * P, 8)
        self.comm.all_to_all(recv, send, [4] * P, [4] * P)
        host = self._host(torch.cat([send, recv])).view(2, P, 4)
        send_splits = host[0, :, 0].tolist()
        recv_splits = host[1, :, 0].tolist()
        totals = host[1, :, 1].tolist()
        gmax = int(host[1, :, 2].max())
        extras = host[1, :, 3].tolist()
        return send_splits, recv_splits, totals, gmax, extras

    def _all_to_all(self, out, inp, out_splits, in_splits, gmax_elems, in_off=None):
        """all_to_all_single in chunks of at most A2A_CHUNK_BYTES per peer. gmax_elems is the
        largest per-peer split over ALL ranks, so every rank runs the same number of calls.
        in_off: where each peer's input starts (the route's owner windows; default back to back)."""
        limit = max(1, self.A2A_CHUNK_BYTES // inp.element_size())
        rounds = (gmax_elems + limit - 1) // limit
        P = self.P
        self._sent(in_splits, inp.element_size())
        if rounds <= 1 and in_off is None:
            self.comm.all_to_all(out, inp, out_splits, in_splits)
            return
        out_off = [0] * P
        for q in range(1, P):
            out_off[q] = out_off[q - 1] + out_splits[q - 1]
        if in_off is None:
            in_off = [0] * P
            for q in range(1, P):
                in_off[q] = in_off[q - 1] + in_splits[q - 1]
        if rounds <= 1:
            self.comm.all_to_all_views_async([out[out_off[q]:out_off[q] + out_splits[q]] for q in range(P)],
                                             [inp[in_off[q]:in_off[q] + in_splits[q]] for q in range(P)]).wait()
            return
        if getattr(self.comm, "backend", None) == "nccl":
            # views straight into the packed buffers: no staging copies
            for r in range(rounds):
                lo = r * limit
                sc = [max(0, min(limit, in_splits[q] - lo)) for q in range(P)]
                rc = [max(0, min(limit, out_splits[q] - lo)) for q in range(P)]
                self.comm.all_to_all_list(
                    [out[out_off[q] + lo:out_off[q] + lo + rc[q]] for q in range(P)],
                    [inp[in_off[q] + lo:in_off[q] + lo + sc[q]] for q in range(P)])
            return
        for r in range(rounds):
            lo = r * limit
            sc = [max(0, min(limit, in_splits[q] - lo)) for q in range(P)]
            rc = [max(0, min(limit, out_splits[q] - lo)) for q in range(P)]
            parts = [inp[in_off[q] + lo:in_off[q] + lo + sc[q]] for q in range(P) if sc[q]]
            send = torch.cat(parts) if parts else inp[:0]
            recv = torch.empty(sum(rc), dtype=out.dtype, device=out.device)
            self.comm.all_to_all(recv, send, rc, sc)
            pos = 0
            for q in range(P):
                if rc[q]:
                    out[out_off[q] + lo:out_off[q] + lo + rc[q]].copy_(recv[pos:pos + rc[q]])
                    pos += rc[q]

    # pipelined insert: chunk c-1, received, is partitioned while chunk c is on the wire
    # (tests set INSERT_CHUNKS / PIPELINE_MIN on the instance)
    INSERT_CHUNKS = 4
    ROUTE_WINDOW_BYTES = 64 << 30
    # records per rank below which one chunk
    PIPELINE_MIN = 0 if os.environ.get("KH_DIST_SELF_EXCHANGE") == "pipelined" else 1 << 22

    def _exchange_count_matrix(self, counts, spl, mine):
        """counts: list over chunks of [P+1] int64 device tensors (per-destination, total); spl:
        splitter k-mers routed to each owner [P]; mine: this rank's [start k-mers, splitters it
        routed] -> (send[c][q], recv[c][q], global max per-peer split, splitters this rank owns,
        walkers and splitters of all ranks). One small all-to-all and ONE host read for all chunks."""
        P, nch = self.P, len(counts)
        mat = torch.stack([c[:P] for c in counts])            # [nch, P]
        mx = mat.max().reshape(1)
        cols = [mat.t(), mx.expand(P).reshape(P, 1), spl[:P].reshape(P, 1),
                mine[:2].reshape(1, 2).expand(P, 2)]
        send = torch.cat(cols, 1).contiguous().view(-1)       # [P, nch + 4]
        w = nch + 4
        if P == 1 and not self.SELF_EXCHANGE:
            recv = send
        else:
            recv = torch.empty_like(send)
            self._sent([w] * P, 8)
            self.comm.all_to_all(recv, send, [w] * P, [w] * P)
        host = self._host(torch.cat([send, recv])).view(2, P, w)
        send_c = [[int(host[0, q, c]) for q in range(P)] for c in range(nch)]
        recv_c = [[int(host[1, q, c]) for q in range(P)] for c in range(nch)]
        gmax = int(host[1, :, nch].max())
        nsp = int(host[1, :, nch + 1].sum())                  # splitters routed to this rank
        walkers = int(host[1, :, nch + 2].sum() + host[1, :, nch + 3].sum())
        splitters = int(host[1, :, nch + 3].sum())
        starts = int(host[1, :, nch + 2].sum())
        return send_c, recv_c, gmax, int(host[0, 0, nch + 2]), nsp, walkers, splitters, starts

    def insert_all(self, recs):
        """Route every record to its owner (+ this block's start k-mers), learn the per-chunk
        counts in one exchange, size the shard from what it receives (kh_reserve; minimizer
        ownership can be skewed on repetitive inputs), then move the words, partitioning each
        received chunk while the next one is on the wire; one build at the end. A shard that
        cannot be sized still takes part in every exchange; every rank raises together at the
        walk's first check (one host read fewer than agreeing here)."""
        sh, P, W = self.shard, self.P, self.shard.W
        n = recs.shape[0]
        exchange = P > 1 or self.SELF_EXCHANGE
        self._err = None
        if self.timer is not None:  # a step = insert_all + assemble
            self.timer.reset()
            self._cur = None
        self.xbytes = 0
        if not exchange and not self.ROUTE_ONE_RANK and hasattr(sh, "insert_records"):
            # one rank: every key is this shard's and nothing moves (as the count exchanges are
            # skipped): the records pass partitions them itself, no owner route + word re-partition
            self._begin("insert")
            sh.reserve(n)
            sh.insert_records(recs)
            self._begin("counts")
            if hasattr(sh, "counters_host") and hasattr(sh.L, "kh_counters"):  # start / splitter counts
                c = sh.counters_host()         # (the library counts this read: kh_host_syncs)
            else:
                c = self._host(sh.counters())
            self._ns, self._nsp = int(c[0]), int(c[1])
            self._walkers, self._splitters = self._ns + self._nsp, self._nsp
            self._starts_all = self._ns
            return n
        nch = 1
        if exchange and self.INSERT_CHUNKS > 1 and n >= self.PIPELINE_MIN:
            # per-peer bytes of a chunk <= chunk records * W * 8: keep every transfer under the
            # per-peer message limit whatever the skew
            nch = max(self.INSERT_CHUNKS, -(-n * W * 8 // self.A2A_CHUNK_BYTES))
        # chunk starts at multiples of 16 records: every chunk's records stay 16-B aligned
        bounds = [min(n, (n * c // nch) & ~15) for c in range(nch)] + [n]
        # one-pass route into per-owner windows (each sized for the whole chunk, so any skew fits)
        # while P windows of the block fit the budget; the two-pass route packs back to back
        windows = getattr(sh, "route_windows", False) and P * n * W * 8 <= self.ROUTE_WINDOW_BYTES
        if windows and recs.is_cuda:  # and a third of this rank's share of what is free
            have = getattr(self, "_ins_words", None)
            have = have.numel() * 8 if have is not None and have.device == recs.device else 0
            share = getattr(self.comm, "ranks_per_device", 1)  # P logical ranks on one GPU
            windows = P * n * W * 8 <= have + torch.cuda.mem_get_info(recs.device)[0] // (3 * share)
        if windows:
            # one-pass route: chunk c's owner windows of (c1 - c0) words each at P * c0 words
            words = self._grow("_ins_words", max(P * n, 1) * W, torch.int64, recs.device, slack=1.0)
        else:
            words = self._grow("_ins_words", max(n, 1) * W, torch.int64, recs.device)
        counts = []
        self._begin("route")
        for c in range(nch):
            c0, c1 = bounds[c], bounds[c + 1]
            if windows:
                counts.append(sh.route_win(recs[c0:c1], P, words[P * c0 * W:], max(c1 - c0, 1)))
            else:
                counts.append(sh.route(recs[c0:c1], P, words[c0 * W:max(c1, c0 + 1) * W], starts=True)[1])

        def views(c, send):  # chunk c's per-peer input (window starts, or back to back)
            c0, c1 = bounds[c], bounds[c + 1]
            if windows:
                offs = [(P * c0 + q * max(c1 - c0, 1)) * W for q in range(P)]
            else:
                offs = [c0 * W + sum(send[:q]) * W for q in range(P)]
            return [words[offs[q]:offs[q] + send[q] * W] for q in range(P)], offs
        self._begin("counts")
        spl = sh.route_splitters(P)
        cnt = sh.counters()
        mine = torch.stack([cnt[0], spl[:P].sum()])
        send_c, recv_c, gmax, self._ns, self._nsp, self._walkers, self._splitters, self._starts_all = \
            self._exchange_count_matrix(counts, spl, mine)
        m = sum(sum(r) for r in recv_c)
        ok = True
        try:
            sh.reserve(m)
        except RuntimeError as ex:  # KmerHashError (NOMEM) or a test shard's error
            self._err, ok = ex, False
        if not exchange:
            self._begin("partition_build")
            if ok:
                sh.insert_words(words, m)      # one rank: the routed words are this shard's
            return m
        recv = self._grow("_ins_recv", max(m, 1) * W, torch.int64, recs.device)
        if nch == 1:
            self._begin("exchange_wait")
            self._all_to_all(recv[:m * W], words, [x * W for x in recv_c[0]],
                             [x * W for x in send_c[0]], gmax * W, in_off=views(0, send_c[0])[1])
            self._begin("partition_build")
            if ok:
                sh.insert_words(recv, m)
            return m
        works, spans, pos = [], [], 0
        for c in range(nch):
            mc = sum(recv_c[c])
            outs, o = [], pos
            for q in range(P):
                outs.append(recv[o * W:(o + recv_c[c][q]) * W])
                o += recv_c[c][q]
            self._sent(send_c[c], W * 8)
            works.append(self.comm.all_to_all_views_async(outs, views(c, send_c[c])[0]))
            spans.append((pos, mc))
            pos += mc
            if c > 0:  # previous chunk received: partition it while this one is on the wire
                self._begin("exchange_wait")
                works[c - 1].wait()
                self._begin("partition")
                p0, pm = spans[c - 1]
                if ok:
                    sh.stage_words(recv[p0 * W:(p0 + pm) * W], pm, m)
        self._begin("exchange_wait")
        works[-1].wait()
        self._begin("partition")
        p0, pm = spans[-1]
        if ok:
            sh.stage_words(recv[p0 * W:(p0 + pm) * W], pm, m)
            self._begin("build")
            sh.finish_words()
        return m

    def assemble(self, total_kmers):
        """Walk this rank's start k-mers (collective); returns the number of rounds. Walks that
        overlap (malformed input) are redone unsegmented (see _redo).

        Short walk first (round 6): splitter segments bound the rounds of long contigs (C5's 10^6-k-mer
        chains), but where contigs are short (C3: <= 200 k-mers) they add a walker per splitter and
        the link / pointer-jumping / retag phase for nothing. Where every rank's mean contig is
        shorter than the splitter spacing the walk goes without segments first; a walker past 4
        spacings ends it (reported with the text count exchange) and every rank walks again,
        segmented, as it then does for the rest of this input's steps."""
        self._seg_off = False
        sh = self.shard
        if self._short_key != (self._walkers, total_kmers):  # another input: try short again
            self._short_key, self._needs_seg = (self._walkers, total_kmers), False
        if not self._needs_seg and hasattr(sh, "mw_short") and sh.mw_short(total_kmers, self._starts_all):
            saved = self._splitters, self._walkers
            self._splitters, self._walkers = 0, self._starts_all
            self._seg_off = True
            try:
                r = self._assemble_migrate(total_kmers, short=True)
            finally:
                self._splitters, self._walkers = saved
                self._seg_off = False
            if r is not None:
                return r
            self._needs_seg = True
        return self._assemble_migrate(total_kmers)

    _short_key = None
    _needs_seg = False

    REDO_MAX = 2  # unsegmented with the default store, then with the store the last attempt needed

    def _flag(self):
        """This walk's overlap / overflow report as a device int64 scalar (shards without it: 0)."""
        sh = self.shard
        if hasattr(sh, "mw_flags") and hasattr(getattr(sh, "L", None), "kh_mwalk_flags_dev"):
            self._flags = sh.mw_flags()
            return self._flags[:1]
        self._flags = None
        return None

    def _redo(self, total_kmers, attempt):
        """Some rank's walk reported overlapping walks (a splitter segment with two predecessors, a
        start k-mer met as a splitter) or outgrew its text store: every rank walks again without
        splitter segments — each start to its own end, as kmer_hash.cpp:41-53 does — with a store
        sized from the last attempt's need. Every rank takes this branch together (the report
        travelled with a count exchange)."""
        if attempt >= self.REDO_MAX:
            raise _lib.KmerHashError(_lib.KH_ERR_NOMEM, "migrating walk: overlapping walks or text store overflow "
                                                        f"after {attempt} redo(s)")
        sh = self.shard
        need = int(self._host(self._flags)[1]) if attempt else 0
        sh.mw_redo(need * 5 // 4 + 4096 if need else 0)
        saved = self._splitters, self._walkers
        self._splitters, self._walkers = 0, self._starts_all
        self._seg_off = True
        try:
            return self._assemble_migrate(total_kmers, attempt + 1)
        finally:
            self._splitters, self._walkers = saved

    def _grow(self, name, n, dtype, device, slack=1.25):
        t = getattr(self, name, None)
        if t is None or t.numel() < n or t.dtype != dtype or t.device != device:
            if t is not None:
                setattr(self, name, None)
                del t  # the old buffer goes back to the allocator before the new one is taken
            t = torch.empty(max(int(n * slack), 16), dtype=dtype, device=device)
            setattr(self, name, t)
        return t

    def _cap(self, r):
        """Slot capacity of round r, the same on every rank: the largest per-destination count of
        round r in the last assemble (+ 25 %), else an even spread of every walker (first round)
        or the last learnt one. Messages past it are held back, never lost."""
        if r < len(self._caps):
            c = self._caps[r]
        elif self._caps:
            c = self._caps[-1]
        else:
            P = self.P
            c = max(1024, (self._walkers + P * P - 1) // (P * P) * 5 // 4 + 1024) if P > 1 else self._walkers + 16
        return max(1, min(max(c, self._cap_floor), self.SLOT_CAP_MAX))

    SLOT_CAP_MAX = 1 << 40  # tests: tiny slots (messages held back), set on the class

    def _assemble_migrate(self, total_kmers, attempt=0, short=False):
        """Walkers move to the rank owning their next k-mer (minimizer sharding keeps runs of
        consecutive k-mers on one rank). A round = local walk -> one all-to-all of fixed-size
        slots: no host read per round; the host reads the global in-flight count only at checks
        (first at the last assemble's round count, then every CHECK_EVERY rounds). Then the text
        records go home in one more all-to-all."""
        sh, P = self.shard, self.P
        M, T = sh.MSG_WORDS, sh.TEXT_REC_WORDS
        dev = sh.zeros(1, torch.int64).device
        local = P == 1 and not self.SELF_EXCHANGE
        failed = self._err is not None  # this shard could not be sized: it sends nothing until the check
        self._begin("walk_init")
        if not failed:
            sh.mw_begin(P, self.comm.rank, total_kmers, self._ns, self._nsp, self._walkers)
        self.rounds = self.checks = 0
        inp, cap_in = None, 0
        if self._caps_walkers != self._walkers:
            # caps learnt from a walk of another walker count describe another input: start over
            self._caps, self._rounds_hint = [], 0
        self._cap_floor = 0
        check_at = self._rounds_hint or self.CHECK_EVERY
        # rounds without splitter segments (KH_SPLIT_BITS=0) grow with the longest chain; a
        # walker advances every round it is not held back, so total_kmers bounds them
        limit = self.MAX_ROUNDS if self._splitters else max(self.MAX_ROUNDS, total_kmers + self.MAX_ROUNDS)
        # [in flight, largest per-destination count] of the rounds since the last check
        live = self._grow("_mw_live", 2 * max(check_at, self.CHECK_EVERY) + 2, torch.int64, dev, slack=1.0)
        maxes, flights, used, base = [], [], [], 0
        while True:
            cap = self._cap(self.rounds)
            used.append(cap)
            sw = _lib.slot_words(cap)
            out = self._grow("_mw_out_%d" % (self.rounds & 1), P * sw, torch.int64, dev)
            lv = 2 * (self.rounds - base)
            self._begin("walk_rounds")
            if failed:
                out.view(-1)[:P * sw].view(P, sw)[:, 0] = 0
                live[lv:lv + 2] = 0
            else:
                sh.mw_round(inp, cap_in, out, cap, live[lv:])
            if local:
                nxt = out      # one rank: slot 0 is the next round's input
            else:
                nxt = self._grow("_mw_in_%d" % (self.rounds & 1), P * sw, torch.int64, dev)
                self._begin("walk_exchange")
                self._sent([sw] * P, 8)
                self.comm.all_to_all(nxt[:P * sw], out[:P * sw], [sw] * P, [sw] * P)
            inp, cap_in = nxt, cap
            self.rounds += 1
            if self.rounds >= check_at or self.rounds >= limit:
                # global max of the window's [in flight, largest per-destination] + errors
                self._begin("walk_check")
                nw = 2 * (self.rounds - base)
                if local:  # one rank: no reduction, the error is this rank's own
                    h = self._host(live[:nw]).tolist() + [1 if self._err is not None else 0]
                    self.syncs -= 1  # counted below
                else:
                    err = torch.tensor([1 if self._err is not None else 0], dtype=torch.int64, device=dev)
                    h = self.comm.max_to_host(torch.cat([live[:nw], err])).tolist()
                self.checks += 1
                self.syncs += 1
                if int(h[-1]):
                    if self._err is not None:
                        raise self._err
                    raise _lib.KmerHashError(_lib.KH_ERR_FULL, "another rank failed to size its shard")
                maxes.extend(int(x) for x in h[1:nw:2])
                flights.extend(int(x) for x in h[0:nw:2])
                if int(h[nw - 2]) == 0:
                    break
                # a round whose demand passed its slots held messages back: later rounds get slots
                # for that demand, so the surplus drains in a few rounds, not thousands
                for m, c in zip(maxes[base:], used[base:]):
                    if m > c:
                        self._cap_floor = max(self._cap_floor, m * 5 // 4 + 256)
                if self.rounds >= limit:
                    raise _lib.KmerHashError(_lib.KH_ERR_CYCLE, f"migrating walk did not end in {limit} rounds")
                base = self.rounds
                check_at = self.rounds + self.CHECK_EVERY
        # the next assemble: slots sized by what each round carried, and its first check at the
        # round after which nothing was in flight (rounds past it are empty: ~60 us each)
        self._caps = [max(256, int(x) * 5 // 4 + 256) for x in maxes]
        self._rounds_hint = next((i + 1 for i, x in enumerate(flights) if x == 0), self.rounds)
        self._caps_walkers = self._walkers
        self._begin("text_group")
        tb = sh.mw_text_bound()
        tout = self._grow("_mw_tout", max(tb, 1) * T, torch.int64, dev)
        counts = sh.mw_text(tout)
        segmented = bool(self._splitters) and hasattr(sh, "mw_segments")
        # unsegmented walks report their store overflow (overlapping walks) with this exchange;
        # segmented ones with the retag exchange (_segments_end), after the segment links
        flag = None if segmented else self._flag()
        send_splits, recv_splits, _, gmax, over = self._exchange_counts(counts, flag)
        if short and flag is not None and any(int(x) >> 40 for x in over):
            sh.mw_abandon()  # a long contig somewhere: every rank walks again, segmented
            return None
        if flag is not None and any(int(x) for x in over):
            return self._redo(total_kmers, attempt)
        r = sum(recv_splits)
        self.text_records = r  # text records this origin received (tools/mem_model.py checks)
        if local:
            trecv = tout
        else:
            self._begin("text_exchange")
            trecv = self._grow("_mw_trecv", max(r, 1) * T, torch.int64, dev)
            self._all_to_all(trecv[:r * T], tout[:sum(send_splits) * T], [c * T for c in recv_splits],
                             [c * T for c in send_splits], gmax * T)
        # every rank takes the same branch (a rank without splitters still links and answers)
        if segmented:
            if not self._segments_end(trecv, r, self._ns + self._nsp):
                return self._redo(total_kmers, attempt)
        else:
            self._begin("materialize")
            sh.mw_end(trecv, r)
        sh.sync()  # the library counts this one (kh_sync)
        self._end()
        return self.rounds

    CHECK_EVERY = 4
    MAX_ROUNDS = 4096
    # every phase name _begin uses, in step order (the bench line reports them in this order)
    PHASES = ("insert", "route", "counts", "exchange_wait", "partition", "partition_build", "build",
              "walk_init", "walk_rounds", "walk_exchange", "walk_check", "text_group", "text_exchange",
              "seg_link", "seg_resolve", "seg_retag", "materialize")  # with splitter segments (the default) C5's 10^6-k-mer chains take ~11

    def _segments_end(self, trecv, r, nseg):
        """Splitter segments: link each segment to its successor's owner, all-gather every rank's
        predecessor table, rank the chains on the device (pointer jumping, no exchange per step),
        send the segments' text to the contig origins, materialise."""
        sh, P = self.shard, self.P
        dev = trecv.device
        L, S, PW = sh.LINK_WORDS, sh.SEG_REC_WORDS, sh.PRED_WORDS
        local = P == 1 and not self.SELF_EXCHANGE  # one rank: every exchange is the identity
        self._begin("seg_link")
        lout = self._grow("_ms_links", max(nseg, 1) * L, torch.int64, dev)
        counts = sh.mw_link(trecv, r, lout)
        if local:
            send_splits, recv_splits, _, gmax, _ = self._exchange_counts(counts)
            nsps = [self._nsp]
        else:
            nsp = torch.tensor([self._nsp], dtype=torch.int64, device=dev)
            send_splits, recv_splits, _, gmax, nsps = self._exchange_counts(counts, nsp)
        m = sum(recv_splits)
        if local:
            lin = lout
        else:
            lin = self._grow("_ms_links_in", max(m, 1) * L, torch.int64, dev)
            self._all_to_all(lin[:m * L], lout[:sum(send_splits) * L], [c * L for c in recv_splits],
                             [c * L for c in send_splits], gmax * L)
        self._begin("seg_resolve")
        stride = max(int(x) for x in nsps)
        preds = self._grow("_ms_preds", max(stride, 1) * PW, torch.int64, dev)
        sh.mw_pred(lin, m, preds, stride)
        if local:
            allp = preds
        else:
            allp = self._grow("_ms_allp", max(P * stride, 1) * PW, torch.int64, dev)
            self.xbytes += (P - 1) * stride * PW * 8
            self.comm.all_gather(allp[:P * stride * PW], preds[:stride * PW])
        sh.mw_resolve(allp, stride)
        self._begin("seg_retag")
        tout = self._grow("_ms_t", max(r + nseg, 1) * S, torch.int64, dev)
        counts = sh.mw_retag(trecv, r, tout)
        flag = self._flag()  # overlapping walks (links, predecessors) or a store overflow, any rank
        send_splits, recv_splits, _, gmax, over = self._exchange_counts(counts, flag)
        if flag is not None and any(int(x) for x in over):
            return False
        m = sum(recv_splits)
        self.seg_records = m
        if local:
            tin = tout
        else:
            tin = self._grow("_ms_tin", max(m, 1) * S, torch.int64, dev)
            self._all_to_all(tin[:m * S], tout[:sum(send_splits) * S], [c * S for c in recv_splits],
                             [c * S for c in send_splits], gmax * S)
        self._begin("materialize")
        sh.mw_end_seg(trecv, r, tin, m)
        return True

    def contigs_text(self):
        """This rank's contig text (D2H; outside the timed region)."""
        return self.shard.contigs_text()


# --------------------------------------------------------------------------------------------
def run_threaded(k, recs, nranks, device=0, info=None, insert_chunks=None, shard_kmers=None,
                 check=None, load_factor=0.5, steps=1):
    """P logical ranks on one GPU (threads): returns the per-rank contig texts. recs: a host
    record array, or a SyntheticKmers whose blocks each rank generates on the GPU (C4-size
    inputs), or a list of host record arrays walked one after another on the same maps (clear
    between them; returns a list of per-rank texts per input). Shards start at shard_kmers
    (default n / P) and grow to what they are routed.
    check(rank, text) (optional) consumes each rank's text instead of returning it (large runs).
    `info` (a dict) receives the round count, per-rank table stats and, per rank, the blocking
    host reads of the last step (insert_all + assemble: this host's and the library's).
    steps > 1 repeats clear + insert + assemble on the same records (buffers sized by step 1)."""
    import gc
    import numpy as np
    # the shards allocate through hipMalloc, not torch's caching allocator: blocks torch still
    # caches from earlier runs in this process are returned to the device first
    gc.collect()
    torch.cuda.empty_cache()
    comms = ThreadComm.group(nranks)
    seq = isinstance(recs, (list, tuple))
    inputs = list(recs) if seq else [recs]
    gen = recs if hasattr(recs, "records_dev") else None
    n0 = gen.n if gen is not None else inputs[0].shape[0]
    out = [[None] * nranks for _ in inputs]
    errs = []
    start = shard_kmers if shard_kmers else max(n0 // nranks, 1)

    def body(r):
        try:
            torch.cuda.set_device(device)
            shard = GpuShard(k, start, device=device, load_factor=load_factor)
            with torch.cuda.stream(shard.stream):
                dm = DistributedKmerHashMap(comms[r], shard)
                if insert_chunks:
                    dm.INSERT_CHUNKS = insert_chunks
                    dm.PIPELINE_MIN = 0
                for i, inp in enumerate(inputs):
                    n = gen.n if gen is not None else inp.shape[0]
                    split = (n + nranks - 1) // nranks
                    b = min(r * split, n)
                    e = min(b + split, n)
                    if gen is not None:
                        mine = gen.records_dev(b, e, device=device, stream=shard.stream)
                    else:
                        mine = torch.from_numpy(np.ascontiguousarray(inp[b:e])).to(shard.dev)
                    for step in range(steps):
                        if step or i:
                            shard.clear()
                        s0 = dm.host_syncs()
                        dm.insert_all(mine)
                        comms[r].barrier()
                        dm.assemble(n)
                        syncs = dm.host_syncs() - s0
                    del mine
                    text = dm.contigs_text()
                    if check is not None:
                        check(r, text)
                    else:
                        out[i][r] = text
                if info is not None:
                    info.setdefault("rounds", dm.rounds)
                    info.setdefault("stats", {})[r] = shard.stats()
                    info.setdefault("syncs", {})[r] = syncs
                    info.setdefault("checks", {})[r] = dm.checks
                    info.setdefault("segmented", {})[r] = dm._needs_seg  # the short walk met a long contig
                    # the counts tools/mem_model.py sizes a rank's buffers from
                    info.setdefault("counts", {})[r] = dict(
                        n_ins=shard.inserted, n_table=shard.n_table, ns=dm._ns, nsp=dm._nsp,
                        walkers_all=dm._walkers, recv_text=dm.text_records, recv_seg=dm.seg_records,
                        cap_slot=max(dm._caps) if dm._caps else 0)
            shard.table.close()
        except BaseException as ex:  # surface thread failures
            errs.append(ex)
            comms[r].sh.barrier.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:  # the failure itself, not the barrier aborts it caused on the other ranks
        errs.sort(key=lambda e: isinstance(e, threading.BrokenBarrierError))
        raise errs[0]
    return out if seq else out[0]


def bench_main(args, w, world, rank, cpu_baseline=None, load_traffic=None):
    """bench.py body for N > 1 ranks (torch.distributed.run, one rank per GPU), or forced at one
    rank (KH_BENCH_FORCE_DIST=1). Weak scaling (n k-mers per GPU) unless the workload is strong
    (C4: n k-mers in all, block split over the ranks, read_kmers.hpp:55-58)."""
    import json
    import os
    import sys
    import time

    import numpy as np
    import torch.distributed as dist
    from .hashmap import SyntheticKmers, record_size

    local = init_rank_process_group()
    comm = TorchComm()
    if comm.world != world or comm.world != args.gpus:
        raise SystemExit(f"bench: the communicator has {comm.world} ranks, --gpus {args.gpus}, "
                         f"WORLD_SIZE {world}")
    k = w["k"]
    strong = bool(w.get("strong"))
    n_total = w["n"] if strong else w["n"] * world
    n_per = (n_total + world - 1) // world
    t = time.time()
    g = SyntheticKmers(k, n_total, w["len_min"], w["len_max"], w["single"], seed=w["seed"], **w.get("gen", {}))
    b, e = g.block(world, rank)
    recs = g.records_dev(b, e, device=local)  # the rank's block, generated in its HBM
    torch.cuda.synchronize()
    print(f"[rank {rank}] generated {e - b} records in {time.time() - t:.1f}s", file=sys.stderr,
          flush=True)
    # each shard holds ~n_total/world keys (it grows to what it is routed); 2 % slack
    shard = GpuShard(k, int(n_per * 1.02) + 4096, device=local, load_factor=getattr(args, "load", 0.5))
    dm = DistributedKmerHashMap(comm, shard)
    dm.timer = PhaseTimer(cuda=True)
    R = record_size(k)
    # a step (or the warmup, which also sizes every buffer) that outlives this ends the rank,
    # naming the phase it is stuck in (a hung collective must not hang the job silently)
    dog = StepWatchdog(float(os.environ.get("KH_DIST_STEP_TIMEOUT", DIST_TIMEOUT_S)), rank, lambda: dm.phase)

    def body():
        with torch.cuda.stream(shard.stream):
            shard.clear()
            dm.insert_all(recs)
            dm.assemble(n_total)

    def step():
        guarded_step(dm, dog, body)

    for _ in range(args.warmup):
        step()
    # the contract's bracket: barrier + synchronize on both sides of the K steps (round 5 put a
    # barrier inside every step: ~0.2 ms of a one-rank step was that closing barrier). Each step
    # still ends in a synchronize, as the single-GPU bench's steps do, for its wall time and the
    # phase events; the steps' own collectives keep the ranks in step.
    times, phases, ptimes, xbytes, syncs = [], [], [], [], []
    dist.barrier()
    torch.cuda.synchronize()
    t_all = time.perf_counter()
    for _ in range(args.steps):
        t0 = time.perf_counter()
        s0 = dm.host_syncs()
        step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
        phases.append(shard.stats())
        ptimes.append(dm.timer.totals())
        xbytes.append(dm.xbytes)
        syncs.append(dm.host_syncs() - s0)
    torch.cuda.synchronize()
    dist.barrier()
    t_all = time.perf_counter() - t_all
    print(f"[rank {rank}] step ms: " + " ".join(f"{1e3 * x:.2f}" for x in times), file=sys.stderr, flush=True)
    for i in (0, len(ptimes) - 1):
        print(f"[rank {rank}] step {i} phases ms: " + " ".join(f"{nm} {v:.3f}" for nm, v in ptimes[i].items()),
              file=sys.stderr, flush=True)
    mine = t_all / args.steps
    tmax = comm.all_reduce_max(mine)
    # per-rank phase times (mean over the timed steps) -> max / min over ranks, in PHASES order
    names = list(DistributedKmerHashMap.PHASES)
    mean_ph = [sum(p.get(nm, 0.0) for p in ptimes) / len(ptimes) for nm in names]
    st0 = phases[-1]
    per_rank = mean_ph + [sum(xbytes) / len(xbytes), max(syncs), st0["ms_build"], st0["ms_insert_kernel"],
                          float(dm.rounds)]
    hi = torch.tensor(per_rank, dtype=torch.float64, device="cuda")
    lo = -hi.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    dist.all_reduce(lo, op=dist.ReduceOp.MAX)
    hi, lo = hi.tolist(), (-lo).tolist()
    nph = len(names)
    rank_phases = {nm: {"max": round(hi[i], 4), "min": round(lo[i], 4)} for i, nm in enumerate(names)
                   if hi[i] > 0 or lo[i] > 0}
    st = phases[-1]
    tot = torch.tensor([st["n_starts"], st["n_lookups"]], dtype=torch.int64, device="cuda")
    dist.all_reduce(tot)
    nc, nl = tot.tolist()
    ok = None
    truth = None if args.no_verify else g.truth(b, e)

    def verify():
        ok_local = int(dm.contigs_text() == truth)
        okt = torch.tensor([ok_local], dtype=torch.int64, device="cuda")
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        if not okt.item() and rank == 0:
            print("bench: contig text differs from the generator ground truth", file=sys.stderr)
        return bool(okt.item())

    if truth is not None:
        ok = verify()
    routed = None
    if world == 1 and not dm.ROUTE_ONE_RANK and not getattr(args, "no_routed", False):
        # The step P > 1 runs, at one rank: records through the one-pass route and the receiver's
        # k_win1 + k_win2 (KH_DIST_ROUTE_ONE_RANK=1) instead of the single-GPU records pass.
        # Timed after the headline steps, same bracket; not part of `value`.
        dm.ROUTE_ONE_RANK = True
        step()
        rt = []
        for _ in range(args.steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            rt.append(time.perf_counter() - t0)
        routed = {"ms_per_step": 1e3 * sum(rt) / len(rt),
                  "insert_pipeline_ms": shard.stats()["ms_insert_kernel"],
                  "phases_ms": {nm: round(v, 4) for nm, v in dm.timer.totals().items()},
                  "verified_vs_truth": verify() if truth is not None else None}
        dm.ROUTE_ONE_RANK = False
    cpu = None
    if rank == 0 and cpu_baseline is not None and not args.no_cpu:
        # the CPU restatement of the reference on a bounded sample of the same generator/config
        # (whole contigs: a rank's block of shuffled records is not a closed set), rank 0 only,
        # after the timed region; the other ranks wait at the closing barrier
        t = time.time()
        sn = min(args.cpu_sample or 20_000_000, n_per)
        gs = SyntheticKmers(k, sn, w["len_min"], w["len_max"], w["single"], seed=w["seed"], **w.get("gen", {}))
        cpu = cpu_baseline(w, gs.records(), gs.truth(), 0)
        cpu["sample"] = f"a {sn}-k-mer set of the same generator/config (rank 0's host share); " + cpu["sample"]
        print(f"cpu baseline took {time.time() - t:.1f}s", file=sys.stderr, flush=True)
    if rank == 0:
        value = (n_total + nl) / tmax
        avg = lambda key: sum(p[key] for p in phases) / len(phases)  # noqa: E731
        build_ms, ins_ms = avg("ms_build"), avg("ms_insert_kernel")
        units = st["n_inserted"]
        b_alg = 2 * R
        traffic, tsrc = (load_traffic(w.get("name", "") + "_dist", n_per) if load_traffic else (None, None))
        tb = traffic.get("k_part_build") if traffic else None
        achieved = units * b_alg / (build_ms / 1e3) / 1e9 if build_ms else 0.0
        out = {
            "metric": "k-mer inserts+lookups/sec (k=51)" if k == 51 else f"k-mer inserts+lookups/sec (k={k})",
            "value": value, "unit": "ops/s", "n_gpus": comm.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": tmax * 1e3, "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": value / 72.6e6, "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": w["desc"], "k": k, "n_kmers_total": n_total,
                       "n_kmers_per_gpu": n_per, "contigs": nc, "lookups": nl,
                       "load_factor": getattr(args, "load", 0.5),
                       "parallelism": f"{world} GPUs, key space sharded by "
                                      f"{'minimizer' if os.environ.get('KH_OWNER') != 'hash' else 'hash'} owner, "
                                      f"RCCL all-to-all per migrating-walker round",
                       "walk_rounds": dm.rounds},
            "inserts_per_s": n_total / tmax, "lookups_per_s": nl / tmax,
            "contigs_per_s": nc / tmax, "verified_vs_truth": ok,
            "phases_ms": {"insert_pipeline_rank0": ins_ms, "build_rank0": build_ms},
            # per-rank stream time of each driver phase (HIP events), max / min over the ranks
            "rank_phases_ms": rank_phases,
            "rank_step_ms": {"max": tmax * 1e3, "mean_rank0": mine * 1e3,
                             "median_step_rank0": 1e3 * sorted(times)[len(times) // 2]},
            "exchange_bytes_per_step": {"max": hi[nph], "min": lo[nph]},
            "host_syncs_per_step": {"max": hi[nph + 1], "min": lo[nph + 1]},
            "build_ms": {"max": hi[nph + 2], "min": lo[nph + 2]},
            "insert_pipeline_ms": {"max": hi[nph + 3], "min": lo[nph + 3]},
            **({"routed_one_rank": routed} if routed else {}),
            "roofline": {"bound": "hbm", "kernel": "k_part_build_pf (rank 0's region build + chains over the "
                                                     "words it received)",
                         "achieved": achieved, "peak": 8000.0, "unit": "GB/s", "frac": achieved / 8000.0,
                         "traffic": tb, "alg_bytes_per_unit": b_alg, "units_per_launch": units,
                         "avg_launch_ms": build_ms,
                         "traffic_GBs": (tb / (build_ms / 1e3) / 1e9) if tb and build_ms else None,
                         "note": "achieved = k-mers in rank 0's shard x 2*sizeof(kmer_pair) / HIP-event time of "
                                 "the build" + (f"; traffic = PMC HBM bytes per launch from {tsrc} (sharded "
                                                f"path at one rank)" if tb else "")},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    torch.cuda.synchronize()
    dist.barrier()
    dist.destroy_process_group()
    dm.close()
    shard.table.close()
