"""Host-side mirror of the reference's k-mer table API over the C ABI.

Reference surface (fractalclockwork/CS267_HW3) -> here:
  kmer_pair / pkmer_t byte layout (kmer_t.hpp:6-8, pkmer_t.hpp:6)  -> numpy uint8 rows [n, R] / [n, P]
  read_kmers(fname, nprocs, rank)        (read_kmers.hpp:54-79)    -> read_kmers()
  DistributedHashMap(size, rank, world)  (hash_map.hpp:50-52)      -> KmerHashTable(k, n_kmers)
  insert_all(kmers)                      (hash_map.hpp:55-80)      -> KmerHashTable.insert_all()
  find(key, result) -> bool              (hash_map.hpp:83-107)     -> KmerHashTable.find()
  initialize_kmers + assemble_contigs    (kmer_hash.cpp:21-55)     -> insert_all() + assemble()
  extract_contig / test_<rank>.dat       (read_kmers.hpp:81-92)    -> contigs_text()
Errors mirror the reference: a walk that misses a k-mer raises (kmer_hash.cpp:47-49).
"""
import ctypes
import os

import numpy as np

from . import _lib
from ._lib import KhStats, KmerHashError, check


def packed_size(k):
    return (k + 3) // 4


def record_size(k):
    return packed_size(k) + 2


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def pack_text(k, text):
    """Fixed-width "KMER BF\\n" lines -> kmer_pair records, uint8 [n, R] (read_kmers.hpp:62-76)."""
    L = _lib.lib()
    buf = np.frombuffer(text, dtype=np.uint8) if not isinstance(text, np.ndarray) else text
    n = ctypes.c_uint64(0)
    check(L.kh_pack_text(k, _ptr(buf), buf.size, None, ctypes.byref(n)))
    recs = np.empty((n.value, record_size(k)), dtype=np.uint8)
    check(L.kh_pack_text(k, _ptr(buf), buf.size, _ptr(recs), ctypes.byref(n)))
    return recs


def kmer_size(fname):
    """read_kmers.hpp:14-25: length of the first whitespace-delimited token."""
    with open(fname, "rb") as f:
        return len(f.readline().split()[0])


def read_kmer_lines(fname, k, nprocs=1, rank=0):
    """read_kmers.hpp:54-68 block split: the raw text of lines [r*ceil(n/P), ...) of rank r."""
    line = k + 4
    size = os.path.getsize(fname)
    n = size // line
    split = (n + nprocs - 1) // nprocs
    start = min(split * rank, n)
    cnt = min(split, n - start)
    with open(fname, "rb") as f:
        f.seek(start * line)
        return f.read(cnt * line)


def read_kmers(fname, k, nprocs=1, rank=0):
    """read_kmers.hpp:54-79: rank r's block of the file as kmer_pair records (host codec)."""
    return pack_text(k, read_kmer_lines(fname, k, nprocs, rank))


def pack_kmer(k, kmer):
    out = np.zeros(packed_size(k), dtype=np.uint8)
    check(_lib.lib().kh_pack_kmer(k, kmer.encode() if isinstance(kmer, str) else kmer, _ptr(out)))
    return out


def unpack_kmer(k, packed):
    packed = np.ascontiguousarray(packed, dtype=np.uint8)
    out = np.zeros(k, dtype=np.uint8)
    check(_lib.lib().kh_unpack_kmer(k, _ptr(packed), _ptr(out)))
    return out.tobytes().decode()


def djb2(k, packed):
    packed = np.ascontiguousarray(packed, dtype=np.uint8)
    return int(_lib.lib().kh_djb2(k, _ptr(packed)))


def next_kmer(k, rec):
    rec = np.ascontiguousarray(rec, dtype=np.uint8)
    out = np.zeros(packed_size(k), dtype=np.uint8)
    check(_lib.lib().kh_next_kmer(k, _ptr(rec), _ptr(out)))
    return out


def device_count():
    n = ctypes.c_int(0)
    rc = _lib.lib().kh_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


class KmerHashTable:
    """GPU-resident open-addressing k-mer table + contig walker (one per GPU / rank)."""

    def __init__(self, k, n_kmers, load_factor=0.5, device=0):
        self.k = k
        self.P = packed_size(k)
        self.R = record_size(k)
        self._L = _lib.lib()
        h = ctypes.c_void_p()
        check(self._L.kh_create(ctypes.byref(h), k, int(n_kmers), float(load_factor), device))
        self._h = h

    # -- lifetime ---------------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._L.kh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def capacity(self):
        return int(self._L.kh_capacity(self._h))

    def clear(self):
        check(self._L.kh_clear(self._h))

    def sync(self):
        check(self._L.kh_sync(self._h))

    def set_stream(self, stream_ptr):
        check(self._L.kh_set_stream(self._h, ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def stats(self):
        s = KhStats()
        check(self._L.kh_get_stats(self._h, ctypes.byref(s)))
        return s.as_dict()

    # -- insert / find ------------------------------------------------------------------------
    def _recs(self, recs):
        recs = np.ascontiguousarray(recs, dtype=np.uint8)
        if recs.size % self.R:
            raise ValueError(f"record buffer of {recs.size} bytes is not a multiple of {self.R}")
        return recs, recs.size // self.R

    def insert_all(self, recs):
        """Synchronous bulk insert of host records; raises on duplicate/full/bad base."""
        recs, n = self._recs(recs)
        check(self._L.kh_insert(self._h, _ptr(recs), n))

    insert = insert_all

    def pack_text_dev(self, text_ptr, nbytes, recs_ptr=None):
        """read_kmers.hpp:62-76 on the GPU (device text -> device records at recs_ptr, 16-B
        aligned); returns the record count. Bad bases surface at the next sync()."""
        n = ctypes.c_uint64(0)
        check(self._L.kh_pack_text_dev(self._h, ctypes.c_void_p(text_ptr), nbytes,
                                       ctypes.c_void_p(recs_ptr) if recs_ptr else None, ctypes.byref(n)))
        return n.value

    def insert_dev(self, dev_ptr, n):
        """Asynchronous insert of n records already in device memory (16-B aligned)."""
        check(self._L.kh_insert_dev(self._h, ctypes.c_void_p(dev_ptr), int(n)))

    def find(self, keys):
        """Batched find of pkmer_t keys -> (records [n, R], found bool[n])."""
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        n = keys.size // self.P
        out = np.zeros((n, self.R), dtype=np.uint8)
        found = np.zeros(n, dtype=np.uint8)
        if n:
            check(self._L.kh_find(self._h, _ptr(keys), n, _ptr(out), _ptr(found)))
        return out, found.astype(bool)

    # -- assemble -------------------------------------------------------------------------
    def set_starts(self, recs):
        recs, n = self._recs(recs)
        check(self._L.kh_set_starts(self._h, _ptr(recs) if n else None, n))

    def assemble(self):
        nc, nb = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(self._L.kh_assemble(self._h, ctypes.byref(nc), ctypes.byref(nb)))
        return nc.value, nb.value

    def assemble_dev(self):
        check(self._L.kh_assemble_dev(self._h))

    def contigs_text(self):
        d, b = ctypes.c_void_p(), ctypes.c_uint64(0)
        check(self._L.kh_contigs_text_dev(self._h, ctypes.byref(d), ctypes.byref(b)))
        out = np.empty(b.value, dtype=np.uint8)
        if b.value:
            check(self._L.kh_contigs_text(self._h, _ptr(out), b.value))
        return out.tobytes()

    def contigs(self):
        return self.contigs_text().decode().splitlines()


class SyntheticKmers:
    """Seeded synthetic dataset (kh_gen_*): records at any position range + ground truth."""

    def __init__(self, k, n, len_min=8, len_max=200, single_permille=0, seed=1, shuffle=True,
                 threads=0, n_long=0, long_len=0, front_starts=False, hot_permille=0, n_motifs=0,
                 hot_flank=False):
        """n_long / long_len / front_starts: the C5 walker skew; hot_permille / n_motifs: the C5
        hot-bucket half (contigs sharing a few minimizer motifs, kh_gen_create_hot); hot_flank: a
        fixed flank before every motif too (the shared stretch is 2M bases: the remap's worst case)."""
        self.k, self.n = k, int(n)
        self.R = record_size(k)
        self._L = _lib.lib()
        h = ctypes.c_void_p()
        check(self._L.kh_gen_create_hot_ex(ctypes.byref(h), k, self.n, len_min, len_max,
                                           single_permille, seed, 1 if shuffle else 0, threads,
                                           n_long, long_len, 1 if front_starts else 0, hot_permille, n_motifs,
                                           1 if hot_flank else 0))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.kh_gen_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_contigs(self):
        return int(self._L.kh_gen_num_contigs(self._h))

    def block(self, nprocs=1, rank=0):
        """read_kmers.hpp:55-58 block split of the record array."""
        split = (self.n + nprocs - 1) // nprocs
        b = min(split * rank, self.n)
        return b, min(b + split, self.n)

    def records(self, begin=0, end=None, out=None):
        end = self.n if end is None else end
        if out is None:
            out = np.empty((end - begin, self.R), dtype=np.uint8)
        check(self._L.kh_gen_records(self._h, begin, end, _ptr(out)))
        return out

    def records_dev(self, begin=0, end=None, device=None, stream=None):
        """Records [begin, end) generated on the GPU into a uint8 torch tensor [m, R] (16-B
        aligned); stream: a torch stream (default: the current one)."""
        import torch
        end = self.n if end is None else end
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        with torch.cuda.device(dev):
            out = torch.empty(max(end - begin, 1) * self.R + 16, dtype=torch.uint8, device=dev)
            s = stream if stream is not None else torch.cuda.current_stream(dev)
            check(self._L.kh_gen_records_dev(self._h, begin, end, ctypes.c_void_p(out.data_ptr()),
                                             ctypes.c_void_p(s.cuda_stream)))
        return out[:(end - begin) * self.R].view(end - begin, self.R)

    def truth(self, begin=0, end=None):
        end = self.n if end is None else end
        nb = ctypes.c_uint64(0)
        check(self._L.kh_gen_truth(self._h, begin, end, None, 0, ctypes.byref(nb)))
        out = np.empty(nb.value, dtype=np.uint8)
        check(self._L.kh_gen_truth(self._h, begin, end, _ptr(out), nb.value, ctypes.byref(nb)))
        return out.tobytes()


__all__ = ["KmerHashTable", "SyntheticKmers", "KmerHashError", "pack_text", "read_kmers", "read_kmer_lines",
           "kmer_size", "pack_kmer", "unpack_kmer", "djb2", "next_kmer", "device_count",
           "packed_size", "record_size"]
