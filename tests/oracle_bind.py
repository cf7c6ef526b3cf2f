"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY (the parity checker).

Importable from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")

_o = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_LIB):
            build()
        o = ctypes.CDLL(ORACLE_LIB)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        o.ko_pack.argtypes = [ctypes.c_int, ctypes.c_char_p, vp]
        o.ko_unpack.argtypes = [ctypes.c_int, vp, vp]
        o.ko_djb2.argtypes = [ctypes.c_int, vp]
        o.ko_djb2.restype = u64
        o.ko_next_kmer.argtypes = [ctypes.c_int, vp, vp]
        o.ko_parse_text.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, vp]
        o.ko_parse_text.restype = ctypes.c_size_t
        o.ko_assemble.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, ctypes.POINTER(vp),
                                  ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
                                  ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_double)]
        o.ko_assemble.restype = ctypes.c_int
        o.ko_assemble_par.argtypes = [ctypes.c_int, vp, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(vp),
                                      ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_double)]
        o.ko_assemble_par.restype = ctypes.c_int
        o.ko_free.argtypes = [vp]
        o.ko_table_new.argtypes = [ctypes.c_int, ctypes.c_size_t]
        o.ko_table_new.restype = vp
        o.ko_table_free.argtypes = [vp]
        o.ko_table_insert.argtypes = [vp, vp]
        o.ko_table_find.argtypes = [vp, vp, vp]
        _o = o
    return _o


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def pack(k, kmer):
    out = np.zeros((k + 3) // 4, np.uint8)
    lib().ko_pack(k, kmer.encode(), _p(out))
    return out


def unpack(k, packed):
    packed = np.ascontiguousarray(packed, np.uint8)
    out = np.zeros(k, np.uint8)
    lib().ko_unpack(k, _p(packed), _p(out))
    return out.tobytes().decode()


def djb2(k, packed):
    return int(lib().ko_djb2(k, _p(np.ascontiguousarray(packed, np.uint8))))


def next_kmer(k, rec):
    out = np.zeros((k + 3) // 4, np.uint8)
    lib().ko_next_kmer(k, _p(np.ascontiguousarray(rec, np.uint8)), _p(out))
    return out


def parse_text(k, text):
    buf = np.frombuffer(text, np.uint8)
    n = len(text) // (k + 4)
    recs = np.zeros((n, (k + 3) // 4 + 2), np.uint8)
    lib().ko_parse_text(k, _p(buf), len(text), _p(recs))
    return recs


def assemble(k, recs):
    """Serial stock-semantics assembly -> (rc, text bytes, n_contigs, n_lookups, t_ins, t_walk)."""
    recs = np.ascontiguousarray(recs, np.uint8)
    n = recs.shape[0] if recs.ndim == 2 else recs.size // ((k + 3) // 4 + 2)
    out = ctypes.c_void_p()
    ln, nc, nl = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    ti, tw = ctypes.c_double(), ctypes.c_double()
    rc = lib().ko_assemble(k, _p(recs), n, ctypes.byref(out), ctypes.byref(ln), ctypes.byref(nc),
                           ctypes.byref(nl), ctypes.byref(ti), ctypes.byref(tw))
    text = b""
    if rc == 0:
        text = ctypes.string_at(out, ln.value)
        lib().ko_free(out)
    return rc, text, nc.value, nl.value, ti.value, tw.value


def assemble_par(k, recs, threads):
    """Thread-parallel DistributedHashMap restatement (threads = ranks) -> same tuple as assemble;
    the text is the ranks' outputs concatenated in rank order."""
    recs = np.ascontiguousarray(recs, np.uint8)
    n = recs.shape[0] if recs.ndim == 2 else recs.size // ((k + 3) // 4 + 2)
    out = ctypes.c_void_p()
    ln, nc, nl = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    ti, tw = ctypes.c_double(), ctypes.c_double()
    rc = lib().ko_assemble_par(k, _p(recs), n, threads, ctypes.byref(out), ctypes.byref(ln),
                               ctypes.byref(nc), ctypes.byref(nl), ctypes.byref(ti), ctypes.byref(tw))
    text = b""
    if rc == 0:
        text = ctypes.string_at(out, ln.value)
        lib().ko_free(out)
    return rc, text, nc.value, nl.value, ti.value, tw.value


class Table:
    def __init__(self, k, size):
        self.k, self.P, self.R = k, (k + 3) // 4, (k + 3) // 4 + 2
        self.h = lib().ko_table_new(k, size)

    def insert(self, rec):
        return lib().ko_table_insert(self.h, _p(np.ascontiguousarray(rec, np.uint8))) == 1

    def find(self, key):
        out = np.zeros(self.R, np.uint8)
        ok = lib().ko_table_find(self.h, _p(np.ascontiguousarray(key, np.uint8)), _p(out)) == 1
        return ok, out

    def __del__(self):
        if getattr(self, "h", None):
            lib().ko_table_free(self.h)
            self.h = None
