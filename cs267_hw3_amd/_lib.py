"""ctypes binding of the C ABI in include/kmer_hash_amd.h (the in-tree libkmerhash_amd.so).

This is the same stub a Python host of the reference would add. The library is
required: there is no CPU fallback, and importing the package on a box where the library was not
built raises immediately.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KH_LIB") or os.path.join(_HERE, "libkmerhash_amd.so")  # KH_LIB: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "kmer_hash_amd.h")

KH_OK = 0
KH_ERR_ARG = -1
KH_ERR_HIP = -2
KH_ERR_NOMEM = -3
KH_ERR_FULL = -4
KH_ERR_NOT_FOUND = -5
KH_ERR_DUPLICATE = -6
KH_ERR_CYCLE = -7
KH_ERR_BAD_BASE = -8
KH_ERR_STATE = -9

c_u64 = ctypes.c_uint64
c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_vp = ctypes.c_void_p


class KhStats(ctypes.Structure):
    _fields_ = [(name, c_u64) for name in (
        "capacity", "n_inserted", "n_starts", "n_contigs", "n_lookups", "out_bytes", "n_chunks",
        "n_dup", "n_full", "n_bad_ext", "n_missing", "n_cycle", "n_spin", "n_chunk_ovf")] + [
        (name, ctypes.c_double) for name in (
            "ms_insert", "ms_insert_kernel", "ms_walk", "ms_materialize")] + [("n_bad_base", c_u64)] + \
            [(f, ctypes.c_double) for f in ("ms_build", "ms_walk_kernel")] + \
            [(f, c_u64) for f in ("n_hot_regions", "n_overflow", "n_spread_regions")]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


ABI_VERSION = 3  # KH_ABI_VERSION of include/kmer_hash_amd.h

# name -> (restype, argtypes)
MSG_WORDS = 5  # KH_MSG_WORDS: migrating-walker message
TEXT_REC_WORDS = 2  # KH_TEXT_REC_WORDS
LINK_WORDS = 4  # KH_LINK_WORDS
PRED_WORDS = 2  # KH_PRED_WORDS


def slot_words(cap):
    """KH_SLOT_WORDS: int64 words of one exchange slot of `cap` messages."""
    return 2 + cap * MSG_WORDS

SEG_REC_WORDS = 3  # KH_SEG_REC_WORDS

_SIGS = {
    "kh_abi_version": (ctypes.c_int, []),
    "kh_device_bytes": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    "kh_packed_size": (ctypes.c_int, [ctypes.c_int]),
    "kh_record_size": (ctypes.c_int, [ctypes.c_int]),
    "kh_last_error": (ctypes.c_char_p, []),
    "kh_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "kh_create": (ctypes.c_int, [ctypes.POINTER(c_vp), ctypes.c_int, c_u64, ctypes.c_double,
                                 ctypes.c_int]),
    "kh_destroy": (ctypes.c_int, [c_vp]),
    "kh_clear": (ctypes.c_int, [c_vp]),
    "kh_reserve": (ctypes.c_int, [c_vp, c_u64]),
    "kh_key_owner": (ctypes.c_int, [c_vp, c_u8p, ctypes.c_int]),
    "kh_set_stream": (ctypes.c_int, [c_vp, c_vp]),
    "kh_sync": (ctypes.c_int, [c_vp]),
    "kh_capacity": (c_u64, [c_vp]),
    "kh_get_stats": (ctypes.c_int, [c_vp, ctypes.POINTER(KhStats)]),
    "kh_insert": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_insert_dev": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_find": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, c_vp]),
    "kh_find_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, c_vp]),
    "kh_set_starts": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_assemble_dev": (ctypes.c_int, [c_vp]),
    "kh_assemble": (ctypes.c_int, [c_vp, ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]),
    "kh_contigs_text": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_contigs_text_dev": (ctypes.c_int, [c_vp, ctypes.POINTER(c_vp), ctypes.POINTER(c_u64)]),
    "kh_contigs_offsets": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_word_count": (ctypes.c_int, [ctypes.c_int]),
    "kh_collect_starts_dev": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_route_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, ctypes.c_int, c_vp, c_vp]),
    "kh_route_starts_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, ctypes.c_int, c_vp, c_vp]),
    "kh_route_starts_win_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, ctypes.c_int, c_vp, c_u64, c_vp]),
    "kh_insert_words_dev": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_insert_words_stage_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, c_u64]),
    "kh_insert_words_finish": (ctypes.c_int, [c_vp]),
    "kh_pack_text_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, ctypes.POINTER(c_u64)]),
    "kh_host_syncs": (ctypes.c_int, [c_vp, ctypes.POINTER(c_u64)]),
    "kh_route_splitters_dev": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int]),
    "kh_counters_dev": (ctypes.c_int, [c_vp, c_vp]),
    "kh_counters": (ctypes.c_int, [c_vp, c_vp]),
    "kh_mwalk_begin": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, c_u64, c_u64, c_u64, c_u64,
                                      ctypes.POINTER(c_u64)]),
    "kh_mwalk_round_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, c_u64, c_vp]),
    "kh_mwalk_text_bound": (ctypes.c_int, [c_vp, ctypes.POINTER(c_u64)]),
    "kh_mwalk_text_dev": (ctypes.c_int, [c_vp, c_vp, c_vp]),
    "kh_mwalk_end_dev": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_mwalk_segments": (ctypes.c_int, [c_vp, ctypes.POINTER(c_u64)]),
    "kh_mwalk_flags_dev": (ctypes.c_int, [c_vp, c_vp]),
    "kh_mwalk_redo": (ctypes.c_int, [c_vp, c_u64]),
    "kh_mwalk_short": (ctypes.c_int, [c_vp, c_u64, c_u64, ctypes.POINTER(ctypes.c_int)]),
    "kh_mwalk_abandon": (ctypes.c_int, [c_vp]),
    "kh_mwalk_link_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, c_vp]),
    "kh_mwalk_pred_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, c_u64]),
    "kh_mwalk_resolve_dev": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_mwalk_retag_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, c_vp]),
    "kh_mwalk_end_seg_dev": (ctypes.c_int, [c_vp, c_vp, c_u64, c_vp, c_u64]),
    "kh_dev_malloc": (ctypes.c_int, [ctypes.POINTER(c_vp), c_u64, ctypes.c_int]),
    "kh_dev_free": (ctypes.c_int, [c_vp]),
    "kh_memcpy_htod": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_memcpy_dtoh": (ctypes.c_int, [c_vp, c_vp, c_u64]),
    "kh_pack_text": (ctypes.c_int, [ctypes.c_int, c_vp, c_u64, c_vp, ctypes.POINTER(c_u64)]),
    "kh_pack_kmer": (ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, c_vp]),
    "kh_unpack_kmer": (ctypes.c_int, [ctypes.c_int, c_vp, c_vp]),
    "kh_djb2": (c_u64, [ctypes.c_int, c_vp]),
    "kh_next_kmer": (ctypes.c_int, [ctypes.c_int, c_vp, c_vp]),
    "kh_gen_create": (ctypes.c_int, [ctypes.POINTER(c_vp), ctypes.c_int, c_u64, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, c_u64, ctypes.c_int,
                                     ctypes.c_int]),
    "kh_gen_create_skewed": (ctypes.c_int, [ctypes.POINTER(c_vp), ctypes.c_int, c_u64, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, c_u64, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]),
    "kh_gen_create_hot": (ctypes.c_int, [ctypes.POINTER(c_vp), ctypes.c_int, c_u64, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_uint32, c_u64, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.c_uint32, ctypes.c_uint32]),
    "kh_gen_create_hot_ex": (ctypes.c_int, [ctypes.POINTER(c_vp), ctypes.c_int, c_u64, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_uint32, c_u64, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                            ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    "kh_gen_destroy": (ctypes.c_int, [c_vp]),
    "kh_gen_num_contigs": (c_u64, [c_vp]),
    "kh_gen_records": (ctypes.c_int, [c_vp, c_u64, c_u64, c_vp]),
    "kh_gen_records_dev": (ctypes.c_int, [c_vp, c_u64, c_u64, c_vp, c_vp]),
    "kh_gen_truth": (ctypes.c_int, [c_vp, c_u64, c_u64, c_vp, c_u64, ctypes.POINTER(c_u64)]),
}

_lib = None


class KmerHashError(RuntimeError):
    """A non-zero status from the C ABI (kh_last_error() text attached)."""

    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        # torch ships its own libamdhip64: load it first so the library binds to that same HIP
        # runtime (two runtimes in one process leave torch with "No HIP GPUs are available")
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if os.environ.get("KH_LIB") and not hasattr(L, name):
                continue  # A/B experiments against an older build
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        if L.kh_abi_version() != ABI_VERSION:  # KhStats and the signatures above are version 3's
            raise ImportError(f"{LIB_PATH}: ABI version {L.kh_abi_version()}, this binding is "
                              f"version {ABI_VERSION} (include/kmer_hash_amd.h KH_ABI_VERSION)")
        _lib = L
    return _lib


def check(rc):
    if rc != KH_OK:
        msg = lib().kh_last_error()
        raise KmerHashError(rc, msg.decode() if msg else "")
    return rc


def declared_symbols(header=HEADER_PATH):
    """Function names declared in include/kmer_hash_amd.h."""
    import re
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(kh_[a-z0-9_]+)\s*\(", text)))
