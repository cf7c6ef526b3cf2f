"""cs267_hw3_amd — MI355X-native k-mer hash table + de Bruijn contig walker.

Drop-in for the hash_map.hpp / kmer_hash.cpp hot path of fractalclockwork/CS267_HW3: the product is
the C-ABI library libkmerhash_amd.so (include/kmer_hash_amd.h) with hand-written gfx950 kernels;
this package is its Python host mirror (ctypes).
"""
from .hashmap import (KmerHashError, KmerHashTable, SyntheticKmers, device_count, djb2,  # noqa: F401
                      kmer_size, next_kmer, pack_kmer, pack_text, packed_size, read_kmer_lines, read_kmers,
                      record_size, unpack_kmer)

__version__ = "0.1.0"
