// packing.hpp (drop-in) — same macros and functions as the reference's packing.hpp:5-107, backed
// by the C ABI codec (include/kmer_hash_amd.h). Unlike the reference, unpackKmer writes exactly
// KMER_LEN chars and needs no lazily built global table.
#pragma once
#include <cstdint>
#include <stdexcept>

#include "../kmer_hash_amd.h"

#ifndef KMER_LEN
#define KMER_LEN 19
#endif

#define PACKED_KMER_LEN ((KMER_LEN + 3) / 4)

inline void packKmer(const char* kmer, unsigned char* packed_kmer) {
    if (kh_pack_kmer(KMER_LEN, kmer, packed_kmer) != KH_OK) throw std::runtime_error(kh_last_error());
}

inline void unpackKmer(const unsigned char packed_kmer[PACKED_KMER_LEN], char* kmer) {
    kh_unpack_kmer(KMER_LEN, packed_kmer, kmer);
}
