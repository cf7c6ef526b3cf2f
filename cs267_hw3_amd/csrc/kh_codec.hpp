// kh_codec.hpp — k-mer codec shared by host C++ and gfx950 device code.
//
// Reference record layout (must stay byte-identical, it is the drop-in wire format):
//   kmer_pair = { unsigned char data[PACKED]; char fb_ext[2]; }     kmer_t.hpp:6-8, pkmer_t.hpp:6
//   PACKED    = (K + 3) / 4                                          packing.hpp:9
//   base i of the k-mer lives in byte i/4 at bits 7-2(i%4) .. 6-2(i%4), A=0 C=1 G=2 T=3,
//   tail padded with 'A' (= 00 bits)                                 packing.hpp:50-92
//   fb_ext[0] = backward extension, fb_ext[1] = forward extension    kmer_t.hpp:43-45
//
// Internal (table) representation. The packed bytes read big-endian are the integer
//   B = V << 2*pad,  V = sum_i code(b_i) * 4^(K-1-i),  pad = 4*PACKED - K
// so next_kmer (kmer_t.hpp:51-53: drop base 0, append the forward base) is
//   V' = ((V << 2) | code(fwd)) mod 4^K
// i.e. a 2-bit shift instead of the reference's unpack/substr/repack string round trip.
// V is held as (hi, lo) with lo = V mod 2^62 (31 bases) and hi = V >> 62 (K-31 bases).
//
// Slot words (open addressing, one slot per k-mer):
//   W=1 (K <= 29): word0 = (V << 6) | ext                      8-byte slot
//   W=2 (K <= 60): word0 = (hi << 6) | ext, word1 = lo         16-byte slot (one dwordx4 probe)
//   ext = bwd_code | fwd_code << 3, codes A0 C1 G2 T3 F4, 5 = not an A/C/G/T/F byte.
//   Live slots never hold all-ones words (ext <= 45 < 63 and lo < 2^62), so all-ones is the
//   EMPTY sentinel for both words.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define KH_HD __host__ __device__ __forceinline__
#else
#define KH_HD inline
#endif

namespace kh {

static constexpr uint64_t EMPTY = ~0ull;
static constexpr uint64_t LO_MASK = (1ull << 62) - 1;
static constexpr int KMAX_W1 = 29;
static constexpr int KMAX = 60;
static constexpr uint32_t EXT_F = 4;
static constexpr uint32_t EXT_BAD = 5;

struct KParams {
    int K;          // bases per k-mer
    int P;          // packed bytes  = (K+3)/4
    int R;          // record bytes  = P + 2 (sizeof(kmer_pair), align 1)
    int pad;        // 4P - K padding bases
    int W;          // slot words (1 or 2)
    uint64_t hi_mask;   // mask for hi after a shift (2K-62 bits, 0 when K <= 31)
    uint64_t v_mask;    // W=1: mask of V (2K bits)
    int M;              // minimizer length (bases) of the sharded owner function
    int owner_mode;     // sharded owner: 0 = minimizer hash (default), 1 = low key_hash bits
    int split_bits;     // walk splitters: k-mers with (key_hash & (2^split_bits - 1)) == 0 and a
                        // predecessor start extra walkers (0 = off); see kh_kernels.hip k_walk
};

// Minimizer length for owner_key: consecutive k-mers of a contig share their minimizer for
// ~(K-M+2)/2 steps on random sequence, so a walk stays on one rank for that long; 4^M distinct
// values keep the shards balanced.
inline int minimizer_len(int K) { return K >= 31 ? 15 : K >= 20 ? 12 : K >= 10 ? 10 : K; }

inline KParams make_params(int K) {
    KParams p;
    p.K = K;
    p.P = (K + 3) / 4;
    p.R = p.P + 2;
    p.pad = 4 * p.P - K;
    p.W = (K <= KMAX_W1) ? 1 : 2;
    int hib = 2 * K - 62;
    p.hi_mask = hib > 0 ? ((1ull << hib) - 1) : 0ull;
    p.v_mask = (2 * K >= 64) ? ~0ull : ((1ull << (2 * K)) - 1);
    p.M = minimizer_len(K);
    p.split_bits = 0;
    p.owner_mode = 0;
    return p;
}

KH_HD uint32_t base_code(uint8_t c) {
    // 'A'=65 'C'=67 'G'=71 'T'=84 'F'=70
    switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    case 'T': return 3;
    case 'F': return EXT_F;
    default: return EXT_BAD;
    }
}

KH_HD uint8_t code_char(uint32_t code) {
    // 0..3 -> ACGT, 4 -> F, anything else -> '?'
    return code == 0 ? 'A' : code == 1 ? 'C' : code == 2 ? 'G' : code == 3 ? 'T' : code == 4 ? 'F' : '?';
}

struct Key {
    uint64_t hi, lo;
};

// Packed big-endian bytes (PACKED of them) -> V as (hi, lo).
KH_HD Key key_from_packed(const uint8_t* b, const KParams& p) {
    unsigned __int128 B = 0;
    for (int j = 0; j < p.P; ++j) B = (B << 8) | b[j];
    B >>= 2 * p.pad;
    Key k;
    k.lo = (uint64_t)B & LO_MASK;
    k.hi = (uint64_t)(B >> 62);
    return k;
}

KH_HD void key_to_packed(Key k, uint8_t* b, const KParams& p) {
    unsigned __int128 B = ((unsigned __int128)k.hi << 62) | k.lo;
    B <<= 2 * p.pad;
    for (int j = p.P - 1; j >= 0; --j) {
        b[j] = (uint8_t)B;
        B >>= 8;
    }
}

// Base i (0 = first/most significant) of the k-mer.
KH_HD uint32_t key_base(Key k, int i, const KParams& p) {
    int sh = 2 * (p.K - 1 - i);  // bit position of base i in V
    if (sh >= 62) return (uint32_t)(k.hi >> (sh - 62)) & 3u;
    return (uint32_t)(k.lo >> sh) & 3u;
}

// kmer_t.hpp:51-53 next_kmer on the integer form.
KH_HD Key key_next(Key k, uint32_t code, const KParams& p) {
    Key n;
    if (p.K <= 31) {
        n.hi = 0;
        n.lo = ((k.lo << 2) | code) & p.v_mask & LO_MASK;
    } else {
        n.hi = ((k.hi << 2) | (k.lo >> 60)) & p.hi_mask;
        n.lo = ((k.lo << 2) | code) & LO_MASK;
    }
    return n;
}

KH_HD uint64_t fmix64(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return h;
}

// Placement hash (NOT the reference's djb2: djb2 over 5 bytes spans < 2^38 at K=19 and would put
// every key of a high-bit shard split on one GPU; SURVEY §7 hard part 1). Placement never changes
// the output, only where a key lives.
KH_HD uint64_t key_hash(Key k) {
#ifdef KH_CHEAP_HASH  // experiment only
    uint64_t h = (k.lo ^ (k.hi << 17)) * 0xff51afd7ed558ccdull;
    return h ^ (h >> 31);
#else
    return fmix64(k.lo ^ fmix64(k.hi ^ 0x9e3779b97f4a7c15ull));
#endif
}

KH_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

// Home slot: Lemire fast range over the high product, exact table size (load 0.5 of 2n slots,
// kmer_hash.cpp:108-109) without a power-of-two round-up.
KH_HD uint64_t home_slot(uint64_t h, uint64_t cap) { return mulhi64(h, cap); }


KH_HD uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// Owner rank of a k-mer in the sharded table: a hash of its minimizer (the M-mer of smallest
// mix32 value among its K-M+1 windows), not of the whole key. Placement never changes the
// output (the reference's owner is std::hash<string> % P, hash_map.hpp:28-30); this one keeps
// runs of consecutive k-mers on one rank so a walker migrates only at minimizer changes.
KH_HD uint32_t owner_key(Key k, const KParams& p, uint32_t nranks) {
    if (nranks == 1) return 0;
    if (p.owner_mode == 1)  // SURVEY §8(e) proposal: hash bits independent of the home slot's
        return (uint32_t)(((key_hash(k) & 0xffffffffull) * nranks) >> 32);
    const uint32_t mask = (uint32_t)((1ull << (2 * p.M)) - 1);
    uint64_t lo = k.lo, hi = k.hi;  // V = hi * 2^62 + lo; windows from the last M bases upward
    uint32_t best = 0xffffffffu;
    for (int j = 0; j <= p.K - p.M; ++j) {
        const uint32_t h = mix32(((uint32_t)lo & mask) ^ 0x5bd1e995u);
        best = h < best ? h : best;
        lo = (lo >> 2) | ((hi & 3u) << 60);
        hi >>= 2;
    }
    return (uint32_t)(((uint64_t)mix32(best ^ 0x9e3779b9u) * nranks) >> 32);
}

// Splitter k-mer: cuts long contigs into independently walked segments (sparse ruling set).
KH_HD bool is_splitter(uint64_t h, const KParams& p) {
    return p.split_bits && (h & ((1ull << p.split_bits) - 1)) == 0;
}

// ---- slot encode/decode ---------------------------------------------------------------
KH_HD uint64_t slot_w0(Key k, uint32_t ext, const KParams& p) {
    return p.W == 1 ? ((k.lo << 6) | ext) : ((k.hi << 6) | ext);
}
KH_HD uint64_t slot_w1(Key k) { return k.lo; }

KH_HD Key slot_key(uint64_t w0, uint64_t w1, const KParams& p) {
    Key k;
    if (p.W == 1) {
        k.hi = 0;
        k.lo = w0 >> 6;
    } else {
        k.hi = w0 >> 6;
        k.lo = w1;
    }
    return k;
}
KH_HD uint32_t slot_ext(uint64_t w0) { return (uint32_t)(w0 & 63u); }
KH_HD uint32_t ext_bwd(uint32_t ext) { return ext & 7u; }
KH_HD uint32_t ext_fwd(uint32_t ext) { return (ext >> 3) & 7u; }

// Record bytes (reference layout) -> key + ext.
KH_HD void parse_record(const uint8_t* rec, const KParams& p, Key& k, uint32_t& ext) {
    k = key_from_packed(rec, p);
    ext = base_code(rec[p.P]) | (base_code(rec[p.P + 1]) << 3);
}

KH_HD void write_record(uint8_t* rec, Key k, uint32_t ext, const KParams& p) {
    key_to_packed(k, rec, p);
    rec[p.P] = code_char(ext_bwd(ext));
    rec[p.P + 1] = code_char(ext_fwd(ext));
}

// ---- reference-compatible djb2 (pkmer_t.hpp:31-37), kept for API parity -----------------
KH_HD uint64_t djb2(const uint8_t* packed, int P) {
    uint64_t h = 5381;
    for (int i = 0; i < P; ++i) h = packed[i] + (h << 5) + h;
    return h;
}

}  // namespace kh
