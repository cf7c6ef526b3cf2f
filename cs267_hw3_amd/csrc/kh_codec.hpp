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
//   Bits of word0 above the key (when the K leaves room, KParams::chain): bits 58-63 = the
//   minimizer window j* (set by the partition passes, see place_hash), bits [idx_lo, 57) = the
//   chain head-record index + 1 (set by the region build, 0 = none), bit 57 = scratch of the build.
//   Every key comparison masks them (slot_keybits).
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
    int M;              // minimizer length (bases): placement region and sharded owner
    int owner_mode;     // sharded owner: 0 = minimizer hash (default), 1 = low key_hash bits
    int split_bits;     // walk splitters: k-mers passing split_test(k, split_bits) and a
                        // predecessor start extra walkers (0 = off); see kh_kernels.hip k_walk
    uint64_t kmask;     // key bits of (word0 >> 6): hi_mask (W=2) or v_mask (W=1)
    int chain;          // word0 has room for j* and a head-record index (chain links, kh_build.hip)
    int idx_lo;         // first bit of the head-record index field in word0 (field = [idx_lo, 57))
    int rbits;          // placement regions = 2^rbits (9..17, by table size: set_region_bits)
    // device bitmap of remapped ("hot") regions, one bit per region (nullptr = none): a region
    // whose minimizer windows bring more k-mers than its window or slice holds has all its keys
    // placed by a hash of the whole key instead (kh_build.hip k_hot_mark; place_w)
    const uint32_t* hot;
    // balanced region bounds (tables above load ~0.6): rb[r] = first slot of region r, rb[2^rbits]
    // = cap, sized from the build's region counts (kh_build.hip k_bounds); nullptr = 2^rbits
    // equal ranges
    const uint64_t* rb;
};

// Minimizer length: consecutive k-mers of a contig share their minimizer for ~(K-M+2)/2 steps on
// random sequence (K=51, M=16: 18.6 k-mers), so a contig's k-mers come in runs that share a
// placement region (and a rank). M must make minimizer *windows* rare in the data: a region's
// load is a sum over the minimizer windows mapped to it, and a window that recurs (a 12-mer
// occurs ~18x in C3's 296M bases) brings all its runs along: C3 region loads (mean 1526 per
// 3052-slot slice) have sd 642 and spill 0.8M keys at M=12, sd 210 and none at M=16
// (simulated at full size).
inline int minimizer_len(int K) { return K >= 31 ? 16 : K >= 20 ? 14 : K >= 14 ? 12 : K; }
static constexpr int JSTAR_SHIFT = 58;   // word0 bits 58-63: minimizer window index j*
static constexpr int SCRATCH_BIT = 57;   // word0 bit 57: build scratch (has a local predecessor)
static constexpr int REGION_BITS_MIN = 9, REGION_BITS_MAX = 17;  // placement regions: 2^rbits
static constexpr uint64_t REGION_SLOTS = 3072;  // target slots per region (one LDS slice)

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
    p.kmask = p.W == 2 ? p.hi_mask : p.v_mask;
    p.idx_lo = 6 + (p.W == 2 ? (hib > 0 ? hib : 0) : 2 * K);
    // chain links need j* (6 bits, K-M+1 <= 49 windows) and an index field of >= 8 bits
    p.chain = (SCRATCH_BIT - p.idx_lo >= 8) && K >= 14 ? 1 : 0;
    p.rbits = REGION_BITS_MAX;
    p.hot = nullptr;
    p.rb = nullptr;
    return p;
}

// Compile-time copy of the shape fields for the bench shapes (KT = 51 or 19; 0 = as given):
// kernels templated on KT call the codec through this copy, so K, W, masks and field positions
// fold into constants (runtime fields: split_bits, rbits, owner_mode).
template <int KT>
KH_HD KParams specialize(const KParams& p) {
    if constexpr (KT == 0) {
        return p;
    } else {
        KParams q = p;
        q.K = KT;
        q.P = (KT + 3) / 4;
        q.R = q.P + 2;
        q.pad = 4 * q.P - KT;
        q.W = KT <= KMAX_W1 ? 1 : 2;
        q.hi_mask = 2 * KT - 62 > 0 ? ((1ull << (2 * KT - 62)) - 1) : 0ull;
        q.v_mask = 2 * KT >= 64 ? ~0ull : ((1ull << (2 * KT)) - 1);
        q.M = KT >= 31 ? 16 : KT >= 20 ? 14 : KT >= 14 ? 12 : KT;
        q.kmask = q.W == 2 ? q.hi_mask : q.v_mask;
        q.idx_lo = 6 + (q.W == 2 ? (2 * KT - 62 > 0 ? 2 * KT - 62 : 0) : 2 * KT);
        q.chain = (57 - q.idx_lo >= 8) && KT >= 14 ? 1 : 0;
        return q;
    }
}
// the specialization a table's K gets (0 = generic)
inline int kt_of(int K) { return K == 51 ? 51 : K == 19 ? 19 : 0; }

// Regions of ~REGION_SLOTS slots: a region's load is a sum of minimizer runs (~20 k-mers), so
// small slices would overflow (at 38 slots per region a quarter of the keys did); 2^9..2^17.
inline void set_region_bits(KParams& p, uint64_t cap) {
    int b = REGION_BITS_MIN;
    while (b < REGION_BITS_MAX && (cap >> b) > REGION_SLOTS) ++b;
    p.rbits = b;
}

KH_HD uint32_t base_code(uint8_t c) {
    // 'A'=65 'C'=67 'G'=71 'T'=84 'F'=70 -> 0 1 2 3 EXT_F, anything else EXT_BAD. Branchless (no
    // divergent switch on the device): the low nibbles of the five are distinct, a 16 x 4-bit table
    // gives the candidate code and the code's own character confirms the whole byte.
    const uint32_t k = (uint32_t)(0x5555555524531505ull >> ((c & 15u) * 4u)) & 15u;
    const uint32_t back = (uint32_t)(0x4654474341ull >> (k * 8u)) & 0xFFu;  // k = 5: 0
    return back == c ? k : EXT_BAD;
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
KH_HD uint64_t key_hash(Key k) { return fmix64(k.lo ^ fmix64(k.hi ^ 0x9e3779b97f4a7c15ull)); }

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

// 32-bit key hash (3 x mix32): the in-region home slot and the splitter test. Cheaper than
// key_hash's two 64-bit fmix rounds; placement never changes outputs.
KH_HD uint32_t key_hash32(Key k) {
    uint32_t h = (uint32_t)k.lo * 0x9E3779B1u + (uint32_t)(k.lo >> 32);
    h = (h ^ (h >> 15)) * 0x85EBCA77u + ((uint32_t)k.hi ^ (uint32_t)(k.hi >> 32));
    h = (h ^ (h >> 13)) * 0xC2B2AE3Du;
    return h ^ (h >> 16);
}

// ---- minimizer ---------------------------------------------------------------------------------
// Window j (0 = the last M bases, K-M = the first M) = bits [2j, 2j + 2M) of V. Its order is
// (w[23:0] * C) mod 2^26 for an odd 18-bit C (a bijection of the window's low 12 bases), and the
// scan's key is w[23:0] * (C << 6) + j: one v_mad_u32_u24 with j as an inline addend per window,
// the order in the top 26 bits and j* in the low 6 (round 4's key, (w[23:0] * C' + w) >> 6 << 6 | j,
// took one v_and_or more per window: 36 VALU per scan, in the records pass and in every walk hop).
// The minimizer is the window of smallest order, ties to the smallest j (j*). Packed result:
// order26 << 6 | j*. The region and the owner rank hash the minimizer window's *content* (2M bits),
// never its order (distinct windows share an order when their low 12 bases agree).
static constexpr uint32_t MINI_C6 = 0x278DDu << 6;  // < 2^24: the u24 multiplier operand
KH_HD uint32_t win_order(uint32_t w) { return ((w & 0xFFFFFFu) * MINI_C6) >> 6; }
KH_HD uint32_t win_key(uint32_t w, uint32_t j) { return (w & 0xFFFFFFu) * MINI_C6 + j; }
#if defined(__HIP_DEVICE_COMPILE__)
// c = MINI_C6 passed through an empty asm: with the constant visible the compiler proves the
// product's low 6 bits zero, turns "+ j" into an or and no longer folds the pair into one
// v_mad_u32_u24 (it emitted v_mul_u32_u24 + v_or_b32 per window)
__device__ __forceinline__ uint32_t mini_c6() {
    uint32_t c = MINI_C6;
    asm volatile("" : "+s"(c));
    return c;
}
__device__ __forceinline__ uint32_t win_key_d(uint32_t w, uint32_t c, uint32_t j) {
    return (uint32_t)__umul24(w, c) + j;
}
#endif

KH_HD uint32_t win_bits(Key k, int j, const KParams& p) {
    const int b = 2 * j;  // V = hi * 2^62 + lo
    const uint64_t t = b < 62 ? (k.lo >> b) | (k.hi << (62 - b)) : k.hi >> (b - 62);
    return (uint32_t)t & (uint32_t)((1ull << (2 * p.M)) - 1);
}

#if defined(__HIP_DEVICE_COMPILE__)
// V as four 32-bit words; every window is one alignbit at a constant shift (unrolled). K and M
// known at compile time (the bench shapes) drop the per-window bounds branch and mask.
template <int K, int M>
__device__ __forceinline__ uint32_t mini_scan_t(Key k) {
    const uint32_t v[5] = {(uint32_t)k.lo, (uint32_t)(k.lo >> 32) | (uint32_t)(k.hi << 30), (uint32_t)(k.hi >> 2),
                           (uint32_t)(k.hi >> 34), 0u};
    constexpr uint32_t mmask = (uint32_t)((1ull << (2 * M)) - 1);
    const uint32_t c6 = mini_c6();
    uint32_t best = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j <= K - M; ++j) {
        const int b = 2 * j;
        const uint32_t w = (b & 31) ? __builtin_amdgcn_alignbit(v[(b >> 5) + 1], v[b >> 5], b & 31) : v[b >> 5];
        const uint32_t o = win_key_d(w & mmask, c6, (uint32_t)j);
        best = o < best ? o : best;
    }
    return best;
}
#endif

KH_HD uint32_t mini_scan(Key k, const KParams& p) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (p.K == 51 && p.M == 16) return mini_scan_t<51, 16>(k);  // uniform branches
    if (p.K == 19 && p.M == 12) return mini_scan_t<19, 12>(k);
    const uint32_t v[5] = {(uint32_t)k.lo, (uint32_t)(k.lo >> 32) | (uint32_t)(k.hi << 30), (uint32_t)(k.hi >> 2),
                           (uint32_t)(k.hi >> 34), 0u};
    const uint32_t mmask = (uint32_t)((1ull << (2 * p.M)) - 1);
    const int last = p.K - p.M;
    const uint32_t c6 = mini_c6();
    uint32_t best = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j <= KMAX - 1; ++j) {
        if (j <= last) {
            const int b = 2 * j;
            const uint32_t w = (b & 31) ? __builtin_amdgcn_alignbit(v[(b >> 5) + 1], v[b >> 5], b & 31) : v[b >> 5];
            const uint32_t o = win_key_d(w & mmask, c6, (uint32_t)j);
            best = o < best ? o : best;
        }
    }
    return best;
#else
    uint32_t best = 0xFFFFFFFFu;
    for (int j = 0; j <= p.K - p.M; ++j) {
        const uint32_t o = win_key(win_bits(k, j, p), (uint32_t)j);
        best = o < best ? o : best;
    }
    return best;
#endif
}
// content of the minimizer window of k (mn = mini_scan(k))
KH_HD uint32_t mini_window(Key k, uint32_t mn, const KParams& p) { return win_bits(k, (int)(mn & 63u), p); }

// Region of a minimizer window (rbits bits of a mix of its content).
KH_HD uint32_t mini_region(uint32_t win, const KParams& p) { return mix32(win ^ 0x5bd1e995u) >> (32 - p.rbits); }

// Placement: the k-mer's region is a hash of its minimizer window; region r owns the slot range
// [region_lo(r), region_lo(r + 1)) (2^rbits equal ranges of the cap slots), and the home slot is
// region_lo(r) + the region length scaled by the 32-bit key hash. A run of consecutive k-mers of
// a contig (same minimizer) lands in one region: the region build links them into chains
// (kh_build.hip) that the walker crosses in one step.
KH_HD uint64_t region_lo(uint32_t r, uint64_t cap, const KParams& p) {
    if (p.rb) return p.rb[r];
    return (r >> p.rbits) ? cap : mulhi64((uint64_t)r << (64 - p.rbits), cap);
}
KH_HD uint64_t home_in(uint64_t lo, uint64_t hi, uint32_t h) { return lo + (((hi - lo) * (uint64_t)h) >> 32); }
struct Place {
    uint32_t r, h;  // region, key_hash32
};
// Hot regions (a repeat family, a low-complexity run, the C5 hot-bucket set: one minimizer window
// shared by far more k-mers than a region holds) are remapped as a whole: their keys go to the
// region of a hash of (the minimizer window, the k-mer's secondary window: the M bases next to the
// minimizer's occurrence on the side of window index j* + M when they fit in the k-mer, else on the
// other side). The secondary window is a fixed stretch of the contig next to the shared one: along
// a run the occurrence moves up one window index per step and the neighbour with it, so a run keeps
// it (it changes at most once, where the first side stops fitting and the other starts) and a
// run still lands in one region and keeps its chain, while the family spreads over one region per
// distinct neighbour (a hash of the whole key spread it too, but broke every run: the C5
// hot-bucket walk was one lookup per k-mer). The neighbour never overlaps the shared window: a
// window overlapping it (the lowest-order other window, say) takes few distinct values over a
// family and piles it into a few regions again. The home inside the region is home_in(.., key_hash32).
// js: the occurrence's window index j* (mini_scan's low 6 bits: the first window of the smallest
// order, so the first with the minimizer's content), or -1 to find it from win
// window index of the minimizer occurrence (js < 0: found from its content win)
KH_HD int occurrence(Key k, uint32_t win, const KParams& p, int js) {
    if (js >= 0) return js;
    for (int j = 0; j <= p.K - p.M; ++j)
        if (win_bits(k, j, p) == win) return j;
    return 0;
}
KH_HD int second_index(int js, const KParams& p) {
    return js + 2 * p.M <= p.K ? js + p.M : (js >= p.M ? js - p.M : (2 * js < p.K - p.M ? p.K - p.M : 0));
}
KH_HD uint32_t second_window(Key k, uint32_t win, const KParams& p, int js = -1) {
    return win_bits(k, second_index(occurrence(k, win, p, js), p), p);
}
KH_HD uint32_t hot_region(Key k, uint32_t win, const KParams& p, int js = -1) {
    return mix32((win * 0x9E3779B1u) ^ second_window(k, win, p, js) ^ 0x2545F491u) >> (32 - p.rbits);
}
KH_HD bool region_is_hot(const uint32_t* hot, uint32_t r) { return hot && ((hot[r >> 5] >> (r & 31u)) & 1u); }
// The bitmap has two levels of 2^17 bits (KParams::hot): level 1 marks minimizer regions whose keys
// are remapped (hot_region); level 2 marks target regions that the remap itself overfills — a family
// whose copies also share the neighbour window (a shared stretch of 2M bases: a repeat) lands in one
// target region — and the remapped keys headed there spread by the bases next to that stretch
// (spread_region). Level 2 is read only for keys level 1 remapped.
static constexpr uint32_t HOT_LEVEL_WORDS = (1u << REGION_BITS_MAX) / 32;
// Level-2 placement of a remapped key whose target region t overfilled: t mixed with the SPREAD_B
// bases right next to the shared stretch (the minimizer and neighbour windows) on the right when
// they fit in the k-mer, else on the left. Those bases are fixed positions of the contig, so along
// a run (the stretch moves one window index per k-mer) they stay the same until the side switches:
// a run changes region at most once more and keeps its chains, while the family spreads over up to
// 4^SPREAD_B regions. Short k (K < 2M + 2 SPREAD_B - 1, no room on either side): whole-key hash.
static constexpr int SPREAD_B = 8;
KH_HD uint32_t spread_region(Key k, uint32_t t, uint32_t win, const KParams& p, int js) {
    if (p.K >= 2 * p.M + 2 * SPREAD_B - 1) {
        const int j = occurrence(k, win, p, js), j2 = second_index(j, p);
        const int lo = j < j2 ? j : j2, hi = (j < j2 ? j2 : j) + p.M;
        const int at = lo >= SPREAD_B ? lo - SPREAD_B : hi;  // K - hi >= SPREAD_B when lo < SPREAD_B
        const uint32_t b = win_bits(k, at, p) & ((1u << (2 * SPREAD_B)) - 1u);
        return mix32((t * 0x85EBCA6Bu) ^ (b * 0x9E3779B1u) ^ 0x68E31DA4u) >> (32 - p.rbits);
    }
    return (uint32_t)(key_hash(k) >> 32) >> (32 - p.rbits);
}
KH_HD uint32_t remap_region(Key k, uint32_t win, const KParams& p, int js = -1) {
    const uint32_t t = hot_region(k, win, p, js);
    return region_is_hot(p.hot + HOT_LEVEL_WORDS, t) ? spread_region(k, t, win, p, js) : t;
}
KH_HD Place place_w(uint32_t win, Key k, const KParams& p, int js = -1) {
    uint32_t r = mini_region(win, p);
    const uint32_t h = key_hash32(k);
    if (region_is_hot(p.hot, r)) r = remap_region(k, win, p, js);
    return Place{r, h};
}
KH_HD Place place(Key k, const KParams& p) {
    const uint32_t mn = mini_scan(k, p);
    return place_w(mini_window(k, mn, p), k, p, (int)(mn & 63u));
}
KH_HD uint64_t home_of(Place pl, uint64_t cap, const KParams& p) {
    return home_in(region_lo(pl.r, cap, p), region_lo(pl.r + 1, cap, p), pl.h);
}

// Owner rank of a k-mer in the sharded table: a hash of its minimizer, not of the whole key.
// Placement never changes the output (the reference's owner is std::hash<string> % P,
// hash_map.hpp:28-30); this one keeps runs of consecutive k-mers on one rank so a walker migrates
// only at minimizer changes, and a chain (same minimizer) never crosses ranks.
KH_HD uint32_t owner_of_mini(uint32_t win, uint32_t nranks) {
    return (uint32_t)(((uint64_t)mix32(win ^ 0x9e3779b9u) * nranks) >> 32);
}
KH_HD uint32_t owner_key(Key k, const KParams& p, uint32_t nranks) {
    if (nranks == 1) return 0;
    if (p.owner_mode == 1)  // SURVEY §8(e) proposal: hash bits independent of the home slot's
        return (uint32_t)(((key_hash(k) & 0xffffffffull) * nranks) >> 32);
    return owner_of_mini(mini_window(k, mini_scan(k, p), p), nranks);
}

// Splitter k-mer: cuts long contigs into independently walked segments (sparse ruling set). The
// top `bits` bits of a one-multiply hash of the key's low word are zero (nested in bits, as the
// walk's density filter needs). One multiply instead of key_hash32's three: the walker tests every
// k-mer it appends and the records pass every record (key_hash32 was ~7 % of k_win1_rec's VALU).
KH_HD uint32_t split_hash(Key k) { return ((uint32_t)k.lo ^ (uint32_t)(k.lo >> 32)) * 0x9E3779B1u; }
KH_HD bool split_test(Key k, int bits) { return bits && split_hash(k) < (1u << (32 - bits)); }
KH_HD bool is_splitter(Key k, const KParams& p) { return split_test(k, p.split_bits); }

// ---- slot encode/decode ---------------------------------------------------------------
KH_HD uint64_t slot_w0(Key k, uint32_t ext, const KParams& p) {
    return p.W == 1 ? ((k.lo << 6) | ext) : ((k.hi << 6) | ext);
}
KH_HD uint64_t slot_w1(Key k) { return k.lo; }

// key bits of word0 (the j* / head-index bits above the key masked off)
KH_HD uint64_t slot_keybits(uint64_t w0, const KParams& p) { return (w0 >> 6) & p.kmask; }

KH_HD Key slot_key(uint64_t w0, uint64_t w1, const KParams& p) {
    Key k;
    if (p.W == 1) {
        k.hi = 0;
        k.lo = slot_keybits(w0, p);
    } else {
        k.hi = slot_keybits(w0, p);
        k.lo = w1;
    }
    return k;
}
// j* carried by a word of the partition passes
KH_HD uint32_t slot_jstar(uint64_t w0) { return (uint32_t)(w0 >> JSTAR_SHIFT); }
KH_HD uint64_t with_jstar(uint64_t w0, uint32_t j) {
    return (w0 & ((1ull << JSTAR_SHIFT) - 1)) | ((uint64_t)j << JSTAR_SHIFT);
}
// head-record index + 1 of a built slot (0 = the walker steps this k-mer itself)
KH_HD uint32_t slot_hidx(uint64_t w0, const KParams& p) {
    return (uint32_t)((w0 >> p.idx_lo) & ((1ull << (SCRATCH_BIT - p.idx_lo)) - 1));
}
KH_HD uint64_t with_hidx(uint64_t w0, uint32_t v, const KParams& p) {
    const uint64_t f = ((1ull << (SCRATCH_BIT - p.idx_lo)) - 1) << p.idx_lo;
    return (w0 & ~f) | (((uint64_t)v << p.idx_lo) & f);
}
// placement regions of the table (2^rbits)
KH_HD uint32_t nreg(const KParams& p) { return 1u << p.rbits; }

// Head records (kh_build.hip chain_heads): word 0 = the run's tail k-mer word 0 (key + ext), the
// link count in the low 6 bits of the index field and, from bit idx_lo + 6 up, the head-record
// index + 1 (within its region) of the run that follows the tail, 0 = none: the walker then looks
// the next k-mer up. The build writes 0 there; k_rec_succ resolves it before a walk.
KH_HD uint32_t rec_links(uint64_t r0, const KParams& p) { return (uint32_t)(r0 >> p.idx_lo) & 63u; }
KH_HD int rec_succ_shift(const KParams& p) { return p.idx_lo + 6; }
KH_HD uint32_t rec_succ(uint64_t r0, const KParams& p) { return (uint32_t)(r0 >> rec_succ_shift(p)); }
// key + ext + j* only (head index and scratch cleared)
KH_HD uint64_t slot_clean(uint64_t w0, const KParams& p) {
    return p.chain ? (w0 & (((1ull << p.idx_lo) - 1) | (63ull << JSTAR_SHIFT))) : w0;
}
// minimizer window / placement of a partition word: from its j* when the word carries one
KH_HD uint32_t word_mini_window(uint64_t w0, uint64_t w1, const KParams& p) {
    const Key k = slot_key(w0, w1, p);
    return win_bits(k, p.chain ? (int)slot_jstar(w0) : (int)(mini_scan(k, p) & 63u), p);
}
KH_HD Place word_place(uint64_t w0, uint64_t w1, const KParams& p) {
    const Key k = slot_key(w0, w1, p);
    const int js = p.chain ? (int)slot_jstar(w0) : (int)(mini_scan(k, p) & 63u);
    return place_w(win_bits(k, js, p), k, p, js);
}
// Partition words also carry the top bits of their minimizer order in the (then unused)
// head-index field, so the region build's link test needs no window extraction.
KH_HD int mtop_bits(const KParams& p) { return SCRATCH_BIT - p.idx_lo < 26 ? SCRATCH_BIT - p.idx_lo : 26; }
KH_HD uint32_t order_top(uint32_t order26, const KParams& p) { return order26 >> (26 - mtop_bits(p)); }
// word0 of a partition word: key + ext, j* and the minimizer order's top bits (chains only)
KH_HD uint64_t part_word0(uint64_t w0, uint32_t mn, const KParams& p) {
    return p.chain ? with_hidx(with_jstar(w0, mn & 63u), order_top(mn >> 6, p), p) : w0;
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
