// kh_build.hip — atomic-free bulk build of the open-addressing k-mer table (gfx950).
//
// Replaces one-CAS-per-key global inserts (bound at ~20 G random CAS/s on MI355X, measured by
// tools/membench) with streaming passes:
//   pass 1   group the batch by the top 9 bits of the placement hash (512 buckets x S1 windows;
//            place: region = a hash of the k-mer's minimizer window, kh_codec.hpp); records
//            are parsed by the pass itself (k_win1_rec) or converted to words first
//            (k_part1_convert, other k), routed words go straight in (k_win1)
//   pass 2   then by the next 8 bits, within each pass-1 bucket, into 2^17 region windows (k_win2)
//            (each 8192-item tile is counting-sorted by bin in LDS so waves write contiguous
//             runs; a run is reserved in its window with one atomicAdd per (tile, bin))
//   build    one workgroup per region (top 17 hash bits) builds its slot range (~cap/2^17 slots,
//            ~49 KB at 200M k-mers) in LDS with LDS CAS linear probing, then writes the slice
//            out with coalesced 16-B stores
//   overflow keys whose probe run leaves their slice take the global CAS path afterwards, so
//            every key satisfies the linear-probing invariant "all slots from home to position
//            are occupied"
//   chains   with the region's keys in LDS, every k-mer whose successor (next_kmer) shares its
//            minimizer (provable from j*: the minimizer window survives the shift and the new
//            window orders above it) looks the successor up in LDS; each chain head (no linked
//            predecessor) gets a head record {tail key + ext, links} and its slot the record index,
//            so the walker crosses a run of ~20 k-mers (K=51) with two requests instead of ~20
// Placement differs from the CAS path; find()/the walk depend only on the invariant, so outputs
// are identical (tests run both paths).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "kh_device.hpp"

#include <cstdio>

namespace kh {

static constexpr int PB = 256;                    // threads per block of the small kernels
// radix bits per pass (pass 2: p.rbits - B1); 8 pass-1 bits measured the same (round 4)
static constexpr int B1 = 9, B2 = REGION_BITS_MAX - B1;
static constexpr int NB1 = 1 << B1, NB2 = 1 << B2;
static constexpr int NBX = NB1 > NB2 ? NB1 : NB2;  // bins of the larger pass (LDS layout)
static constexpr uint32_t NREG_MAX = 1u << (B1 + B2);
static_assert(B1 <= REGION_BITS_MIN && B1 + B2 == REGION_BITS_MAX && NBX <= 512, "regions of the placement hash");
static constexpr int BUILD_THREADS = 512;
static constexpr int T1 = 2;                      // consecutive tiles per pass-1 block
static constexpr uint32_t S1 = 8;                 // pass-1 windows (atomic counters) per bucket
static constexpr uint32_t NW1 = NB1 * S1;
static_assert(NW1 <= PART_W1_COUNTERS, "counter layout");
// splitter buffer of k_win1 in the dynamic-LDS tail: (4 KB - 2 KB gpos - wsum - counter) / 16 B
static constexpr uint32_t WIN_SPLIT_LCAP = 120;
static_assert(PART_TILE * 18 + 3 * 512 * 4 + 8 + WIN_SPLIT_LCAP * 16 + 8 <= PART_TILE * 16 + PART_TILE * 2 + 512 * 16,
              "k_win1 LDS tail");
static constexpr uint64_t LDS_BYTES = 160 * 1024;
// the windowed passes (k_win1 / k_win2) sort tiles of WIN_TILE words: 8192 doubles the runs each
// bin gets per tile (C3 pass 1: 16 words = 256 B instead of 128 B) in 152 KiB of LDS
static constexpr int WIN_TILE = 8192;
constexpr size_t sort_lds(int tile) { return (size_t)tile * 16 + tile * 2 + 2 * NBX * 4 + NBX * 8; }
constexpr size_t sort_lds_nb(int tile, int nb) { return (size_t)tile * 16 + tile * 2 + 2 * nb * 4 + nb * 8; }
static_assert(sort_lds(WIN_TILE) + 64 <= 160 * 1024, "k_win LDS");
static constexpr int REC_TILE = 3584;  // records pass 1 (k_win1_rec): two blocks per CU
static_assert(2 * (sort_lds(REC_TILE) + 64) <= 160 * 1024, "k_win1_rec LDS");
// records pass 1: 512 threads per block (640 threads over 3840-record tiles, 20 waves per CU
// instead of 16: C3 8.50 -> 9.07 ms; profiles/r05/ab/ab_rec640.txt)
static constexpr int REC_TB = 512, REC_TILE_P1 = REC_TILE;
static uint64_t win_blocks1(uint64_t n) { return (n + (uint64_t)T1 * WIN_TILE - 1) / ((uint64_t)T1 * WIN_TILE); }
// pass-2 blocks per bucket
static uint64_t win_G(uint64_t n) {
    const uint64_t tiles_per_bucket = (n / NB1 + WIN_TILE - 1) / WIN_TILE + 1;
    constexpr uint64_t tpb = 2;  // tiles per pass-2 block (1 / 2 / 3 measured the same, round 4)
    return (tiles_per_bucket + tpb - 1) / tpb;
}

uint64_t part_count_words() { return (NW1 + 2 * NREG_MAX) / 2; }

// Every word can miss its windows (a hot bucket fills all of its pass-1 windows): the list holds
// the whole batch, so it never runs out while the table has free slots.
uint64_t part_overflow_cap(uint64_t n) { return n + 65536; }

// Window capacities. Regions are picked by minimizer, so a region's load is a sum of runs of
// ~19 k-mers (compound Poisson: variance = mu * E[S^2]/E[S] ~ 30 mu at K=51, M=16: C3 sd 210 for
// mu 1526, simulated): the region windows hold mu + 7 sigma; pass-1 windows see 1/S1 of a bucket
// (sigma^2 = mu1 (1 + 30/S1)). A full window spills to the overflow list (global CAS inserts),
// never loses a key.
static constexpr double CLUMP = 30.0;
uint32_t part_region_cap(const KParams& p, uint64_t n) {
    const double mu = (double)n / nreg(p);
    return (uint32_t)(mu + 7.0 * sqrt(CLUMP * mu) + 16.0);
}

uint32_t part_win1_cap(uint64_t n) {
    const double mu = (double)n / NW1;
    return (uint32_t)(mu + 10.0 * sqrt(mu * (1.0 + CLUMP / S1)) + 64.0);
}

uint64_t part_buf1_words(const KParams& p, uint64_t n) {
    const uint64_t w = (uint64_t)NW1 * part_win1_cap(n);
    return (w > n ? w : n) * p.W;
}

uint64_t part_buf2_words(const KParams& p, uint64_t n) {
    const uint64_t w = (uint64_t)nreg(p) * part_region_cap(p, n);
    return (w > n ? w : n) * p.W;
}

// Largest region slice a build holds in LDS. Equal ranges: cap / 2^rbits (+1). Balanced bounds
// (p.rb): as much as three 512-thread blocks per CU leave (~53 KB: 3,260 16-B slots), so a region
// may take up to that many slots (k_bounds falls back to equal ranges when one would not fit).
static uint64_t region_max_slots(const KParams& p, uint64_t cap) {
    const uint64_t eq = cap / nreg(p) + 1;
    if (!p.rb) return eq;
    // LDS per block = 8 W sm + (sm / 8 + 32) * 2 + 16 <= LDS_BYTES / 3
    uint64_t sm = ((LDS_BYTES / 3 - 96) * 4) / (32ull * p.W + 1);
    if (p.chain && sm >= (1ull << (58 - p.idx_lo)) - 1) sm = (1ull << (58 - p.idx_lo)) - 2;
    return sm > eq ? sm : eq;
}
// build LDS: the slice, plus the chain head list (<= slots/8 + 32 entries, part_head_cap) when
// chains are built (successors live in the slots' own index fields)
static uint64_t build_lds(const KParams& p, uint64_t cap, bool chains) {
    const uint64_t sm = region_max_slots(p, cap);
    return sm * 8ull * p.W + (chains ? (sm / 8 + 32) * 2 : 0) + 16;
}

bool region_slots_fit(const KParams& p, uint64_t cap) { return build_lds(p, cap, false) <= LDS_BYTES; }

// head records per region: room for chains of >= 8 slots (C3: 413 for ~75 heads); 0 = no chains
uint32_t part_head_cap(const KParams& p, uint64_t cap) {
    // a slot's successor (index + 1) must fit its [idx_lo, 58) field while the build links
    if (!p.chain || build_lds(p, cap, true) > LDS_BYTES || region_max_slots(p, cap) >= (1ull << (58 - p.idx_lo)))
        return 0;
    const uint64_t lim = (1ull << (SCRATCH_BIT - p.idx_lo)) - 1;
    const uint64_t h = region_max_slots(p, cap) / 8 + 32;
    return (uint32_t)(h < lim ? h : lim);
}

bool part_usable(const KParams& p, uint64_t cap, uint64_t n) {
    return n >= (1ull << 20) && region_slots_fit(p, cap) && cap >= (uint64_t)nreg(p) * 8;
}


// Region of a partition word in passes 1 and 2: the minimizer region, or the key-hash region when
// that one is remapped (hot_on: the table has remapped regions; one uniform test per block).
__device__ __forceinline__ uint32_t part_region(uint32_t win, Key k, const KParams& p, bool hot_on, int js = -1) {
    const uint32_t r = mini_region(win, p);
    return (hot_on && region_is_hot(p.hot, r)) ? remap_region(k, win, p, js) : r;
}

// ---- record -> word conversion (k other than 51 / 19) ---------------------------------------------
// Parse the reference records once, one per thread per 256-record sub-tile (the next sub-tile's
// 16-B loads are in flight while this one is parsed), emit internal words in input order and the
// start / splitter bits; the windowed pass 1 then reads the words.
template <int PK>
__device__ __forceinline__ void parse_record_regs_t(uint64_t x0, uint64_t x1, int pad, Key& k, uint32_t& ext);

template <int W, int PK = 0, int KT = 0>
__global__ __launch_bounds__(PB) void k_part1_convert(KParams p_in, const uint8_t* __restrict__ recs,
                                                      uint64_t n, uint64_t* words_out,
                                                      uint64_t* start_mask, uint64_t* split_mask, uint32_t* samp) {
    const KParams p = specialize<KT>(p_in);
    __shared__ __attribute__((aligned(16))) uint8_t stage[2][PB * 17 + 16];
    const uint64_t b0 = (uint64_t)blockIdx.x * T1 * PART_TILE;
    const uint64_t b1 = min(b0 + (uint64_t)T1 * PART_TILE, n);
    const uint32_t R = (uint32_t)p.R;
    const uint32_t nsub = (uint32_t)((b1 - b0 + PB - 1) / PB);
    uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0;
    auto fetch = [&](uint32_t j) {
        const uint64_t sub = b0 + (uint64_t)j * PB;
        const uint32_t nvec = (uint32_t)(min((uint64_t)PB, b1 - sub) * R) >> 4;
        const uint4* src = reinterpret_cast<const uint4*>(recs + sub * R);
        if (threadIdx.x < nvec) r0 = src[threadIdx.x];
        if (threadIdx.x + PB < nvec) r1 = src[threadIdx.x + PB];
    };
    if (nsub) fetch(0);
    for (uint32_t j = 0; j < nsub; ++j) {
        const uint64_t sub = b0 + (uint64_t)j * PB;
        const uint32_t cnt = (uint32_t)min((uint64_t)PB, b1 - sub);
        const uint32_t bytes = cnt * R, nvec = bytes >> 4;
        uint8_t* st = stage[j & 1];
        if (threadIdx.x < nvec) reinterpret_cast<uint4*>(st)[threadIdx.x] = r0;
        if (threadIdx.x + PB < nvec) reinterpret_cast<uint4*>(st)[threadIdx.x + PB] = r1;
        for (uint32_t x = (nvec << 4) + threadIdx.x; x < bytes; x += PB) st[x] = recs[sub * R + x];
        if (j + 1 < nsub) fetch(j + 1);
        lds_barrier();  // LDS hand-off only: __syncthreads would also wait for the prefetch above
        const bool valid = threadIdx.x < cnt;
        Key k{0, 0};
        uint32_t ext = 0;
        if (valid) {
            if constexpr (PK != 0) {  // 3 aligned 8-B LDS reads + funnel shifts instead of 15 byte reads
                const uint32_t a = threadIdx.x * (uint32_t)(PK + 2), a8 = a & ~7u, sh = (a & 7u) * 8u;
                const uint64_t* q = reinterpret_cast<const uint64_t*>(st + a8);
                const uint64_t u0 = q[0], u1 = q[1], u2 = q[2];
                const uint64_t x0 = sh ? (u0 >> sh) | (u1 << (64 - sh)) : u0;
                const uint64_t x1 = sh ? (u1 >> sh) | (u2 << (64 - sh)) : u1;
                parse_record_regs_t<PK>(x0, x1, p.pad, k, ext);
            } else {
                parse_record(st + threadIdx.x * R, p, k, ext);
            }
        }
        const bool is_start = valid && ext_bwd(ext) == EXT_F;
        const uint64_t bal = __ballot(is_start);
        const uint64_t wb = sub + (threadIdx.x & ~63u);
        if ((threadIdx.x & 63) == 0 && wb < b1 && start_mask) start_mask[wb >> 6] = bal;
        if (split_mask) {
            const uint64_t sb = __ballot(valid && !is_start && is_splitter(k, p));
            if ((threadIdx.x & 63) == 0 && wb < b1) split_mask[wb >> 6] = sb;
        }
        if (valid) {
            // the word carries its minimizer window j* (pass 1 reads the region from it)
            const uint32_t mn = mini_scan(k, p);
            // 1-in-256 sample of the minimizer regions (one lane per sub-tile; records are in
            // shuffled order) for the hot-region mark before pass 1
            if (samp && threadIdx.x == 0) atomicAdd(&samp[mini_region(mini_window(k, mn, p), p)], 1u);
            const uint64_t w0 = part_word0(slot_w0(k, ext, p), mn, p);
            const uint64_t i = sub + threadIdx.x;
            if (W == 2) {
                *reinterpret_cast<ulonglong2*>(words_out + i * 2) = make_ulonglong2(w0, k.lo);
            } else {
                words_out[i] = w0;
            }
        }
    }
}

// Both extension bytes (e = c0 | c1 << 8) -> base_code(c0) | base_code(c1) << 3, with v_perm_b32 as
// an 8-entry byte table indexed by c & 7 (A C G T F -> 1 3 7 4 6, distinct): one table of codes,
// one of the character each index stands for; a byte that is not its index's character is
// EXT_BAD, base_code's exact test (checked against base_code for all 2^16 byte pairs when written).
// 2 perms + ~7 VALU instead of ~18 (two 64-bit table shifts per byte).
__device__ __forceinline__ uint32_t ext_codes2(uint32_t e) {
    const uint32_t sel = (e & 0x0707u) | 0x0C0C0000u;                 // bytes 2, 3: 0x00
    const uint32_t code = __builtin_amdgcn_perm(0x02040503u, 0x01050005u, sel);  // 5 0 5 1 | 3 5 4 2
    const uint32_t back = __builtin_amdgcn_perm(0x47460054u, 0x43004100u, sel);  // - A - C | T - F G
    const uint32_t d = back ^ e;
    const uint32_t c0 = (d & 0xFFu) ? EXT_BAD : (code & 0xFFu);
    const uint32_t c1 = (d & 0xFF00u) ? EXT_BAD : (code >> 8);
    return c0 | (c1 << 3);
}
static_assert(EXT_BAD == 5 && EXT_F == 4, "ext_codes2 tables");

// same with the packed size PK known at compile time: constant shifts, no SALU per record
template <int PK>
__device__ __forceinline__ void parse_record_regs_t(uint64_t x0, uint64_t x1, int pad, Key& k, uint32_t& ext) {
    const unsigned __int128 be = ((unsigned __int128)__builtin_bswap64(x0) << 64) | __builtin_bswap64(x1);
    const unsigned __int128 B = (be >> (8 * (16 - PK))) >> (2 * pad);
    k.lo = (uint64_t)B & LO_MASK;
    k.hi = (uint64_t)(B >> 62);
    const unsigned __int128 xx = ((unsigned __int128)x1 << 64) | x0;
    const uint32_t e = (uint32_t)(xx >> (8 * PK)) & 0xFFFFu;
    ext = ext_codes2(e);
}

// ---- build ------------------------------------------------------------------------------------
// The region slice in LDS. W=2 slots are stored as two arrays (word 0 of slot i at w[i], word 1
// at w[sm + i], sm = the block's slice capacity) rather than 16-B pairs: the random 8-B CAS, probe
// reads and atomicOr of the build touch one word of a slot, and with 16-B interleaving those
// words sit only in every other bank pair (a 32-lane group of ds_read_b64 spread over 16 bank pairs
// instead of 32; the interleaved layout measured 3.64 -> 3.75 ms at C3, round 4).
template <int W>
struct Slice {
    unsigned long long* w;
    uint32_t sm;
    static constexpr bool SPLIT = W == 2;
    __device__ __forceinline__ unsigned long long* p0(uint32_t i) const { return w + i; }
    __device__ __forceinline__ unsigned long long* p1(uint32_t i) const { return w + (sm + i); }  // W == 2 only
    __device__ __forceinline__ uint64_t w0(uint32_t i) const { return *p0(i); }
    __device__ __forceinline__ uint64_t w1(uint32_t i) const { return W == 2 ? *p1(i) : 0ull; }
    __device__ __forceinline__ void get(uint32_t i, uint64_t& a, uint64_t& b) const {
        a = *p0(i);
        b = W == 2 ? *p1(i) : 0ull;
    }
    __device__ __forceinline__ void put(uint32_t i, uint64_t a, uint64_t b) const {
        *p0(i) = a;
        if (W == 2) *p1(i) = b;
    }
};

// LDS insert with linear probing inside the slice: the slot (>= 0), LDS_DUP (key present) or
// LDS_OUT (the run left the slice).
static constexpr int LDS_DUP = -1, LDS_OUT = -2;
template <int W>
__device__ __forceinline__ int lds_insert(const KParams& p, const Slice<W>& lt, uint32_t S, uint64_t loc,
                                          uint64_t w0, uint64_t w1, unsigned long long* stats) {
    const uint64_t want0 = slot_keybits(w0, p);
    uint32_t spins = 0;
    while (loc < S) {
        const unsigned long long old = atomicCAS(lt.p0((uint32_t)loc), (unsigned long long)EMPTY, w0);
        if (old == EMPTY) {
            if (W == 2)
                __hip_atomic_store(lt.p1((uint32_t)loc), (unsigned long long)w1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            return (int)loc;
        }
        if (slot_keybits(old, p) == want0) {
            if (W == 1) {
                atomicAdd(&stats[ST_DUP], 1ull);
                return LDS_DUP;
            }
            const unsigned long long o1 =
                __hip_atomic_load(lt.p1((uint32_t)loc), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (o1 == EMPTY) {  // the claiming lane has not stored word1 yet: retry this slot
                if (++spins > (1u << 24)) {
                    atomicAdd(&stats[ST_SPIN], 1ull);
                    return LDS_DUP;
                }
                continue;
            }
            if (o1 == w1) {
                atomicAdd(&stats[ST_DUP], 1ull);
                return LDS_DUP;
            }
        }
        ++loc;
    }
    return LDS_OUT;
}

// The same with block steps: one step reads the word0s of the 4-slot block holding `loc` and takes
// the first slot at or after `loc` that is EMPTY (CAS) or holds the key's high word (duplicate
// test), so a probe run of d slots costs ~d/4 steps. The build's phases run the lanes' keys in
// lockstep, so a wave waits for its longest run: this shortens exactly that tail. Slots are
// taken in the same order (first EMPTY at or after home) as lds_insert.
template <int W>
__device__ __forceinline__ int lds_insert_blk(const KParams& p, const Slice<W>& lt, uint32_t S, uint32_t loc,
                                              uint64_t w0, uint64_t w1, unsigned long long* stats) {
    const uint64_t want0 = slot_keybits(w0, p);
    uint32_t spins = 0;
    while (loc < S) {
        const uint32_t base = loc & ~3u;
        uint64_t v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = lt.w0(base + q);  // past S: inside the LDS allocation, masked
        int hit = -1;
        bool key = false;
#pragma unroll
        for (int q = 3; q >= 0; --q) {
            const uint32_t i = base + q;
            const bool e = v[q] == EMPTY, m = !e && slot_keybits(v[q], p) == want0;
            if (i >= loc && i < S && (e || m)) {
                hit = q;
                key = m;
            }
        }
        if (hit < 0) {
            loc = base + 4;
            continue;
        }
        const uint32_t i = base + (uint32_t)hit;
        if (!key) {
            const unsigned long long old = atomicCAS(lt.p0(i), (unsigned long long)EMPTY, w0);
            if (old == EMPTY) {
                if (W == 2)
                    __hip_atomic_store(lt.p1(i), (unsigned long long)w1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                return (int)i;
            }
            loc = i;  // lost the slot: look at it again (the winner may hold this key)
            continue;
        }
        if (W == 1) {
            atomicAdd(&stats[ST_DUP], 1ull);
            return LDS_DUP;
        }
        const unsigned long long o1 = __hip_atomic_load(lt.p1(i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (o1 == EMPTY) {  // claimed, word1 not stored yet: look again
            if (++spins > (1u << 24)) {
                atomicAdd(&stats[ST_SPIN], 1ull);
                return LDS_DUP;
            }
            loc = i;
            continue;
        }
        if (o1 == w1) {
            atomicAdd(&stats[ST_DUP], 1ull);
            return LDS_DUP;
        }
        loc = i + 1;
    }
    return LDS_OUT;
}

// ---- chains ------------------------------------------------------------------------------------
// After a region's keys are in LDS (lt: S slots): link every k-mer x to its successor y =
// next_kmer(x) when y provably shares x's minimizer (x's minimizer window j* is not the one that
// drops out, and the window y appends orders strictly above it: then y's minimizer value is x's,
// y is in this region) and y is in this slice; y is not linked into when it is a splitter (the
// walker must stop before those). A link is only ever made to the key next_kmer(x) itself, so a
// chain record is exact whatever the regions are. Heads (a successor, no predecessor) of this
// region get a record {tail word0 with the link count in the index field, tail word1} and their
// slot the record index + 1. succ: S 16-bit entries; hcnt: the region's record counter (zeroed).
// While a region's chains are built, a slot's [idx_lo, 58) field holds its successor's slot + 1
// (0 = none) and a spare top bit marks "has a linked predecessor" (w1 bit 63 at W=2: lo < 2^62;
// w0 bit 63 at W=1: j* < 32 there); both are set with LDS atomicOr. After the head records are
// written, a head slot's field holds its record index + 1 (heads have no predecessor) and every
// slot that has a predecessor is cleaned at write-out.
static constexpr uint32_t NO_SUCC = 0xFFFFFFFFu;
template <int W>
__device__ __forceinline__ uint32_t succ_of(uint64_t w0, const KParams& p) {
    return (uint32_t)((w0 >> p.idx_lo) & ((1ull << (58 - p.idx_lo)) - 1)) - 1u;  // NO_SUCC when 0
}
template <int W>
__device__ __forceinline__ unsigned long long* pred_word(const Slice<W>& lt, uint32_t t) {
    return W == 2 ? lt.p1(t) : lt.p0(t);
}
static constexpr unsigned long long PRED = 1ull << 63;
// slot as written to the table: successor field and predecessor bit cleaned unless it is a head
// whose field is its record index
template <int W>
__device__ __forceinline__ void clean_out(uint64_t& w0, uint64_t& w1, const KParams& p) {
    const bool pred = ((W == 2 ? w1 : w0) & PRED) != 0;
    if (pred) w0 = slot_clean(w0, p);
    if (W == 2) w1 &= LO_MASK;
    else w0 &= ~PRED;
}

// Block-step search of a slice for key (want0, lo) from slot t: BLK slots per step (word 0 of each,
// 16-B LDS reads with the split layout), the first slot at or after t that is EMPTY (absent) or
// holds the key's high word (then word 1 decides).
template <int W, int BLK>
__device__ __forceinline__ uint32_t link_probe(const KParams& p, const Slice<W>& lt, uint32_t S, uint32_t t,
                                               uint64_t want0, uint64_t lo) {
    while (t < S) {
        const uint32_t base = t & ~(uint32_t)(BLK - 1);
        uint64_t v[BLK];
        if constexpr (Slice<W>::SPLIT && BLK % 2 == 0) {
#pragma unroll
            for (int q = 0; q < BLK; q += 2) {
                const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(lt.p0(base + q));
                v[q] = x.x;
                v[q + 1] = x.y;
            }
        } else {
#pragma unroll
            for (int q = 0; q < BLK; ++q) v[q] = lt.w0(base + q);
        }
        int hit = -1;
        bool key = false;
#pragma unroll
        for (int q = BLK - 1; q >= 0; --q) {
            const uint32_t i = base + q;
            const bool e = v[q] == EMPTY, m = !e && slot_keybits(v[q], p) == want0;
            if (i >= t && i < S && (e || m)) {
                hit = q;
                key = m;
            }
        }
        if (hit < 0) {
            t = base + BLK;
            continue;
        }
        const uint32_t i = base + (uint32_t)hit;
        if (!key) return NO_SUCC;  // EMPTY: the key is not in this slice
        if (W == 1 || (lt.w1(i) & LO_MASK) == lo) return i;
        t = i + 1;
    }
    return NO_SUCC;
}

// The slot of x's successor in this slice, or NO_SUCC. With mtop (x is a word of this region's
// window carrying the top bits of its minimizer order) the test needs no window extraction and
// y's home is this region's; a tie in the top bits counts as "no link" (never a wrong link).
template <int W, bool MTOP>
__device__ __forceinline__ uint32_t chain_link(const KParams& p, const Slice<W>& lt, uint32_t S,
                                               uint64_t lo, uint64_t cap, uint64_t w0, uint64_t w1, bool dense = false) {
    const uint32_t f = ext_fwd(slot_ext(w0));
    const uint32_t j = slot_jstar(w0) & (W == 1 ? 31u : 63u);
    if (f > 3u || (int)j >= p.K - p.M) return NO_SUCC;
    const Key x = slot_key(w0, w1 & LO_MASK, p);
    const Key y = key_next(x, f, p);
    uint32_t mw = 0;
    if (MTOP) {
        if (order_top(win_order(win_bits(y, 0, p)), p) <= slot_hidx(w0, p)) return NO_SUCC;
    } else {
        mw = win_bits(x, (int)j, p);
        if (win_order(win_bits(y, 0, p)) <= win_order(mw)) return NO_SUCC;
    }
    const uint32_t hy = key_hash32(y);
    if (is_splitter(y, p)) return NO_SUCC;
    // (y holds x's minimizer one window further: j* + 1)
    const uint64_t home = MTOP ? home_in(lo, lo + S, hy) : home_of(place_w(mw, y, p, (int)j + 1), cap, p);
    if (home < lo || home >= lo + S) return NO_SUCC;
    const uint64_t want0 = W == 1 ? y.lo : y.hi;
    // block steps (see lds_insert_blk): ~d/4 steps for a run of d slots
    if (MTOP) {
        // sparse slices (load 0.5: y sits at or right after its home): 2-slot steps, one 16-B
        // LDS read each (C3 build 2.89 -> 2.76 ms, LDS bank conflicts 0.47 -> 0.41 of LDS cycles);
        // dense slices (> 2/3 full, longer runs): 4-slot steps (load 0.85: 4.96 vs 5.11 ms)
        return dense ? link_probe<W, 4>(p, lt, S, (uint32_t)(home - lo), want0, y.lo)
                     : link_probe<W, 2>(p, lt, S, (uint32_t)(home - lo), want0, y.lo);
    }
    for (uint32_t t = (uint32_t)(home - lo); t < S; ++t) {
        uint64_t v0, v1;
        lt.get(t, v0, v1);  // interleaved: both words in one LDS read (a match needs no second trip)
        if (v0 == EMPTY) break;
        if (slot_keybits(v0, p) == want0 && (W == 1 || (v1 & LO_MASK) == y.lo)) return t;
    }
    return NO_SUCC;
}

// record x's link (own slot i: successor field; the successor's predecessor bit)
template <int W>
__device__ __forceinline__ void put_link(const Slice<W>& lt, uint32_t i, uint32_t nx, const KParams& p) {
    if (nx == NO_SUCC) return;
    atomicOr(lt.p0(i), (unsigned long long)(nx + 1) << p.idx_lo);
    atomicOr(pred_word<W>(lt, nx), PRED);
}
template <int W>
__device__ __forceinline__ bool is_head(const Slice<W>& lt, uint32_t i, const KParams& p) {
    uint64_t w0, wp;  // wp: the word holding the predecessor bit
    if (W == 2) {
        lt.get(i, w0, wp);
    } else {
        w0 = wp = lt.w0(i);
    }
    return w0 != EMPTY && succ_of<W>(w0, p) != NO_SUCC && !(wp & PRED);
}

// Head records of the listed heads (hlist[0, min(*hcnt, hcap))): walk each chain to its tail.
template <int W, int TB>
__device__ __forceinline__ void chain_heads(const KParams& p, const Slice<W>& lt, const uint16_t* hlist,
                                            uint32_t r, bool fresh, uint64_t* headrec, uint32_t hcap,
                                            const uint32_t* hcnt) {
    const uint32_t nh = min(*hcnt, hcap);
    // the region's record count (after the records: k_rec_succ resolves only these)
    if (threadIdx.x == 0) reinterpret_cast<uint32_t*>(headrec + (uint64_t)nreg(p) * hcap * 2)[r] = nh;
    for (uint32_t id = threadIdx.x; id < nh; id += TB) {
        const uint32_t i = hlist[id];
        const uint64_t w0 = lt.w0(i);
        bool own = true;
        if (!fresh) {
            // the walker reads a record at the region of the key it looked up: in a slice reloaded
            // from the table only keys of this region may own one (others may have spilled in)
            const Key hk = slot_key(w0, W == 2 ? lt.w1(i) & LO_MASK : 0ull, p);
            own = place(hk, p).r == r;
        }
        if (!own) {
            *lt.p0(i) = slot_clean(w0, p);  // no record: the walker steps this k-mer itself
            continue;
        }
        uint32_t t = succ_of<W>(w0, p), links = 1;
        uint64_t tw0 = lt.w0(t);
        while (succ_of<W>(tw0, p) != NO_SUCC && links < 63u) {
            t = succ_of<W>(tw0, p);
            tw0 = lt.w0(t);
            ++links;
        }
        const uint64_t tw1 = W == 2 ? lt.w1(t) & LO_MASK : 0ull;
        *reinterpret_cast<ulonglong2*>(headrec + ((uint64_t)r * hcap + id) * 2) =
            make_ulonglong2(with_hidx(tw0 & ((1ull << p.idx_lo) - 1), links, p), tw1);  // succ 0
        *lt.p0(i) = with_hidx(slot_clean(w0, p), id + 1, p);
    }
}

// Chains over every slot of the slice (a slice reloaded from the table, or the large-window
// build): links, then heads into the dense list, then the records.
template <int W, int TB>
__device__ __forceinline__ void region_chains(const KParams& p, const Slice<W>& lt, uint16_t* hlist, uint32_t S,
                                              uint64_t lo, uint64_t cap, uint32_t r, bool fresh, uint64_t* headrec,
                                              uint32_t hcap, uint32_t* hcnt) {
    for (uint32_t i = threadIdx.x; i < S; i += TB) {
        const uint64_t w0 = lt.w0(i);
        if (w0 != EMPTY) put_link<W>(lt, i, chain_link<W, false>(p, lt, S, lo, cap, w0, lt.w1(i)), p);
    }
    lds_barrier();
    for (uint32_t i = threadIdx.x; i < S; i += TB) {
        if (is_head<W>(lt, i, p)) {
            const uint32_t id = atomicAdd(hcnt, 1u);
            if (id < hcap) hlist[id] = (uint16_t)i;
            else *lt.p0(i) = slot_clean(lt.w0(i), p);  // no record room: no index
        }
    }
    lds_barrier();
    chain_heads<W, TB>(p, lt, hlist, r, fresh, headrec, hcap, hcnt);
    lds_barrier();
}

// Build from the region windows, one region per block at a time (windows larger than the
// prefetching kernel holds in registers: > 12 words per thread, i.e. > ~760M k-mers per table).
template <int W>
__global__ __launch_bounds__(BUILD_THREADS) void k_part_build(KParams p, const uint64_t* buf2,
                                                              uint64_t* slots, uint64_t cap, int table_empty,
                                                              uint64_t* ovf, uint64_t ovf_cap,
                                                              unsigned long long* ctr,
                                                              unsigned long long* stats,
                                                              uint32_t RC, const uint32_t* rcnt,
                                                              uint64_t* headrec, uint32_t hcap, uint32_t smax,
                                                              const uint64_t* __restrict__ rbt) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lt_[];
    uint16_t* hlist = reinterpret_cast<uint16_t*>(lt_ + (uint64_t)smax * W);
    const Slice<W> lt{lt_, smax};
    __shared__ uint32_t hcnt;
    const uint32_t NR = nreg(p);
    for (uint32_t r = blockIdx.x; r < NR; r += gridDim.x) {
        if (threadIdx.x == 0) hcnt = 0;
        const uint64_t lo = rbt[r], hi = rbt[r + 1];
        const uint32_t S = (uint32_t)(hi - lo);
        if (W == 2) {
            const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(slots + lo * 2);
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) {
                ulonglong2 v = table_empty ? make_ulonglong2(EMPTY, EMPTY) : g2[i];
                if (v.x != EMPTY) v.x = slot_clean(v.x, p);  // earlier chain bits are rebuilt
                lt.put(i, v.x, v.y);
            }
        } else {
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) {
                const unsigned long long v = table_empty ? (unsigned long long)EMPTY : (unsigned long long)slots[lo + i];
                *lt.p0(i) = v == EMPTY ? v : slot_clean(v, p);
            }
        }
        __syncthreads();
        const uint64_t b = (uint64_t)r * RC, e = b + min(rcnt[r], RC);
        for (uint64_t j = b + threadIdx.x; j < e; j += BUILD_THREADS) {
            uint64_t w0, w1 = 0;
            if (W == 2) {
                const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(buf2 + j * 2);
                w0 = v.x;
                w1 = v.y;
            } else {
                w0 = buf2[j];
            }
            // every word of region r's window is a key of region r; the slot keeps key, ext and j*
            const uint64_t home = home_in(lo, hi, key_hash32(slot_key(w0, w1, p)));
            const bool out = lds_insert<W>(p, lt, S, home - lo, slot_clean(w0, p), w1, stats) == LDS_OUT;
            const unsigned long long idx = wave_reserve(&ctr[CT_OVF2], out);
            if (out) {
                if (idx < ovf_cap) {
                    ovf[idx * W] = w0;
                    if (W == 2) ovf[idx * W + 1] = w1;
                } else {
                    atomicAdd(&stats[ST_FULL], 1ull);
                }
            }
        }
        __syncthreads();
        if (hcap) region_chains<W, BUILD_THREADS>(p, lt, hlist, S, lo, cap, r, table_empty != 0, headrec, hcap, &hcnt);
        if (W == 2) {
            ulonglong2* dst = reinterpret_cast<ulonglong2*>(slots + lo * 2);
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) {
                uint64_t x, y;
                lt.get(i, x, y);
                if (hcap && x != EMPTY) clean_out<W>(x, y, p);
                dst[i] = make_ulonglong2(x, y);
            }
        } else {
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) {
                uint64_t v = lt.w0(i), u = 0;
                if (hcap && v != EMPTY) clean_out<W>(v, u, p);
                slots[lo + i] = v;
            }
        }
        __syncthreads();
    }
}

// ---- sorted slice insert (fresh 16-B slices) -----------------------------------------------------
// Linear probing in the slice costs random LDS CAS (bank conflicts) and, at high load, long probe
// runs: ~(1 + 1/(1-a)^2)/2 slots per insert (23 at a = 0.85), and a wave waits for its lanes'
// longest run. Instead the slice is laid out
// as sequential linear probing in home order would leave it: with c(h) keys of home h,
// C(h) = c(0) + .. + c(h) and M(h) = max over h' <= h of (h' - C(h' - 1)), the keys of home h take
// slots C(h - 1) + M(h) + 0, 1, .. (E(h) = C(h) + M(h) is the first free slot after them), so an
// insert is one LDS atomic (its rank among its home's keys) and two block scans over the slots, with
// no probing and no CAS; every key lies at or after its home with no EMPTY slot in between, which is
// all a linear-probing lookup needs. Keys of one home are consecutive, so duplicates are found by
// comparing with the earlier keys of the same home.
// Thread t scans the slots [t*E, t*E + E) of the slice: returns through hist[i] the first slot of
// home i (C(i-1) + M(i)); wsum / wmax: TB / 64 words of LDS scratch.
// The count prefix C and the prefix max M come from ONE block scan over pairs (s, m) = (keys of a
// stretch of homes, max over its homes i of i - (keys before i within the stretch)), combined as
// (s1, m1) . (s2, m2) = (s1 + s2, max(m1, m2 - s1)) (associative): one barrier per region instead
// of a sum scan and a max scan with a barrier each.
template <int TB>
__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t& total, uint32_t* wsum);
template <int TB>
__device__ __forceinline__ void sorted_starts(uint32_t* hist, uint32_t S, uint32_t* wsum, int32_t* wmax) {
    const uint32_t E = (S + TB - 1) / TB;
    const uint32_t i0 = min(threadIdx.x * E, S), i1 = min(i0 + E, S);
    uint32_t s = 0;
    int32_t mr = INT32_MIN / 2;  // (far below any i - C: no slot)
    for (uint32_t i = i0; i < i1; ++i) {
        mr = max(mr, (int32_t)i - (int32_t)s);
        s += hist[i];
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t xs = s;
    int32_t xm = mr;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {  // inclusive wave scan of the pairs
        const uint32_t ys = __shfl_up(xs, o, 64);
        const int32_t ym = __shfl_up(xm, o, 64);
        if (lane >= o) {
            xm = max(ym, xm - (int32_t)ys);
            xs += ys;
        }
    }
    if (lane == 63) {
        wsum[w] = xs;
        wmax[w] = xm;
    }
    lds_barrier();
    uint32_t ps = 0;             // the waves before this one
    int32_t pm = INT32_MIN / 2;
#pragma unroll
    for (int k = 0; k < TB / 64; ++k)
        if (k < w) {
            pm = max(pm, wmax[k] - (int32_t)ps);
            ps += wsum[k];
        }
    const uint32_t es = __shfl_up(xs, 1, 64);  // the lanes before this one in the wave
    const int32_t em = __shfl_up(xm, 1, 64);
    if (lane) {
        pm = max(pm, em - (int32_t)ps);
        ps += es;
    }
    const uint32_t base = ps;      // C(i0 - 1)
    int32_t m = pm;                // max over the homes before i0 of i - C(i - 1)
    uint32_t c = base;
    for (uint32_t i = i0; i < i1; ++i) {
        const uint32_t ci = hist[i];
        m = max(m, (int32_t)i - (int32_t)c);
        hist[i] = c + (uint32_t)m;
        c += ci;
    }
}

// Build from fixed region windows: each thread holds up to IPT words of the region it inserts;
// region hand-offs use LDS-only barriers, so a block's window loads (issued right after the
// previous region's write-out), LDS work and slice stores overlap across blocks.
// Occupancy: three 512-thread blocks per CU (LDS ~50 KB per block with the chain head list, and
// <= 80 VGPRs: 6 waves per SIMD) beat two blocks that hold a second register copy of the next
// region's window during the whole region (C3: 4.34 vs 5.20 ms); the next window reuses the
// registers of this one once its words are consumed.
// FRESH (the table was empty: every slice starts EMPTY) is a compile-time variant: with the
// reload-and-rechain path compiled in, spills on that path made the compiler drain every
// outstanding store (vmcnt(0)) at the top of each region; the fresh kernel has no spills and its
// slice stores drain in the background (C3 build 4.31 -> 3.86 ms).
template <int W, int IPT, int KT, bool FRESH, bool SORT = false>
__global__ __launch_bounds__(BUILD_THREADS) __attribute__((amdgpu_waves_per_eu(6, 8))) void k_part_build_pf(KParams p_in, const uint64_t* __restrict__ buf2,
                                                                 uint64_t* slots, uint64_t cap,
                                                                 uint64_t* ovf, uint64_t ovf_cap,
                                                                 unsigned long long* ctr,
                                                                 unsigned long long* stats, uint32_t RC,
                                                                 const uint32_t* __restrict__ rcnt,
                                                                 uint64_t* headrec, uint32_t hcap, uint32_t smax,
                                                                 const uint64_t* __restrict__ rbt) {
    const KParams p = specialize<KT>(p_in);
    extern __shared__ __attribute__((aligned(16))) unsigned long long lt_[];
    uint16_t* hlist = reinterpret_cast<uint16_t*>(lt_ + (uint64_t)smax * W);
    const Slice<W> lt{lt_, smax};
    __shared__ uint32_t hcnt;
    uint64_t a[IPT], b[IPT];
    // window of region r (m = its fill, read one region ahead as a vector load: a scalar load
    // would be waited for at the next LDS barrier, which waits on lgkmcnt)
    // z: a per-lane zero the compiler cannot fold makes the address per-lane
    uint32_t z = 0;
    asm volatile("" : "+v"(z));
    auto fill = [&](uint32_t r) { return r < nreg(p) ? min(rcnt[r + z], RC) : 0u; };
    auto load = [&](uint32_t r, uint32_t m, uint64_t (&x)[IPT], uint64_t (&y)[IPT]) {
        const uint64_t base = (uint64_t)(r < nreg(p) ? r : 0) * RC;
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint32_t i = threadIdx.x + (uint32_t)j * BUILD_THREADS;
            const uint64_t g = base + (i < m ? i : 0);
            uint64_t v0, v1 = 0;
            if (W == 2) {
                const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(buf2 + g * 2);
                v0 = v.x;
                v1 = v.y;
            } else {
                v0 = buf2[g];
            }
            x[j] = i < m ? v0 : EMPTY;
            y[j] = v1;
        }
    };
    uint32_t r = blockIdx.x;
    uint32_t m_cur = fill(r);
    load(r, m_cur, a, b);
    const uint32_t NR = nreg(p);
    if (SORT)  // the whole LDS slice reset once (see the sorted insert below)
        for (uint32_t i = threadIdx.x; i < smax; i += BUILD_THREADS) {
            *lt.p0(i) = EMPTY;
            *lt.p1(i) = 0ull;
        }
    for (; r < NR; r += gridDim.x) {
        const uint64_t lo = rbt[r], hi = rbt[r + 1];
        const uint32_t S = (uint32_t)(hi - lo);
        const uint32_t m_next = fill(r + gridDim.x);  // in flight during this region
        // block-step probing (lds_insert_blk) where the slice fills above ~2/3 (balanced tables at
        // load 0.85: build 21.3 -> 13.0 ms); slot steps below (C3 at 0.5: 3.71 vs 3.90 ms)
        const bool dense = 3u * m_cur > 2u * S;
        if (threadIdx.x == 0) hcnt = 0;
        int pos[IPT];  // LDS slot of each word inserted here (chains walk from these)
        if constexpr (SORT) {
            static_assert(FRESH && Slice<W>::SPLIT, "the sorted slice needs a fresh table and the split layout");
            // sorted slice (FRESH only): word 0 EMPTY, the word-1 array holds the home counts.
            // Every slot of the LDS slice is already reset (word 0 EMPTY, word 1 zero: zero home
            // counts): before the first region, then by each write-out for the slots it reads;
            // slots past a region's S are never written. The write-out then needs no barrier of
            // its own: this one orders it before the next region's count atomics (a separate
            // reset pass per region measured 2.91-2.92 vs 2.90 ms, round 4).
            uint32_t* hist = reinterpret_cast<uint32_t*>(lt.p1(0));
            lds_barrier();
#pragma unroll
            for (int j = 0; j < IPT; ++j) {  // home | rank among the keys of that home << 16
                pos[j] = LDS_DUP;
                if (a[j] == EMPTY) continue;
                const uint32_t h = (uint32_t)(home_in(lo, hi, key_hash32(slot_key(a[j], b[j], p))) - lo);
                pos[j] = (int)(h | (atomicAdd(&hist[h], 1u) << 16));
            }
            lds_barrier();
            __shared__ uint32_t wsum[BUILD_THREADS / 64];
            __shared__ int32_t wmax[BUILD_THREADS / 64];
            sorted_starts<BUILD_THREADS>(hist, S, wsum, wmax);
            lds_barrier();
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if (pos[j] < 0) continue;
                const uint32_t slot = hist[(uint32_t)pos[j] & 0xFFFFu] + ((uint32_t)pos[j] >> 16);
                if (slot >= S) {  // the run left the slice: global CAS insert after the build
                    const unsigned long long idx = atomicAdd(&ctr[CT_OVF2], 1ull);
                    if (idx < ovf_cap) {
                        ovf[idx * W] = a[j];
                        if (W == 2) ovf[idx * W + 1] = b[j];
                    } else {
                        atomicAdd(&stats[ST_FULL], 1ull);
                    }
                    pos[j] = LDS_OUT;
                } else {
                    pos[j] = (int)(slot | ((uint32_t)pos[j] & 0xFFFF0000u));  // slot | rank << 16
                }
            }
            lds_barrier();  // every lane has read the starts before the word-1 array is written
#pragma unroll
            for (int j = 0; j < IPT; ++j)
                if (pos[j] >= 0) lt.put((uint32_t)pos[j] & 0xFFFFu, slot_clean(a[j], p), b[j]);
            lds_barrier();
            // duplicates: the keys of one home are consecutive, so a key equal to this one is one of
            // the `rank` keys right before it
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if (pos[j] < 0) continue;
                const uint32_t sl = (uint32_t)pos[j] & 0xFFFFu, rk = (uint32_t)pos[j] >> 16;
                pos[j] = (int)sl;
                const uint64_t want0 = slot_keybits(a[j], p);
                for (uint32_t t = sl - rk; t < sl; ++t) {
                    if (slot_keybits(lt.w0(t), p) == want0 && (W == 1 || lt.w1(t) == b[j])) {
                        atomicAdd(&stats[ST_DUP], 1ull);
                        break;
                    }
                }
            }
        } else {
        if (W == 2) {
            const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(slots + lo * 2);
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) {
                ulonglong2 v = FRESH ? make_ulonglong2(EMPTY, EMPTY) : g2[i];
                if (v.x != EMPTY) v.x = slot_clean(v.x, p);  // earlier chain bits are rebuilt
                lt.put(i, v.x, v.y);
            }
        } else {
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) {
                const unsigned long long v = FRESH ? (unsigned long long)EMPTY : (unsigned long long)slots[lo + i];
                *lt.p0(i) = v == EMPTY ? v : slot_clean(v, p);
            }
        }
        if (FRESH)
            lds_barrier();
        else
            __syncthreads();
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            pos[j] = LDS_DUP;
            if (a[j] == EMPTY) continue;
            // every word of region r's window is a key of region r; the slot keeps key, ext and j*
            // (the order bits stay in the register copy for the link test)
            const uint64_t home = home_in(lo, hi, key_hash32(slot_key(a[j], b[j], p)));
            pos[j] = dense ? lds_insert_blk<W>(p, lt, S, (uint32_t)(home - lo), slot_clean(a[j], p), b[j], stats)
                           : lds_insert<W>(p, lt, S, home - lo, slot_clean(a[j], p), b[j], stats);
            if (pos[j] == LDS_OUT) {  // rare after the hot remap: a per-lane atomic (no spills)
                const unsigned long long idx = atomicAdd(&ctr[CT_OVF2], 1ull);
                if (idx < ovf_cap) {
                    ovf[idx * W] = a[j];
                    if (W == 2) ovf[idx * W + 1] = b[j];
                } else {
                    atomicAdd(&stats[ST_FULL], 1ull);
                }
            }
        }
        lds_barrier();
        }  // probing insert
        // The next region's window goes into a/b as soon as this region's words are consumed
        // (after the inserts, or after the links that read them), so its loads are in flight
        // during the remaining phases and never queue behind the write-out's stores.
        if (hcap && !FRESH) {
            load(r + gridDim.x, m_next, a, b);
            region_chains<W, BUILD_THREADS>(p, lt, hlist, S, lo, cap, r, false, headrec, hcap, &hcnt);
        } else if (hcap) {
            // fresh slice: its keys are exactly this thread's words, so links are computed from
            // registers (no pass over empty slots) and every key knows its slot
            // (pos[j] | HAS_SUCC: the key was linked, so a head needs only its predecessor bit read)
            constexpr int HAS_SUCC = 1 << 30;
#pragma unroll
            for (int j = 0; j < IPT; ++j)
                if (pos[j] >= 0) {
                    const uint32_t nx = chain_link<W, true>(p, lt, S, lo, cap, a[j], b[j], dense);
                    put_link<W>(lt, (uint32_t)pos[j], nx, p);
                    if (nx != NO_SUCC) pos[j] |= HAS_SUCC;
                }
            load(r + gridDim.x, m_next, a, b);
            lds_barrier();
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if (pos[j] < 0) continue;
                const uint32_t sl = (uint32_t)pos[j] & 0xFFFFu;
                if (!(pos[j] & HAS_SUCC) || (*pred_word<W>(lt, sl) & PRED)) continue;
                const uint32_t id = atomicAdd(&hcnt, 1u);
                if (id < hcap)
                    hlist[id] = (uint16_t)sl;
                else
                    *lt.p0(sl) = slot_clean(lt.w0(sl), p);  // no record room: no index
            }
            lds_barrier();
            chain_heads<W, BUILD_THREADS>(p, lt, hlist, r, true, headrec, hcap, &hcnt);
            lds_barrier();
        } else {
            load(r + gridDim.x, m_next, a, b);
        }
        if (W == 2) {
            // two slots per step: both LDS reads are in flight before either store
            ulonglong2* dst = reinterpret_cast<ulonglong2*>(slots + lo * 2);
            for (uint32_t i0 = threadIdx.x; i0 < S; i0 += 2 * BUILD_THREADS) {
                // opaque to the optimiser: no per-thread 64-bit store base hoisted out of the region
                // loop (it was spilled, and its reload waited for every load in flight: vmcnt(0))
                uint32_t i = i0;
                asm volatile("" : "+v"(i));
                const uint32_t i2 = i + BUILD_THREADS;
                const bool two = i2 < S;
                uint64_t x, y, x2, y2;
                lt.get(i, x, y);
                lt.get(two ? i2 : i, x2, y2);
                if (SORT) {  // the word-1 array held the home counts: empty slots are all-ones
                    y = x == EMPTY ? EMPTY : y;
                    y2 = x2 == EMPTY ? EMPTY : y2;
                }
                if (hcap && x != EMPTY) clean_out<W>(x, y, p);
                if (hcap && x2 != EMPTY) clean_out<W>(x2, y2, p);
                if (SORT) {  // this thread's slots, read above: reset for the next region
                    *lt.p0(i) = EMPTY;
                    *lt.p1(i) = 0ull;
                    if (two) {
                        *lt.p0(i2) = EMPTY;
                        *lt.p1(i2) = 0ull;
                    }
                }
                dst[i] = make_ulonglong2(x, y);
                if (two) dst[i2] = make_ulonglong2(x2, y2);
            }
        } else {
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) {
                uint64_t v = lt.w0(i), u = 0;
                if (hcap && v != EMPTY) clean_out<W>(v, u, p);
                slots[lo + i] = v;
            }
        }
        if (!SORT) lds_barrier();  // fused: the next region's first barrier orders it
        m_cur = m_next;
    }
}

// Grid of the prefetching build: 16384 blocks (8 regions each at C3). A resident grid (3 blocks
// per CU, ~170 regions each) measured slower, 3.71 -> 4.05 ms, and 2 generations of blocks 3.93:
// region loads vary (sd ~7 %), so dynamic block dispatch balances better than a static split.
// Same box, C3 build: 8192 blocks 3.73-3.79, 16384 3.69, 32768 3.72, 65536 3.75 ms.
// Round 4, final kernel: 8192 / 16384 / 24576 / 32768 blocks 2.79-2.81 ms.
static unsigned pf_grid() { return 16384u; }

template <int W, int IPT, int KT, class... A>
static void pf_launch(bool fresh, bool sorted, size_t lds, hipStream_t s, A... a) {
    if constexpr (W == 2 && Slice<W>::SPLIT) {
        if (fresh && sorted) {
            k_part_build_pf<W, IPT, KT, true, true><<<pf_grid(), BUILD_THREADS, lds, s>>>(a...);
            return;
        }
    }
    if (fresh) {
        k_part_build_pf<W, IPT, KT, true><<<pf_grid(), BUILD_THREADS, lds, s>>>(a...);
    } else {
        k_part_build_pf<W, IPT, KT, false><<<pf_grid(), BUILD_THREADS, lds, s>>>(a...);
    }
}

// Region-window build: the prefetching kernel when a window fits IPT words per thread.
template <int W>
static void launch_build_windows(const KParams& p, const PartBuffers& B, TableView t, bool table_empty,
                                 uint64_t ovf_cap, unsigned long long* ctr, unsigned long long* stats, uint32_t RC,
                                 const uint32_t* rcnt, size_t lds, hipStream_t s) {
    const int te = table_empty ? 1 : 0;
    const uint32_t smax = (uint32_t)region_max_slots(p, t.cap);
    const uint32_t hcap = B.headrec ? B.hcap : 0u;
    // fresh slices: sorted slice insert instead of LDS CAS probing; the word-1 array of the split
    // layout holds the home counts, so 16-B slots only. C3 build at load 0.5: 3.63 -> 2.96 ms; at
    // 0.85 (balanced bounds): 12.5 -> 5.0 ms
    const bool sorted = W == 2 && Slice<W>::SPLIT;
    if (debug_flag("plain_build"))  // tests: the large-window kernel at small sizes
        k_part_build<W><<<8192, BUILD_THREADS, lds, s>>>(p, B.buf2, t.slots, t.cap, te, B.buf1, ovf_cap, ctr,
                                                         stats, RC, rcnt, B.headrec, hcap, smax, B.rbt);
    else if (RC <= 4u * BUILD_THREADS)
        with_kt<W>(p.K, [&](auto kt) { pf_launch<W, 4, decltype(kt)::value>(table_empty, sorted, lds, s, p, B.buf2, t.slots, t.cap, B.buf1, ovf_cap,
                                                               ctr, stats, RC, rcnt, B.headrec, hcap, smax, B.rbt); });
    else if (RC <= 6u * BUILD_THREADS)
        with_kt<W>(p.K, [&](auto kt) { pf_launch<W, 6, decltype(kt)::value>(table_empty, sorted, lds, s, p, B.buf2, t.slots, t.cap, B.buf1, ovf_cap,
                                                               ctr, stats, RC, rcnt, B.headrec, hcap, smax, B.rbt); });
    else if (RC <= 12u * BUILD_THREADS)
        with_kt<W>(p.K, [&](auto kt) { pf_launch<W, 12, decltype(kt)::value>(table_empty, sorted, lds, s, p, B.buf2, t.slots, t.cap, B.buf1, ovf_cap,
                                                                ctr, stats, RC, rcnt, B.headrec, hcap, smax, B.rbt); });
    else
        k_part_build<W><<<8192, BUILD_THREADS, lds, s>>>(p, B.buf2, t.slots, t.cap, te, B.buf1, ovf_cap, ctr,
                                                         stats, RC, rcnt, B.headrec, hcap, smax, B.rbt);
}

template <int W>
__global__ __launch_bounds__(PB) void k_insert_overflow(KParams p, const uint64_t* ovf, uint64_t ovf_cap,
                                                        const unsigned long long* ctr, uint64_t* slots,
                                                        uint64_t cap, unsigned long long* stats) {
    const uint64_t m = min((uint64_t)ctr[CT_OVF2], ovf_cap);
    for (uint64_t i = (uint64_t)blockIdx.x * PB + threadIdx.x; i < m; i += (uint64_t)gridDim.x * PB) {
        const uint64_t w0 = ovf[i * W], w1 = (W == 2) ? ovf[i * W + 1] : 0;
        // overflow words come from the partition passes: their j* gives the placement hash
        insert_one<W>(slot_key(w0, w1, p), slot_clean(w0, p), home_of(word_place(w0, w1, p), cap, p), p, slots, cap,
                      stats);
    }
}

// ---- windowed passes with a template block size --------------------------------------------
// The two LDS-sorted passes hold a 4096-word tile (64 KB + 8 KB of bin ids) per block, so LDS caps
// them at 2 blocks per CU; with TB = 512 threads per block that is 16 waves per CU instead of 8
// (half the items per thread), for the same tile and run lengths.
template <int TB>
__device__ __forceinline__ uint32_t block_scan_u32(uint32_t v, uint32_t& total, uint32_t* wsum) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    lds_barrier();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < TB / 64; ++i) {
        const uint32_t s = wsum[i];
        pre += i < w ? s : 0u;
        tot += s;
    }
    total = tot;
    return pre + x - v;
}

// 16-B load of a streamed input (records, pass-1 / pass-2 windows). Non-temporal loads here
// measured slower (C3 9.79 -> 9.87 ms): the windows' partly written lines stay in L2 either way.
__device__ __forceinline__ ulonglong2 ld_stream16(const void* q) { return *reinterpret_cast<const ulonglong2*>(q); }

template <int W, int TB, int TILE>
__device__ __forceinline__ void load_words_tb(const uint64_t* __restrict__ words, uint64_t base, uint64_t end,
                                              uint64_t last, uint64_t* a, uint64_t* b) {
    constexpr int IPT = TILE / TB;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint64_t i = base + (uint64_t)j * TB + threadIdx.x;
        const uint64_t ii = i < end ? i : last;
        uint64_t x0, x1 = 0;
        if (W == 2) {
            const ulonglong2 v = ld_stream16(words + 2 * ii);
            x0 = v.x;
            x1 = v.y;
        } else {
            x0 = words[ii];
        }
        a[j] = i < end ? x0 : EMPTY;
        b[j] = i < end ? x1 : 0;
    }
}

template <int W, int TB, int TILE>
__device__ __forceinline__ void load_words_win_tb(const uint64_t* __restrict__ buf1, uint32_t bk, uint32_t CAP1,
                                                  const uint32_t* pre, uint64_t base, uint64_t end, uint64_t* a,
                                                  uint64_t* b) {
    constexpr int IPT = TILE / TB;
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        const uint32_t v = (uint32_t)(base + (uint64_t)j * TB + threadIdx.x);
        const bool ok = v < (uint32_t)end;
        uint32_t w = 0, pw = 0;
#pragma unroll
        for (uint32_t q = 1; q < S1; ++q)
            if (v >= pre[q]) {
                w = q;
                pw = pre[q];
            }
        const uint64_t i = ok ? (uint64_t)(bk * S1 + w) * CAP1 + (v - pw) : (uint64_t)bk * S1 * CAP1;
        uint64_t x0, x1 = 0;
        if (W == 2) {
            const ulonglong2 x = ld_stream16(buf1 + 2 * i);
            x0 = x.x;
            x1 = x.y;
        } else {
            x0 = buf1[i];
        }
        a[j] = ok ? x0 : EMPTY;
        b[j] = ok ? x1 : 0;
    }
}

// Counting-sort one tile (items in registers) by bin in LDS, reserve each bin's run in its window
// with one atomicAdd (counter(bin)), prefetch the next tile (next()), write the runs to
// out[window(bin) + reserved + rank] (positions past cap -> overflow list).
// WRANK: ranks by wave_rank_all (few bins: the route's owners) instead of one LDS atomic per item
// LATE: g is published after next() issues the next tile's loads; only where those loads are
// unconditional (the waitcnt for g then leaves them in flight: vmcnt(N)); behind conditional loads
// the compiler waits for vmcnt(0), i.e. for the prefetch itself, so g is published before next().
template <int W, int TB, int NB, int TILE, bool WRANK = false, bool LATE = true, class CtrF, class WinF, class NextF>
__device__ __forceinline__ void sort_reserve_write(uint64_t* a, uint64_t* b, const uint32_t* bin, uint64_t* items,
                                                   uint16_t* sbin, uint32_t* hist, uint32_t* start, uint32_t* gpos,
                                                   uint32_t* wsum, CtrF counter, WinF window, uint32_t cap,
                                                   uint64_t* out, uint64_t* ovf, uint64_t ovf_cap,
                                                   unsigned long long* ctr, unsigned long long* stats, NextF next) {
    constexpr int IPT = TILE / TB;
    static_assert(NB <= TB, "one bin per thread");
    __shared__ uint32_t spill;  // some bin's run passes its window's end (block-uniform after the barrier)
    if (threadIdx.x < NB) hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) spill = 0;
    lds_barrier();
    uint32_t rank[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (WRANK)
            rank[j] = wave_rank_all(hist, bin[j], a[j] != EMPTY);
        else
            rank[j] = (a[j] != EMPTY) ? atomicAdd(&hist[bin[j]], 1u) : 0u;
    }
    lds_barrier();
    const uint32_t hv = threadIdx.x < NB ? hist[threadIdx.x] : 0u;
    // the bin's window reservation goes out first: its round trip (~1-2 us) overlaps the scan, the
    // LDS scatter and the next tile's load issue; g is published for the write-out just before its
    // barrier (lds_barrier waits for LDS only, so the atomic stays in flight across the others)
    uint32_t g = 0;
    if (threadIdx.x < NB && hv) g = atomicAdd(counter(threadIdx.x), hv);
    uint32_t total;
    const uint32_t st = block_scan_u32<TB>(hv, total, wsum);
    if (threadIdx.x < NB) start[threadIdx.x] = st;
    lds_barrier();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (a[j] != EMPTY) {
            const uint32_t pos = start[bin[j]] + rank[j];
            // words 0 and 1 in two arrays: random 8-B stores over every bank pair (interleaved
            // 16-B items measured the same, round 4)
            items[pos] = a[j];
            if (W == 2) items[TILE + pos] = b[j];
            sbin[pos] = (uint16_t)bin[j];
        }
    }
    if (!LATE && threadIdx.x < NB) {
        gpos[threadIdx.x] = g;
        if (hv && g + hv > cap) spill = 1;
    }
    __builtin_amdgcn_sched_barrier(0);
    next();  // the next tile's loads are in flight while this one is written
    if (LATE && threadIdx.x < NB) {
        gpos[threadIdx.x] = g;
        if (hv && g + hv > cap) spill = 1;
    }
    lds_barrier();
#pragma unroll 4
    for (uint32_t x = threadIdx.x; x < total; x += TB) {
        const uint32_t q = sbin[x];
        const uint32_t w = gpos[q] + (x - start[q]);
        if (w < cap) {
            const uint64_t v0 = items[x], v1 = (W == 2) ? items[TILE + x] : 0;
            const uint64_t g = window(q) + w;
            if (W == 2) {
                *reinterpret_cast<ulonglong2*>(out + g * 2) = make_ulonglong2(v0, v1);
            } else {
                out[g] = v0;
            }
        }
    }
    if (spill) {
        // full windows: the spilled tail of each bin's run goes to the overflow list with ONE
        // reservation per tile (a hot bucket spills most of every tile; per-wave reservations on
        // the list's single counter serialised: c5h pass 1 1.4 -> 13.5 ms)
        __shared__ uint32_t keepv[NB];
        __shared__ unsigned long long sbase;
        uint32_t sp = 0;
        if (threadIdx.x < NB) {
            const uint32_t g = gpos[threadIdx.x];
            const uint32_t keep = g >= cap ? 0u : min(hv, cap - g);
            keepv[threadIdx.x] = keep;
            sp = hv - keep;
        }
        uint32_t stot;
        const uint32_t so = block_scan_u32<TB>(sp, stot, wsum);
        if (threadIdx.x < NB) hist[threadIdx.x] = so;  // hist is free after the bin scan
        if (threadIdx.x == 0) sbase = atomicAdd(&ctr[CT_OVF], (unsigned long long)stot);
        lds_barrier();
        for (uint32_t x = threadIdx.x; x < total; x += TB) {
            const uint32_t q = sbin[x];
            const uint32_t rr = x - start[q];
            if (rr >= keepv[q]) {
                const uint64_t d = sbase + hist[q] + (rr - keepv[q]);
                if (d < ovf_cap) {
                    ovf[d * W] = items[x];
                    if (W == 2) ovf[d * W + 1] = items[TILE + x];
                } else {
                    atomicAdd(&stats[ST_FULL], 1ull);
                }
            }
        }
    }
    lds_barrier();
}

// pass 1 on words: bucket = top 9 hash bits, S1 windows per bucket (window blockIdx % S1)
template <int W, int TB, bool COLLECT, int TILE, int KT>
__global__ __launch_bounds__(TB) void k_win1(KParams p_in, const uint64_t* __restrict__ words, uint64_t n,
                                             uint32_t CAP1, uint32_t* wcnt, uint64_t* buf1, uint64_t* ovf,
                                             uint64_t ovf_cap, unsigned long long* ctr,
                                             unsigned long long* stats, uint64_t* splits, uint64_t splits_cap,
                                             int jstar_in) {
    const KParams p = specialize<KT>(p_in);
    const bool hot_on = p.hot && ctr[CT_HOT];  // uniform: some region is remapped
    constexpr int IPT = TILE / TB;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + TILE * 2);
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + TILE);
    uint32_t* start = hist + NBX;
    uint32_t* gpos = start + NBX;
    // block-scan partials in static LDS: 80 KB + a few bytes keeps these kernels at one block
    // (8 waves) per CU, measured faster than two (C3: pass 1 1.79-1.89 vs 1.98 ms, pass 2
    // 1.61-1.67 vs 1.69); the splitter buffer (COLLECT) uses the dynamic region's unused tail
    __shared__ uint32_t wsum[TB / 64];
    uint32_t* scount = gpos + NBX;
    uint64_t* sbuf = reinterpret_cast<uint64_t*>(scount + 2);
    const uint32_t sub = blockIdx.x % S1;
    const uint64_t b0 = (uint64_t)blockIdx.x * T1 * TILE;
    uint64_t a[IPT], b[IPT];
    if (COLLECT && threadIdx.x == 0) *scount = 0;
    load_words_tb<W, TB, TILE>(words, b0, min(b0 + TILE, n), b0 < n ? b0 : 0, a, b);
    if (COLLECT) lds_barrier();  // the splitter counter is zero before any wave counts
    for (int tt = 0; tt < T1; ++tt) {
        const uint64_t base = b0 + (uint64_t)tt * TILE;
        if (base >= n) break;  // uniform
        uint32_t bin[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            // minimizer -> region (bucket = its top B1 bits); the word carries j* onward
            const Key kk = slot_key(a[j], b[j], p);
            // words of k_part1_convert carry j*; routed words do not
            const uint32_t mn = jstar_in ? slot_jstar(a[j]) : mini_scan(kk, p);
            bin[j] = part_region(mini_window(kk, mn, p), kk, p, hot_on, (int)(mn & 63u)) >> (p.rbits - B1);
            const bool live = a[j] != EMPTY;
            // splitter k-mers this shard owns (they head migrating-walk segments, kh_mseg.hip)
            if (COLLECT && live && ext_bwd(slot_ext(a[j])) != EXT_F && is_splitter(kk, p)) {
                const uint32_t pos = atomicAdd(scount, 1u);
                if (pos < WIN_SPLIT_LCAP) {
                    sbuf[pos * W] = a[j];
                    if (W == 2) sbuf[pos * W + 1] = b[j];
                } else {
                    const unsigned long long o = atomicAdd(&ctr[CT_N_SPLIT], 1ull);
                    if (o < splits_cap) {
                        splits[o * W] = a[j];
                        if (W == 2) splits[o * W + 1] = b[j];
                    }
                }
            }
            if (live && !jstar_in) a[j] = part_word0(slot_clean(a[j], p), mn, p);
        }
        const uint64_t nbase = base + TILE;
        sort_reserve_write<W, TB, NB1, TILE>(
            a, b, bin, items, sbin, hist, start, gpos, wsum,
            [&](uint32_t q) { return &wcnt[q * S1 + sub]; },
            [&](uint32_t q) { return (uint64_t)(q * S1 + sub) * CAP1; }, CAP1, buf1, ovf, ovf_cap, ctr, stats,
            [&]() { load_words_tb<W, TB, TILE>(words, nbase, (tt + 1 < T1) ? min(nbase + TILE, n) : nbase, base, a, b); });
    }
    if (COLLECT) {  // this block's splitters: one list reservation
        __syncthreads();
        const uint32_t k = min(*scount, WIN_SPLIT_LCAP);
        unsigned long long* sbase = reinterpret_cast<unsigned long long*>(sbuf + WIN_SPLIT_LCAP * W);
        if (threadIdx.x == 0) *sbase = k ? atomicAdd(&ctr[CT_N_SPLIT], (unsigned long long)k) : 0ull;
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < k; x += TB) {
            const uint64_t o = *sbase + x;
            if (o < splits_cap) {
                splits[o * W] = sbuf[x * W];
                if (W == 2) splits[o * W + 1] = sbuf[x * W + 1];
            }
        }
    }
}

// pass 1 on records (k with a compile-time packed size PK): the windowed pass 1
// reading the reference records itself — one unaligned 16-B load per record (a record is PK + 2
// <= 16 bytes), parsed in registers after the tile's loads land, with the start / splitter bits
// of the record pass — instead of a record -> word copy and a second pass over the copy.
template <int PK>
__device__ __forceinline__ void load_record16(const uint8_t* __restrict__ recs, uint64_t i, uint64_t n,
                                              uint64_t& x0, uint64_t& x1) {
    if (i + 1 < n) {  // the 16 bytes stay inside the next record
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        u64x2 v;
        __builtin_memcpy(&v, recs + i * (uint64_t)(PK + 2), 16);
        x0 = v.x;
        x1 = v.y;
    } else {
        load_record_regs(recs, i, (uint32_t)(PK + 2), x0, x1);
    }
}

// ROUTE: the sharded path's one-pass route instead (kh_route_starts_win_dev): bins are the owner
// ranks (P <= MAX_RANKS), owner q's run of each tile goes to its window buf1 + q * CAP1 words
// (CAP1 = the caller's window size, >= the records routed), wcnt[q] counts them.
template <int W, int TB, int TILE, int PK, int KT, bool ROUTE = false>
__global__ __launch_bounds__(TB) void k_win1_rec(KParams p_in, const uint8_t* __restrict__ recs, uint64_t n,
                                                 uint32_t CAP1, uint32_t* wcnt, uint64_t* buf1,
                                                 uint64_t* start_mask, uint64_t* split_mask, uint64_t* ovf,
                                                 uint64_t ovf_cap, unsigned long long* ctr,
                                                 unsigned long long* stats, uint32_t P = 1,
                                                 unsigned long long* spl = nullptr) {
    const KParams p = specialize<KT>(p_in);
    constexpr int NB = ROUTE ? MAX_RANKS : NB1;
    // ROUTE: splitter k-mers routed to each owner (its migrating walk seeds a walker at each; the
    // owner's host learns their number with the route counts instead of reading its list)
    __shared__ uint32_t rspl[ROUTE ? MAX_RANKS : 1];
    if (ROUTE && spl) {
        if (threadIdx.x < MAX_RANKS) rspl[threadIdx.x] = 0;
        __syncthreads();
    }
    constexpr int IPT = TILE / TB;
    const bool hot_on = !ROUTE && p.hot && ctr[CT_HOT];
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + TILE * 2);
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + TILE);
    uint32_t* start = hist + NB;
    uint32_t* gpos = start + NB;
    __shared__ uint32_t wsum[TB / 64];
    const uint32_t sub = ROUTE ? 0u : blockIdx.x % S1;
    // persistent blocks: tile t, t + gridDim.x, ...; the next tile's loads are always in flight
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    // a wave's 64 records are one contiguous run of 64 * R bytes: lane l loads the run's l-th
    // aligned 16-B block (coalesced, no straddling), and each lane later gathers the two blocks
    // holding its record by cross-lane shuffles
    const uint32_t R = PK ? (uint32_t)(PK + 2) : (uint32_t)p.R;  // PK = 0: any record of <= 15 bytes
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nbytes = n * (uint64_t)R;
    uint64_t a[IPT], b[IPT];  // raw 16-B blocks until parsed, then the words
    // ROUTE: loads only where a block is needed. Otherwise every lane loads
    // (its address clamped into the records): blocks 62 and 63 and those of a wave past the batch
    // are never read (a record's two blocks are <= 61; past the batch no record is valid), and
    // unconditional loads let the compiler count them, so the sort's reservation wait leaves the
    // next tile's loads in flight (vmcnt(N) instead of vmcnt(0))
    constexpr bool UNCOND = !ROUTE;
    // the block holding the last record byte: the conditional path loads it whole as well (the
    // records buffer is read 16 B at a time up to that block's end)
    const uint64_t glast = nbytes ? (nbytes - 1) & ~15ull : 0;
    auto load = [&](uint64_t base, uint64_t end) {
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t r0 = base + (uint64_t)j * TB + (threadIdx.x & ~63u);  // the wave's first record
            const uint64_t g = ((r0 * R) & ~15ull) + 16ull * lane;
            if (UNCOND) {
                const ulonglong2 v = ld_stream16(recs + (g < glast ? g : glast));
                a[j] = v.x;
                b[j] = v.y;
                continue;
            }
            a[j] = b[j] = 0;
            if (r0 < end && lane < 62 && g < nbytes) {
                const ulonglong2 v = ld_stream16(recs + g);
                a[j] = v.x;
                b[j] = v.y;
            }
        }
    };
    uint64_t t = blockIdx.x;
    if (t < ntiles) load(t * TILE, min(t * TILE + TILE, n));
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * TILE;
        uint32_t bin[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t s0 = base + (uint64_t)j * TB;
            const bool valid = s0 + threadIdx.x < n;
            Key k{0, 0};
            uint32_t ext = 0;
            {
                const uint64_t r0 = s0 + (threadIdx.x & ~63u);
                const uint32_t off = (uint32_t)((r0 * R) & 15u) + lane * R;  // from the first block
                const int blk = (int)(off >> 4);
                const uint32_t o = off & 15u;
                const uint64_t p0 = __shfl(a[j], blk, 64), p1 = __shfl(b[j], blk, 64);
                const uint64_t q0 = __shfl(a[j], blk + 1, 64), q1 = __shfl(b[j], blk + 1, 64);
                uint64_t w0 = p0, w1 = p1, w2 = q0;
                if (o >= 8u) {
                    w0 = p1;
                    w1 = q0;
                    w2 = q1;
                }
                const uint32_t sh = (o & 7u) * 8u;
                if (valid) {
                    if constexpr (PK != 0)
                        parse_record_regs_t<PK>(funnel64(w0, w1, sh), funnel64(w1, w2, sh), p.pad, k, ext);
                    else
                        parse_record_regs(funnel64(w0, w1, sh), funnel64(w1, w2, sh), p, k, ext);
                }
            }
            const uint32_t mn = mini_scan(k, p);
            if (s0 < n) {  // uniform: one start / splitter word per 64 consecutive records
                const bool is_start = valid && ext_bwd(ext) == EXT_F;
                const uint64_t bal = __ballot(is_start);
                const uint64_t sb = split_mask ? __ballot(valid && !is_start && is_splitter(k, p)) : 0;
                const uint64_t wb = s0 + (threadIdx.x & ~63u);
                if ((threadIdx.x & 63) == 0 && wb < n) {
                    if (start_mask) start_mask[wb >> 6] = bal;
                    if (split_mask) split_mask[wb >> 6] = sb;
                }
            }
            a[j] = valid ? part_word0(slot_w0(k, ext, p), mn, p) : EMPTY;
            b[j] = (valid && W == 2) ? k.lo : 0;
            if (ROUTE) {
                bin[j] = P == 1 ? 0u
                                : (p.owner_mode == 1 ? owner_key(k, p, P) : owner_of_mini(mini_window(k, mn, p), P));
                if (spl && valid && ext_bwd(ext) != EXT_F && is_splitter(k, p))
                    atomicAdd(&rspl[bin[j]], 1u);
            } else
                bin[j] = part_region(mini_window(k, mn, p), k, p, hot_on, (int)(mn & 63u)) >> (p.rbits - B1);
        }
        const uint64_t nt = t + gridDim.x, nbase = nt * TILE;
        if constexpr (ROUTE) {
            // owner runs need no LDS staging: ranks per (tile, owner) by wave-aggregated LDS
            // atomics, one reservation per (tile, owner), then every lane stores its word at its
            // run position (a tile's run of an owner is contiguous: L2 merges the 16-B stores)
            __shared__ uint32_t rh[MAX_RANKS], rg[MAX_RANKS];
            if (threadIdx.x < MAX_RANKS) rh[threadIdx.x] = 0;
            lds_barrier();
            uint32_t rank[IPT];
#pragma unroll
            for (int j = 0; j < IPT; ++j) rank[j] = wave_rank_all(rh, bin[j], a[j] != EMPTY);
            lds_barrier();
            if (threadIdx.x < P) {
                const uint32_t h = rh[threadIdx.x];
                rg[threadIdx.x] = h ? atomicAdd(&wcnt[threadIdx.x], h) : 0u;
            }
            lds_barrier();
#pragma unroll
            for (int j = 0; j < IPT; ++j) {
                if (a[j] == EMPTY) continue;
                const uint64_t d = (uint64_t)bin[j] * CAP1 + rg[bin[j]] + rank[j];
                if (W == 2)
                    *reinterpret_cast<ulonglong2*>(buf1 + d * 2) = make_ulonglong2(a[j], b[j]);
                else
                    buf1[d] = a[j];
            }
            load(nbase, nt < ntiles ? min(nbase + TILE, n) : nbase);
            lds_barrier();  // every lane has read rg before the next tile's counts
        } else {
            sort_reserve_write<W, TB, NB, TILE, false, UNCOND>(
                a, b, bin, items, sbin, hist, start, gpos, wsum, [&](uint32_t q) { return &wcnt[q * S1 + sub]; },
                [&](uint32_t q) { return (uint64_t)(q * S1 + sub) * CAP1; }, CAP1, buf1, ovf, ovf_cap, ctr, stats,
                [&]() { load(nbase, nt < ntiles ? min(nbase + TILE, n) : nbase); });
        }
    }
    if (ROUTE && spl) {
        __syncthreads();
        if (threadIdx.x < P && rspl[threadIdx.x]) atomicAdd(&spl[threadIdx.x], (unsigned long long)rspl[threadIdx.x]);
    }
}

// pass 2: next 8 hash bits within bucket bk, into the region windows (RC words each)
template <int W, int TB, int TILE, int KT>
__global__ __launch_bounds__(TB) void k_win2(KParams p_in, const uint64_t* __restrict__ buf1, uint64_t G,
                                             uint32_t RC, uint32_t* rcnt,
                                             uint64_t* buf2, uint64_t* ovf, uint64_t ovf_cap,
                                             unsigned long long* ctr, unsigned long long* stats, uint32_t CAP1,
                                             const uint32_t* wcnt) {
    const KParams p = specialize<KT>(p_in);
    const bool hot_on = p.hot && ctr[CT_HOT];
    constexpr int IPT = TILE / TB;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + TILE * 2);
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + TILE);
    uint32_t* start = hist + NBX;
    uint32_t* gpos = start + NBX;
    __shared__ uint32_t wsum[TB / 64];  // static: one block per CU (see k_win1)
    const uint32_t bk = blockIdx.x / (uint32_t)G, g = blockIdx.x % (uint32_t)G;
    const uint32_t b2 = (uint32_t)(p.rbits - B1);  // pass-2 bits: regions per bucket = 2^b2
    // the bucket's S1 pass-1 windows read as one virtual range [0, e)
    uint32_t pre[S1 + 1];
    pre[0] = 0;
#pragma unroll
    for (uint32_t j = 0; j < S1; ++j) pre[j + 1] = pre[j] + min(wcnt[bk * S1 + j], CAP1);
    const uint64_t e = pre[S1];
    uint64_t a[IPT], b[IPT];
    auto load = [&](uint64_t t) {
        load_words_win_tb<W, TB, TILE>(buf1, bk, CAP1, pre, t, t < e ? min(t + TILE, e) : t, a, b);
    };
    load((uint64_t)g * TILE);
    for (uint64_t t = (uint64_t)g * TILE; t < e; t += G * TILE) {
        uint32_t bin[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j)
        {
            const Key kk = slot_key(a[j], b[j], p);
            const int js = p.chain ? (int)slot_jstar(a[j]) : (int)(mini_scan(kk, p) & 63u);
            bin[j] = part_region(win_bits(kk, js, p), kk, p, hot_on, js) & ((1u << b2) - 1u);
        }
        sort_reserve_write<W, TB, NB2, TILE>(
            a, b, bin, items, sbin, hist, start, gpos, wsum,
            [&](uint32_t q) { return &rcnt[(bk << b2) | q]; },
            [&](uint32_t q) { return (uint64_t)((bk << b2) | q) * RC; }, RC, buf2, ovf, ovf_cap, ctr, stats,
            [&]() { load(t + G * TILE); });
    }
}

template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
    return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

static constexpr size_t WIN_LDS = sort_lds(WIN_TILE);
// words passes (k_win1 on words, k_win2): 1024 threads (8 words each) instead of 512 (16 each):
// one 152-KiB block per CU, so the thread count is the CU's whole occupancy (C5H insert 7.39 ->
// 7.24 ms, routed one-rank step 11.04 -> 10.85, C3 unchanged; profiles/r05/ab/ab_win_passes_1024.txt)
static constexpr int WIN_TB = 1024;

// pass 1 on words (routed words, or records converted by k_part1_convert); wsplits: collect the
// splitter k-mers of the words (sharded path)
template <int W>
static hipError_t win1_launch(const KParams& p, const uint64_t* words, uint64_t n, uint32_t CAP1, uint32_t* wcnt,
                              const PartBuffers& B, uint64_t ovf_cap, unsigned long long* ctr,
                              unsigned long long* stats, hipStream_t s, uint64_t* wsplits, uint64_t wsplits_cap,
                              bool jstar_in = false) {
    const unsigned nb = (unsigned)win_blocks1(n);
    const int ji = (jstar_in && p.chain) ? 1 : 0;
    return with_kt<W>(p.K, [&](auto kt) {
        constexpr int KT = decltype(kt)::value;
        hipError_t e;
        constexpr int TB = WIN_TB;
        if (wsplits) {
            if ((e = allow_lds(k_win1<W, TB, true, WIN_TILE, KT>, WIN_LDS)) != hipSuccess) return e;
            k_win1<W, TB, true, WIN_TILE, KT><<<nb, TB, WIN_LDS, s>>>(p, words, n, CAP1, wcnt, B.buf1, B.overflow,
                                                                      ovf_cap, ctr, stats, wsplits, wsplits_cap, ji);
        } else {
            if ((e = allow_lds(k_win1<W, TB, false, WIN_TILE, KT>, WIN_LDS)) != hipSuccess) return e;
            k_win1<W, TB, false, WIN_TILE, KT><<<nb, TB, WIN_LDS, s>>>(p, words, n, CAP1, wcnt, B.buf1, B.overflow,
                                                                       ovf_cap, ctr, stats, nullptr, 0, ji);
        }
        return hipSuccess;
    });
}


// pass 1 on the reference records (k with 13 or 5 packed bytes): persistent blocks, one per CU
// (one 152-KiB block fits a CU), a multiple of S1
template <int W>
static hipError_t win1_rec_launch(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t CAP1,
                                  uint32_t* wcnt, const PartBuffers& B, uint64_t* start_mask, uint64_t* split_mask,
                                  uint64_t ovf_cap, unsigned long long* ctr, unsigned long long* stats,
                                  hipStream_t s) {
    constexpr int PK = W == 2 ? 13 : 5;
    // tiles of REC_TILE records: two blocks per CU (4 waves per SIMD) for the VALU-heavy parse and
    // minimizer scan (C3: 2.49 ms at 8192-record tiles and one block per CU, 2.30 at 3584; the
    // words pass 2 keeps 8192: 1.60 vs 1.87 ms at 3584).
    auto go = [&](auto tile_c) -> hipError_t {
        constexpr int TILE = decltype(tile_c)::value;
        constexpr size_t lds = sort_lds(TILE);
        const uint64_t bpc = LDS_BYTES / (lds + 64);  // resident blocks per CU
        uint64_t grid = ((uint64_t)cu_count() * bpc + S1 - 1) / S1 * S1;
        const uint64_t ntiles = (n + TILE - 1) / TILE;
        if (grid > ntiles) grid = (ntiles + S1 - 1) / S1 * S1;
        if (grid == 0) grid = S1;
        return with_kt<W>(p.K, [&](auto kt) {
            constexpr int KT = decltype(kt)::value;
            hipError_t e;
            if ((e = allow_lds(k_win1_rec<W, REC_TB, TILE, PK, KT>, lds)) != hipSuccess) return e;
            k_win1_rec<W, REC_TB, TILE, PK, KT><<<(unsigned)grid, REC_TB, lds, s>>>(
                p, recs, n, CAP1, wcnt, B.buf1, start_mask, split_mask, B.overflow, ovf_cap, ctr, stats);
            return hipSuccess;
        });
    };
    return go(std::integral_constant<int, REC_TILE_P1>{});
}

// One-pass route (sharded insert): records -> owner windows, start bits in the same pass.
template <int U = 0>
__global__ void k_route_win_counts(const uint32_t* cnt, uint32_t P, uint64_t n, uint64_t* counts) {
    const uint32_t q = threadIdx.x;
    if (q < P) counts[q] = cnt[q];
    if (q == 0) counts[P] = n;
}

template <int W, int PK>
static hipError_t route_win_launch(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t P, uint64_t* words,
                                   uint64_t win, uint32_t* cnt, uint64_t* counts, uint64_t* start_mask,
                                   unsigned long long* ctr, unsigned long long* stats, hipStream_t s,
                                   unsigned long long* spl) {
    constexpr size_t lds = 0;  // the route stages nothing in LDS (k_win1_rec ROUTE)
    hipError_t e;
    if ((e = hipMemsetAsync(cnt, 0, (size_t)MAX_RANKS * 4, s)) != hipSuccess) return e;
    if (n) {
        uint64_t grid = (uint64_t)cu_count() * 4;  // resident blocks loop over the tiles
        const uint64_t ntiles = (n + REC_TILE - 1) / REC_TILE;
        if (grid > ntiles) grid = ntiles;
        e = with_kt<W>(p.K, [&](auto kt) {
            constexpr int KT = decltype(kt)::value;
            hipError_t x;
            if ((x = allow_lds(k_win1_rec<W, 512, REC_TILE, PK, KT, true>, lds)) != hipSuccess) return x;
            k_win1_rec<W, 512, REC_TILE, PK, KT, true><<<(unsigned)grid, 512, lds, s>>>(
                p, recs, n, (uint32_t)win, cnt, words, start_mask, nullptr, nullptr, 0, ctr, stats, P,
                p.split_bits ? spl : nullptr);
            return hipGetLastError();
        });
        if (e != hipSuccess) return e;
    }
    k_route_win_counts<<<1, MAX_RANKS, 0, s>>>(cnt, P, n, counts);
    return hipGetLastError();
}

hipError_t launch_route_win(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t P, uint64_t* words,
                            uint64_t win, uint32_t* cnt, uint64_t* counts, uint64_t* start_mask,
                            unsigned long long* ctr, unsigned long long* stats, hipStream_t s,
                            unsigned long long* spl) {
    if (win < n || win >= (1ull << 32) || p.R > 15) return hipErrorInvalidValue;  // 64 records in 62 blocks
    if (p.W == 1)
        return p.P == 5 ? route_win_launch<1, 5>(p, recs, n, P, words, win, cnt, counts, start_mask, ctr, stats, s, spl)
                        : route_win_launch<1, 0>(p, recs, n, P, words, win, cnt, counts, start_mask, ctr, stats, s, spl);
    return p.P == 13 ? route_win_launch<2, 13>(p, recs, n, P, words, win, cnt, counts, start_mask, ctr, stats, s, spl)
                     : route_win_launch<2, 0>(p, recs, n, P, words, win, cnt, counts, start_mask, ctr, stats, s, spl);
}

// pass 2: bucket -> region windows (RC words each)
template <int W>
static hipError_t win2_launch(const KParams& p, const PartBuffers& B, uint64_t n, uint32_t RC, uint32_t* rcnt,
                              uint64_t ovf_cap, unsigned long long* ctr, unsigned long long* stats, uint32_t CAP1,
                              const uint32_t* wcnt, hipStream_t s) {
    const uint64_t G = win_G(n);
    return with_kt<W>(p.K, [&](auto kt) {
        constexpr int KT = decltype(kt)::value;
        hipError_t e;
        if ((e = allow_lds(k_win2<W, WIN_TB, WIN_TILE, KT>, WIN_LDS)) != hipSuccess) return e;
        k_win2<W, WIN_TB, WIN_TILE, KT><<<(unsigned)(NB1 * G), WIN_TB, WIN_LDS, s>>>(p, B.buf1, G, RC, rcnt, B.buf2,
                                                                              B.overflow, ovf_cap, ctr, stats, CAP1,
                                                                              wcnt);
        return hipSuccess;
    });
}

// ---- balanced region bounds (tables above load ~0.6) ---------------------------------------------
// A region's key count is a sum of minimizer runs (sd ~14 % of the mean at C3 sizes), so equal
// slices at load 0.85 overflow one region in ten: the overflow probes linearly across full slices
// (C3 at 0.85: 193 ms/step). Balanced bounds give region r a slice proportional to its count
// (plus a 1/8-mean prior, so no slice is empty): every region builds at the table's load. The
// bounds come from the first build after a clear and stay until the next clear; lookups read
// them from rb (two adjacent words per region). When a slice would exceed the LDS slice
// (region_max_slots), equal ranges are written instead.
// A region whose proportional slice would pass the LDS slice (a clump of remapped runs at load
// 0.85) gets its count clamped so that its slice fits (a few fixed-point rounds: clamping frees
// capacity, which grows the others' slices); the keys past its slice take the global CAS insert.
// Only if the clamped bounds still do not fit are equal ranges written (round 4 fell back to equal
// ranges whenever one region did not fit: at load 0.85 that overflowed a tenth of the regions).
template <int Unused = 0>
__global__ __launch_bounds__(1024) void k_bounds(KParams p, uint64_t cap, const uint32_t* counts, uint32_t RC,
                                                 uint64_t smax, uint64_t* rb) {
    __shared__ unsigned long long wsum[16];
    __shared__ unsigned long long wmax[16];
    __shared__ int bad;
    const uint32_t NR = nreg(p);
    const uint32_t per = (NR + 1023) / 1024;
    const uint32_t r0 = threadIdx.x * per;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t cmax = ~0ull;  // clamp of the region counts
    auto cnt = [&](uint32_t r) -> uint64_t {
        const uint64_t c = counts ? min(counts[r], RC) : 0u;
        return c < cmax ? c : cmax;
    };
    // block sum (and max) of this thread's clamped counts
    auto reduce = [&](uint64_t v, uint64_t m, uint64_t& tot, uint64_t& mx) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            v += __shfl_xor(v, o, 64);
            const uint64_t y = __shfl_xor(m, o, 64);
            m = y > m ? y : m;
        }
        __syncthreads();
        if (lane == 0) {
            wsum[w] = v;
            wmax[w] = m;
        }
        __syncthreads();
        tot = 0;
        mx = 0;
        for (uint32_t i = 0; i < 16; ++i) {
            tot += wsum[i];
            mx = wmax[i] > mx ? wmax[i] : mx;
        }
    };
    uint64_t N0 = 0, mx = 0;
    {
        uint64_t v = 0, m = 0;
        for (uint32_t r = r0; r < r0 + per && r < NR; ++r) {
            v += cnt(r);
            m = cnt(r) > m ? cnt(r) : m;
        }
        reduce(v, m, N0, mx);
    }
    const double beta = (double)N0 / NR / 8.0 + 1.0;  // prior: no region gets an empty slice
    uint64_t N = N0;
    for (int it = 0; it < 6; ++it) {
        const double sc = (double)cap / ((double)N + beta * NR);
        const double lim = 0.97 * (double)smax / sc - beta;
        if ((double)mx <= lim) break;  // every slice fits
        cmax = lim < 1.0 ? 1ull : (uint64_t)lim;
        uint64_t v = 0, m = 0;
        for (uint32_t r = r0; r < r0 + per && r < NR; ++r) {
            v += cnt(r);
            m = cnt(r) > m ? cnt(r) : m;
        }
        reduce(v, m, N, mx);
    }
    uint64_t loc = 0;
    for (uint32_t r = r0; r < r0 + per && r < NR; ++r) loc += cnt(r);
    // exclusive scan of loc over the block (16 waves)
    uint64_t x = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(x, o, 64);
        if ((int)lane >= o) x += y;
    }
    __syncthreads();
    if (threadIdx.x == 0) bad = 0;
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint64_t pre = 0;
    for (uint32_t i = 0; i < 16; ++i) pre += i < w ? wsum[i] : 0ull;
    pre += x - loc;
    const double scale = (double)cap / ((double)N + beta * NR);
    auto bound = [&](uint32_t r, uint64_t P) -> uint64_t {
        const uint64_t b = (uint64_t)(((double)P + beta * r) * scale);
        return r == 0 ? 0ull : (r >= NR || b > cap ? cap : b);
    };
    uint64_t P = pre, prev = bound(r0, pre);
    for (uint32_t r = r0; r < r0 + per && r < NR; ++r) {
        P += cnt(r);
        const uint64_t nx = bound(r + 1, P);
        if (nx - prev > smax) bad = 1;
        prev = nx;
    }
    __syncthreads();
    const bool eq = bad || !counts || N == 0;
    P = pre;
    for (uint32_t r = r0; r < r0 + per && r < NR; ++r) {
        rb[r] = eq ? (r ? mulhi64((uint64_t)r << (64 - p.rbits), cap) : 0ull) : bound(r, P);
        P += cnt(r);
    }
    if (threadIdx.x == 0) rb[NR] = cap;
}

void launch_bounds(const KParams& p, uint64_t cap, const uint32_t* counts, uint32_t RC, uint64_t* rb, hipStream_t s) {
    k_bounds<<<1, 1024, 0, s>>>(p, cap, counts, RC, region_max_slots(p, cap), rb);
}

// Hot threshold with balanced bounds: the count whose proportional slice fills the LDS slice
// (3 % margin for the prior and rounding); 0 = equal ranges (the slice's own size).
static uint32_t balanced_T(const KParams& p, uint64_t cap, uint64_t n) {
    if (!p.rb || !cap) return 0u;
    const double t = 0.97 * (double)region_max_slots(p, cap) * (double)n / (double)cap;
    return t < 1.0 ? 1u : (t > 4.0e9 ? 0xFFFFFFFFu : (uint32_t)t);
}

// ---- hot regions ---------------------------------------------------------------------------------
// A minimizer window shared by far more k-mers than a region holds (a repeat family, a low-complexity
// run; the C5 hot-bucket set) would pile its whole family into one ~3K-slot slice: the window
// overflows, the slice fills, and every spilled key linear-probes from inside the full slice. The
// fixup between pass 2 and the build remaps such regions as a whole (kh_codec.hpp place_w): keys of a
// remapped region go to the region of a second mix of their key hash, i.e. evenly over all regions,
// and every lookup (find, walk, CAS insert) places keys the same way from the bitmap.
//   k_hot_mark     region r is remapped when it already was, or (an empty table's build) when its
//                  count exceeds what its window (RC) or its slice (S_r slots) holds; the bitmap is
//                  rewritten and the remapped regions listed (CT_HOT)
//   k_hot_gather   the listed regions' window words join the overflow list; their windows empty
//   k_ovf_scatter  every overflow-list word goes to the window of its (remapped) region; what does
//                  not fit goes to list B (buf1, CT_OVF2), which the global CAS insert takes
// Cost without hot regions: three launches over nothing (~15 us); words move only for remapped
// regions and for windows that were full.
// counts: exact region counts (sample_shift 0) or a 1-in-2^sample_shift sample of the batch
// (k_part1_convert / k_sample_regions); a sampled region counts as hot only above twice the
// threshold and with >= 16 samples (the exact mark after pass 2 catches what the sample misses). CT_HOT is the bitmap's
// population; list_new lists the regions this mark added (CT_HOTNEW) for k_hot_gather.
template <int Unused = 0>
__global__ __launch_bounds__(256) void k_hot_mark(KParams p, uint64_t cap, uint32_t RC, int slack16, int sample_shift,
                                                  const uint32_t* counts, uint32_t* hot, uint32_t* hot_list,
                                                  unsigned long long* ctr, int allow_new, int list_new, uint32_t Tfix,
                                                  int ct = CT_HOT, int both = 0) {
    const uint32_t NR = nreg(p);
    const uint32_t r = blockIdx.x * 256u + threadIdx.x;
    bool h = false, hn = false, h2 = false;
    if (r < NR) {
        // equal ranges: what the slice holds; balanced bounds (Tfix): what the largest slice holds
        const uint32_t S = Tfix ? Tfix : (uint32_t)(region_lo(r + 1, cap, p) - region_lo(r, cap, p));
        const uint64_t T = min(RC, S - (slack16 ? S / 16u : 0u));
        const bool old = (hot[r >> 5] >> (r & 31u)) & 1u;
        // sampled: also at least 16 samples, so a small sample (the first of 16 upload chunks: 0.4
        // samples per region on average) cannot mark a region on Poisson noise alone
        const bool over = sample_shift ? counts[r] >= 16u && ((uint64_t)counts[r] << sample_shift) > 2 * T
                                       : counts[r] > T;
        hn = allow_new && !old && over;
        h = old || hn;
        if (both) {  // the exact mark: an overfull region is marked at both levels (see hot_fixup)
            const bool old2 = (hot[HOT_LEVEL_WORDS + (r >> 5)] >> (r & 31u)) & 1u;
            hn = allow_new && over && !(old && old2);
            h2 = old2 || (allow_new && over);
        }
    }
    const uint64_t m = __ballot(h);
    const uint32_t lane = lane_id();
    const uint32_t r0 = r - lane;  // the wave's 64 regions: two bitmap words
    if (r0 < NR && (lane == 0 || lane == 32)) hot[(r0 >> 5) + (lane >> 5)] = (uint32_t)(m >> lane);
    if (lane == 0 && m) atomicAdd(&ctr[ct], (unsigned long long)__popcll(m));
    if (both) {
        const uint64_t m2 = __ballot(h2);
        if (r0 < NR && (lane == 0 || lane == 32))
            hot[HOT_LEVEL_WORDS + (r0 >> 5) + (lane >> 5)] = (uint32_t)(m2 >> lane);
        if (lane == 0 && m2) atomicAdd(&ctr[CT_HOT2], (unsigned long long)__popcll(m2));
    }
    const unsigned long long i = wave_reserve(&ctr[CT_HOTNEW], list_new && hn);
    if (list_new && hn) hot_list[i] = r;
}

// Sampled region counts go through a per-block LDS table first (hashed, one slot per region; a
// region colliding with another goes straight to the global counter): a hot family's samples hit
// one global counter ~30K times at C5H, and same-address atomics serialise (~11 ns each:
// k_sample_records 0.34 ms at C5H vs 0.04 at C3); per block they become one atomic per region.
static constexpr uint32_t SAMPLE_TAB = 1024;
struct SampleTab {
    uint32_t key[SAMPLE_TAB];  // region + 1, 0 = free
    uint32_t cnt[SAMPLE_TAB];
};
__device__ __forceinline__ void sample_init(SampleTab& t) {
    for (uint32_t i = threadIdx.x; i < SAMPLE_TAB; i += blockDim.x) t.key[i] = t.cnt[i] = 0u;
    __syncthreads();
}
__device__ __forceinline__ void sample_add(SampleTab& t, uint32_t* counts, uint32_t r) {
    const uint32_t h = (r * 0x9E3779B1u) >> 22;  // 10 bits
    const uint32_t prev = atomicCAS(&t.key[h], 0u, r + 1u);
    if (prev == 0u || prev == r + 1u)
        atomicAdd(&t.cnt[h], 1u);
    else
        atomicAdd(&counts[r], 1u);
}
__device__ __forceinline__ void sample_flush(SampleTab& t, uint32_t* counts) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < SAMPLE_TAB; i += blockDim.x)
        if (t.key[i]) atomicAdd(&counts[t.key[i] - 1u], t.cnt[i]);
}
static_assert(SAMPLE_TAB == 1u << 10, "sample_add hashes to 10 bits");

// A 1-in-256 sample of routed words (the sharded path's first stage / one-shot insert): region
// counts for the sampled mark, so a hot family is placed by key hash in pass 1 already.
template <int W>
__global__ __launch_bounds__(256) void k_sample_regions(KParams p, const uint64_t* __restrict__ words, uint64_t m,
                                                        uint32_t* counts) {
    __shared__ SampleTab tab;
    sample_init(tab);
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) << 8; i < m; i += ((uint64_t)gridDim.x * 256) << 8) {
        const uint64_t w0 = words[i * W], w1 = W == 2 ? words[i * W + 1] : 0ull;
        sample_add(tab, counts, mini_region(word_mini_window(w0, w1, p), p));
    }
    sample_flush(tab, counts);
}

// The same sample read straight from the reference records (the records pass 1, k_win1_rec, has
// no earlier pass to count in): record 256 i, one aligned 16-B pair of loads each.
template <int W, int KT>
__global__ __launch_bounds__(256) void k_sample_records(KParams p_in, const uint8_t* __restrict__ recs, uint64_t n,
                                                        uint32_t* counts) {
    const KParams p = specialize<KT>(p_in);
    __shared__ SampleTab tab;
    sample_init(tab);
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) << 8; i < n; i += ((uint64_t)gridDim.x * 256) << 8) {
        uint64_t x0, x1;
        load_record_regs(recs, i, (uint32_t)p.R, x0, x1);
        Key k;
        uint32_t ext;
        parse_record_regs(x0, x1, p, k, ext);
        sample_add(tab, counts, mini_region(mini_window(k, mini_scan(k, p), p), p));
    }
    sample_flush(tab, counts);
}

template <int W>
__global__ __launch_bounds__(256) void k_hot_gather(uint32_t RC, uint32_t* rcnt, const uint32_t* hot_list,
                                                    const uint64_t* __restrict__ buf2, uint64_t* ovf, uint64_t ovf_cap,
                                                    unsigned long long* ctr, unsigned long long* stats) {
    __shared__ unsigned long long base;
    const uint64_t nh = ctr[CT_HOTNEW];
    for (uint64_t i = blockIdx.x; i < nh; i += gridDim.x) {
        const uint32_t r = hot_list[i];
        const uint32_t m = min(rcnt[r], RC);
        if (threadIdx.x == 0) base = m ? atomicAdd(&ctr[CT_OVF], (unsigned long long)m) : 0ull;
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < m; j += 256) {
            const uint64_t d = base + j;
            if (d >= ovf_cap) {
                atomicAdd(&stats[ST_FULL], 1ull);
                continue;
            }
            const uint64_t g = (uint64_t)r * RC + j;
            if (W == 2) {
                *reinterpret_cast<ulonglong2*>(ovf + d * 2) = *reinterpret_cast<const ulonglong2*>(buf2 + g * 2);
            } else {
                ovf[d] = buf2[g];
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) rcnt[r] = 0;
    }
}

template <int W>
__global__ __launch_bounds__(256) void k_ovf_scatter(KParams p, uint32_t RC, uint32_t* rcnt,
                                                     const uint64_t* __restrict__ ovf, uint64_t ovf_cap, uint64_t* buf2,
                                                     uint64_t* ovf2, uint64_t ovf2_cap, unsigned long long* ctr,
                                                     unsigned long long* stats) {
    const uint64_t m = min((uint64_t)ctr[CT_OVF], ovf_cap);
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
        uint64_t w0, w1 = 0;
        if (W == 2) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(ovf + i * 2);
            w0 = v.x;
            w1 = v.y;
        } else {
            w0 = ovf[i];
        }
        const uint32_t r = word_place(w0, w1, p).r;  // remapped regions: the key-hash region
        const uint32_t pos = wave_count_add(rcnt, r, true);
        if (pos < RC) {
            const uint64_t g = (uint64_t)r * RC + pos;
            if (W == 2) {
                *reinterpret_cast<ulonglong2*>(buf2 + g * 2) = make_ulonglong2(w0, w1);
            } else {
                buf2[g] = w0;
            }
        }
        const unsigned long long d = wave_reserve(&ctr[CT_OVF2], pos >= RC);
        if (pos >= RC) {
            if (d < ovf2_cap) {
                ovf2[d * W] = w0;
                if (W == 2) ovf2[d * W + 1] = w1;
            } else {
                atomicAdd(&stats[ST_FULL], 1ull);
            }
        }
    }
}

template <int W>
static void hot_fixup(const KParams& p, uint64_t cap, uint64_t n, uint32_t RC, bool allow_new, const PartBuffers& B,
                      uint64_t ovf_cap, uint64_t ovf2_cap, unsigned long long* ctr, unsigned long long* stats,
                      hipStream_t s) {
    KParams q = p;
    q.hot = B.hot;
    // Exact counts after pass 2: a region its window or slice cannot hold is marked at both levels —
    // level 1 remaps its own keys (a hot family the sample missed), level 2 spreads the keys the
    // level-1 remap sent into it (a family sharing its neighbour window too, which the sampled
    // level-2 mark missed: C5F had ~37K such keys left to the global CAS insert, whose probe runs
    // through full slices then made the insert 1.1 ms and the walk's lookups of them ~3 ms).
    // Then the newly marked regions' words are re-placed.
    (void)hipMemsetAsync(ctr + CT_HOT2, 0, 8, s);
    k_hot_mark<<<(nreg(p) + 255) / 256, 256, 0, s>>>(q, cap, RC, 0, 0, B.rcnt, B.hot, B.hot_list, ctr,
                                                     allow_new ? 1 : 0, 1, balanced_T(p, cap, n), CT_HOT, 1);
    k_hot_gather<W><<<1024, 256, 0, s>>>(RC, B.rcnt, B.hot_list, B.buf2, B.overflow, ovf_cap, ctr, stats);
    k_ovf_scatter<W><<<2048, 256, 0, s>>>(q, RC, B.rcnt, B.overflow, ovf_cap, B.buf2, B.buf1, ovf2_cap, ctr, stats);
}

template <int W>
static hipError_t build_launch(const KParams& p, uint64_t total, TableView t, bool table_empty, const PartBuffers& B,
                               unsigned long long* ctr, unsigned long long* stats, hipStream_t s,
                               hipEvent_t after_hot = nullptr) {
    hipError_t e;
    const size_t lds = (size_t)build_lds(p, t.cap, B.headrec && B.hcap);
    if ((e = allow_lds(k_part_build<W>, lds)) != hipSuccess) return e;
    if ((e = with_kt<W>(p.K, [&](auto kt) {
             constexpr int KT = decltype(kt)::value;
             hipError_t x;
             if constexpr (W == 2 && Slice<W>::SPLIT) {  // the sorted-slice variants (pf_launch)
                 if ((x = allow_lds(k_part_build_pf<W, 4, KT, true, true>, lds)) != hipSuccess) return x;
                 if ((x = allow_lds(k_part_build_pf<W, 6, KT, true, true>, lds)) != hipSuccess) return x;
                 if ((x = allow_lds(k_part_build_pf<W, 12, KT, true, true>, lds)) != hipSuccess) return x;
             }
             if ((x = allow_lds(k_part_build_pf<W, 4, KT, true>, lds)) != hipSuccess) return x;
             if ((x = allow_lds(k_part_build_pf<W, 6, KT, true>, lds)) != hipSuccess) return x;
             if ((x = allow_lds(k_part_build_pf<W, 12, KT, true>, lds)) != hipSuccess) return x;
             if ((x = allow_lds(k_part_build_pf<W, 4, KT, false>, lds)) != hipSuccess) return x;
             if ((x = allow_lds(k_part_build_pf<W, 6, KT, false>, lds)) != hipSuccess) return x;
             return allow_lds(k_part_build_pf<W, 12, KT, false>, lds);
         })) != hipSuccess)
        return e;
    const uint32_t RC = part_region_cap(p, total);
    const uint64_t ovf2_cap = part_buf1_words(p, total) / p.W;  // list B lives in buf1 (dead after pass 2)
    if ((e = hipMemsetAsync(ctr + CT_OVF2, 0, 24, s)) != hipSuccess) return e;  // CT_OVF2, CT_HOT, CT_HOTNEW
    static_assert(CT_HOT == CT_OVF2 + 1 && CT_HOTNEW == CT_HOT + 1, "counter layout");
    hot_fixup<W>(p, t.cap, total, RC, table_empty, B, part_overflow_cap(total), ovf2_cap, ctr, stats, s);
    // the remapped-region count (CT_HOT) is final here: the caller may read it beside the build
    if (after_hot && (e = hipEventRecord(after_hot, s)) != hipSuccess) return e;
    KParams q = p;  // the build and the CAS inserts place keys of remapped regions by key hash
    q.hot = B.hot;
    // balanced bounds: an empty table's build sizes every region slice from its final count
    if (p.rb && table_empty) launch_bounds(p, t.cap, B.rcnt, RC, const_cast<uint64_t*>(B.rbt), s);
    launch_build_windows<W>(q, B, t, table_empty, ovf2_cap, ctr, stats, RC,
                            reinterpret_cast<const uint32_t*>(B.rcnt), lds, s);
    k_insert_overflow<W><<<1024, PB, 0, s>>>(q, B.buf1, ovf2_cap, ctr, t.slots, t.cap, stats);
    return hipGetLastError();
}

// ---- CAS-path hot prepass --------------------------------------------------------------------------
template <int W, bool REC>
__global__ __launch_bounds__(256) void k_region_count(KParams p, const uint8_t* __restrict__ recs,
                                                      const uint64_t* __restrict__ words, uint64_t n, uint32_t* rcnt,
                                                      int remapped) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        uint32_t win;
        Key k;
        if (REC) {
            uint32_t ext;
            parse_record(recs + i * (uint64_t)p.R, p, k, ext);
            win = mini_window(k, mini_scan(k, p), p);
        } else {
            const uint64_t w0 = words[i * W], w1 = W == 2 ? words[i * W + 1] : 0ull;
            k = slot_key(w0, w1, p);
            win = word_mini_window(w0, w1, p);
        }
        // remapped: the region the insert will use (hot regions by key hash)
        (void)wave_count_add(rcnt, remapped ? place_w(win, k, p).r : mini_region(win, p), true);
    }
}

hipError_t launch_hot_prepass(const KParams& p, const uint8_t* recs, const uint64_t* words, uint64_t n,
                              uint64_t cap, uint32_t* rcnt, uint32_t* hot, uint32_t* hot_list,
                              unsigned long long* ctr, hipStream_t s, uint64_t total) {
    hipError_t e;
    {
        FillSet f;
        f.add(rcnt, (uint64_t)nreg(p) * 4, 0);
        f.add(ctr + CT_HOT, 16, 0);
        if ((e = launch_fill(f, s)) != hipSuccess) return e;
    }
    if (n) {
        const unsigned grid = (unsigned)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
        if (p.W == 2) {
            if (recs) k_region_count<2, true><<<grid, 256, 0, s>>>(p, recs, nullptr, n, rcnt, 0);
            else k_region_count<2, false><<<grid, 256, 0, s>>>(p, nullptr, words, n, rcnt, 0);
        } else {
            if (recs) k_region_count<1, true><<<grid, 256, 0, s>>>(p, recs, nullptr, n, rcnt, 0);
            else k_region_count<1, false><<<grid, 256, 0, s>>>(p, nullptr, words, n, rcnt, 0);
        }
    }
    // linear probing across region boundaries: remap what would fill more than 15/16 of a slice.
    // The first of several staged batches (total > n) is a sample of the build: its counts are
    // scaled up (with the sampled mark's noise guard) instead of compared with whole slices.
    KParams q = p;
    q.hot = hot;
    int shift = 0;
    while (n && total > n && ((uint64_t)n << (shift + 1)) <= total) ++shift;
    const uint32_t Tb = balanced_T(p, cap, total > n ? total : n);
    k_hot_mark<<<(nreg(p) + 255) / 256, 256, 0, s>>>(q, cap, 0xFFFFFFFFu, shift ? 0 : 1, shift, rcnt, hot, hot_list,
                                                     ctr, 1, 0, Tb);
    auto count_placed = [&]() -> hipError_t {  // the region each key goes to under the bitmap so far
        hipError_t x;
        if ((x = hipMemsetAsync(rcnt, 0, (size_t)nreg(p) * 4, s)) != hipSuccess) return x;
        if (n) {
            const unsigned grid = (unsigned)((n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048);
            if (p.W == 2) {
                if (recs) k_region_count<2, true><<<grid, 256, 0, s>>>(q, recs, nullptr, n, rcnt, 1);
                else k_region_count<2, false><<<grid, 256, 0, s>>>(q, nullptr, words, n, rcnt, 1);
            } else {
                if (recs) k_region_count<1, true><<<grid, 256, 0, s>>>(q, recs, nullptr, n, rcnt, 1);
                else k_region_count<1, false><<<grid, 256, 0, s>>>(q, nullptr, words, n, rcnt, 1);
            }
        }
        return hipGetLastError();
    };
    // level 2: target regions the remap overfills (kh_codec.hpp remap_region)
    if ((e = count_placed()) != hipSuccess) return e;
    if ((e = hipMemsetAsync(ctr + CT_HOT2, 0, 8, s)) != hipSuccess) return e;
    k_hot_mark<<<(nreg(p) + 255) / 256, 256, 0, s>>>(q, cap, 0xFFFFFFFFu, shift ? 0 : 1, shift, rcnt, hot + HOT_WORDS,
                                                     hot_list, ctr, 1, 0, Tb, CT_HOT2);
    if (p.rb) {  // balanced bounds from the counts after the remap (a hot-aware count)
        if ((e = count_placed()) != hipSuccess) return e;
        launch_bounds(p, cap, rcnt, 0xFFFFFFFFu, const_cast<uint64_t*>(p.rb), s);
    }
    return hipGetLastError();
}

// Hot regions from a 1-in-256 sample of the batch (in B.rcnt, left zeroed for pass 2).
template <int W>
static hipError_t sample_records(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t* counts, hipStream_t s) {
    const uint64_t ns = (n + 255) >> 8;
    const unsigned nb = (unsigned)((ns + 255) / 256 < 1024 ? (ns + 255) / 256 : 1024);
    return with_kt<W>(p.K, [&](auto kt) {
        k_sample_records<W, decltype(kt)::value><<<nb, 256, 0, s>>>(p, recs, n, counts);
        return hipGetLastError();
    });
}

static hipError_t sample_mark(const KParams& p, uint64_t cap, uint64_t n, uint32_t RC, const PartBuffers& B,
                              unsigned long long* ctr, hipStream_t s) {
    hipError_t e;
    KParams q = p;
    q.hot = B.hot;
    if ((e = hipMemsetAsync(ctr + CT_HOT, 0, 16, s)) != hipSuccess) return e;  // CT_HOT, CT_HOTNEW
    k_hot_mark<<<(nreg(p) + 255) / 256, 256, 0, s>>>(q, cap, RC, 0, 8, B.rcnt, B.hot, B.hot_list, ctr, 1, 0,
                                                     balanced_T(p, cap, n));
    // the region counts for level 2 (sample_level2, always next) and its counter
    FillSet f;
    f.add(B.rcnt, (uint64_t)nreg(p) * 4, 0);
    f.add(ctr + CT_HOT2, 8, 0);
    return launch_fill(f, s);
}

// Level 2 of the bitmap (kh_codec.hpp remap_region): a 1-in-256 sample of the batch counted by its
// placement under level 1 marks the target regions the remap overfills (a family whose copies also
// share the neighbour window lands in one), so their remapped keys spread by key hash before pass 1
// instead of piling into one window and the global CAS list (quadratic probe runs in the worst
// case). Same sampled threshold as level 1. Returns at once when level 1 marked nothing.
template <int W, bool REC, int KT>
__global__ __launch_bounds__(256) void k_sample_placed(KParams p_in, const uint8_t* __restrict__ recs,
                                                       const uint64_t* __restrict__ words, uint64_t n, uint32_t* counts,
                                                       const unsigned long long* ctr) {
    if (!ctr[CT_HOT]) return;
    const KParams p = specialize<KT>(p_in);
    __shared__ SampleTab tab;
    sample_init(tab);
    for (uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) << 8; i < n; i += ((uint64_t)gridDim.x * 256) << 8) {
        uint32_t r;
        if (REC) {
            uint64_t x0, x1;
            load_record_regs(recs, i, (uint32_t)p.R, x0, x1);
            Key k;
            uint32_t ext;
            parse_record_regs(x0, x1, p, k, ext);
            const uint32_t mn = mini_scan(k, p);
            r = place_w(mini_window(k, mn, p), k, p, (int)(mn & 63u)).r;
        } else {
            r = word_place(words[i * W], W == 2 ? words[i * W + 1] : 0ull, p).r;
        }
        sample_add(tab, counts, r);
    }
    sample_flush(tab, counts);
}

// recs (records) or words (partition words carrying j*) of a batch of n, scaled to a build of
// RC-word windows; counts: zeroed region counters (left zeroed)
template <int W>
static hipError_t sample_level2(const KParams& p, const uint8_t* recs, const uint64_t* words, uint64_t n,
                                uint64_t cap, uint32_t RC, uint64_t total, const PartBuffers& B,
                                unsigned long long* ctr, hipStream_t s) {
    KParams q = p;
    q.hot = B.hot;
    const uint64_t ns = (n + 255) >> 8;
    const unsigned nb = (unsigned)((ns + 255) / 256 < 1024 ? (ns + 255) / 256 : 1024);
    hipError_t e;
    if ((e = with_kt<W>(p.K, [&](auto kt) {
             constexpr int KT = decltype(kt)::value;
             if (recs)
                 k_sample_placed<W, true, KT><<<nb, 256, 0, s>>>(q, recs, nullptr, n, B.rcnt, ctr);
             else
                 k_sample_placed<W, false, KT><<<nb, 256, 0, s>>>(q, nullptr, words, n, B.rcnt, ctr);
             return hipGetLastError();
         })) != hipSuccess)
        return e;
    // (ctr[CT_HOT2] was zeroed by sample_mark)
    k_hot_mark<<<(nreg(p) + 255) / 256, 256, 0, s>>>(q, cap, RC, 0, 8, B.rcnt, B.hot + HOT_WORDS, B.hot_list, ctr, 1, 0,
                                                     balanced_T(p, cap, total), CT_HOT2);
    return hipMemsetAsync(B.rcnt, 0, (size_t)nreg(p) * 4, s);
}

template <int W>
static bool rec_pass_ok(const KParams& p) {
    return (p.P == 13 && W == 2) || (p.P == 5 && W == 1);
}

// One batch: pass 1 (records or words), pass 2, build, overflow inserts.
template <int W, bool REC>
static hipError_t part_insert(const KParams& p, const uint8_t* recs, const uint64_t* words, uint64_t n,
                              TableView t, bool table_empty, const PartBuffers& B, uint64_t* start_mask,
                              uint64_t* split_mask, unsigned long long* ctr, unsigned long long* stats, hipStream_t s,
                              hipEvent_t after_records = nullptr, uint64_t* wsplits = nullptr,
                              uint64_t wsplits_cap = 0, hipEvent_t before_build = nullptr,
                              hipEvent_t after_hot = nullptr) {
    hipError_t e;
    const uint64_t ovf_cap = part_overflow_cap(n);
    const uint32_t CAP1 = part_win1_cap(n), RC = part_region_cap(p, n);
    uint32_t* wcnt = B.wcnt;
    uint32_t* rcnt = B.rcnt;
    {
        FillSet f;
        f.add(ctr + CT_OVF, 8, 0);
        f.add(wcnt, (uint64_t)NW1 * 4, 0);
        f.add(rcnt, (uint64_t)nreg(p) * 4, 0);
        if ((e = launch_fill(f, s)) != hipSuccess) return e;
    }
    // records of a compiled shape (k=51 / k=19 packed sizes): pass 1 reads them itself, no
    // record -> word copy (other shapes: the convert pass + pass 1 on its words)
    const bool rec_pass = REC && rec_pass_ok<W>(p);
    // empty table: a 1-in-256 sample of the batch's minimizer regions marks the hot ones before
    // pass 1, so their keys are sorted straight into their key-hash regions (no spill storm)
    const bool sample = table_empty;
    uint32_t* samp = (REC && sample) ? rcnt : nullptr;
    if (rec_pass && sample) {
        if ((e = sample_records<W>(p, recs, n, rcnt, s)) != hipSuccess) return e;
        if ((e = sample_mark(p, t.cap, n, RC, B, ctr, s)) != hipSuccess) return e;
        if ((e = sample_level2<W>(p, recs, nullptr, n, t.cap, RC, n, B, ctr, s)) != hipSuccess) return e;
    }
    if (!REC && sample) {
        const uint64_t ns = (n + 255) >> 8;
        k_sample_regions<W><<<(unsigned)((ns + 255) / 256 < 1024 ? (ns + 255) / 256 : 1024), 256, 0, s>>>(p, words, n,
                                                                                                          rcnt);
    }
    if (rec_pass) {
        if ((e = win1_rec_launch<W>(p, recs, n, CAP1, wcnt, B, start_mask, split_mask, ovf_cap, ctr, stats, s)) !=
            hipSuccess)
            return e;
    } else {
        if (REC) {  // records -> words (input order) in buf2, which pass 2 only writes after pass 1
            const unsigned nb = (unsigned)((n + (uint64_t)T1 * PART_TILE - 1) / ((uint64_t)T1 * PART_TILE));
            if (W == 2 && p.K == 51)  // compile-time shape: aligned 8-B LDS reads, constant masks
                k_part1_convert<W, 13, 51><<<nb, PB, 0, s>>>(p, recs, n, B.buf2, start_mask, split_mask, samp);
            else if (W == 1 && p.K == 19)
                k_part1_convert<W, 5, 19><<<nb, PB, 0, s>>>(p, recs, n, B.buf2, start_mask, split_mask, samp);
            else if (p.P == 13)
                k_part1_convert<W, 13><<<nb, PB, 0, s>>>(p, recs, n, B.buf2, start_mask, split_mask, samp);
            else if (p.P == 5)
                k_part1_convert<W, 5><<<nb, PB, 0, s>>>(p, recs, n, B.buf2, start_mask, split_mask, samp);
            else
                k_part1_convert<W><<<nb, PB, 0, s>>>(p, recs, n, B.buf2, start_mask, split_mask, samp);
            words = B.buf2;
        }
        if (sample && (e = sample_mark(p, t.cap, n, RC, B, ctr, s)) != hipSuccess) return e;
        if (sample && (e = sample_level2<W>(p, nullptr, words, n, t.cap, RC, n, B, ctr, s)) != hipSuccess) return e;
        // converted records and routed words (k_route_scatter) both carry j* and the order bits
        if ((e = win1_launch<W>(p, words, n, CAP1, wcnt, B, ovf_cap, ctr, stats, s, REC ? nullptr : wsplits,
                                wsplits_cap, true)) != hipSuccess)
            return e;
    }
    // start / splitter bits are complete: the caller's compaction may start
    if (after_records && (e = hipEventRecord(after_records, s)) != hipSuccess) return e;
    if ((e = win2_launch<W>(p, B, n, RC, rcnt, ovf_cap, ctr, stats, CAP1, wcnt, s)) != hipSuccess) return e;
    if (before_build && (e = hipEventRecord(before_build, s)) != hipSuccess) return e;
    return build_launch<W>(p, n, t, table_empty, B, ctr, stats, s, after_hot);
}

// Staged build (sharded insert): words arrive in chunks (one per all-to-all chunk). Each chunk is
// partitioned at once (pass 1 into its own windows, pass 2 appending to the region windows of a
// build sized for `total` words) while the next chunk is still on the wire; one build at the end.
template <int W>
static hipError_t part_stage(const KParams& p, const uint64_t* words, uint64_t m, uint64_t total, bool first,
                             const PartBuffers& B, unsigned long long* ctr, unsigned long long* stats,
                             hipStream_t s, uint64_t* wsplits, uint64_t wsplits_cap, bool sample, uint64_t cap) {
    hipError_t e;
    if (first) {
        if ((e = hipMemsetAsync(ctr + CT_OVF, 0, 8, s)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(B.rcnt, 0, (size_t)nreg(p) * 4, s)) != hipSuccess) return e;
    }
    if (m == 0) return hipSuccess;
    const uint32_t CAP1 = part_win1_cap(m), RC = part_region_cap(p, total);
    if (sample) {  // the first chunk's sample marks the hot regions
        const uint64_t ns = (m + 255) >> 8;
        k_sample_regions<W><<<(unsigned)((ns + 255) / 256 < 1024 ? (ns + 255) / 256 : 1024), 256, 0, s>>>(p, words, m,
                                                                                                          B.rcnt);
        // the sample covers this chunk: scale it to the whole build (chunks are alike)
        const uint32_t RCm = (uint32_t)((uint64_t)RC * m / total);
        if ((e = sample_mark(p, cap, m, RCm, B, ctr, s)) != hipSuccess) return e;
        if ((e = sample_level2<W>(p, nullptr, words, m, cap, RCm, m, B, ctr, s)) != hipSuccess) return e;
    }
    if ((e = hipMemsetAsync(B.wcnt, 0, (size_t)NW1 * 4, s)) != hipSuccess) return e;
    if ((e = win1_launch<W>(p, words, m, CAP1, B.wcnt, B, part_overflow_cap(total), ctr, stats, s, wsplits,
                            wsplits_cap, true)) != hipSuccess)
        return e;
    if ((e = win2_launch<W>(p, B, m, RC, B.rcnt, part_overflow_cap(total), ctr, stats, CAP1, B.wcnt, s)) != hipSuccess)
        return e;
    return hipGetLastError();
}

hipError_t launch_part_stage(const KParams& p, const uint64_t* words, uint64_t m, uint64_t total, bool first,
                             const PartBuffers& b, unsigned long long* ctr, unsigned long long* stats,
                             hipStream_t s, uint64_t* wsplits, uint64_t wsplits_cap, bool sample, uint64_t cap) {
    return p.W == 1 ? part_stage<1>(p, words, m, total, first, b, ctr, stats, s, wsplits, wsplits_cap, sample, cap)
                    : part_stage<2>(p, words, m, total, first, b, ctr, stats, s, wsplits, wsplits_cap, sample, cap);
}

// Staged build from reference records (kh_insert's chunked host upload): the chunk is converted
// (start / splitter bits into its slice of the masks, words into words_tmp), then partitioned like
// a routed chunk; first: counters of the build; sample: this chunk's 1-in-256 sample marks the hot
// regions before its pass 1.
template <int W>
static hipError_t part_stage_recs(const KParams& p, const uint8_t* recs, uint64_t m, uint64_t total, bool first,
                                  const PartBuffers& B, uint64_t* words_tmp, uint64_t* start_mask, uint64_t* split_mask,
                                  unsigned long long* ctr, unsigned long long* stats, hipStream_t s, bool sample,
                                  uint64_t cap) {
    hipError_t e;
    if (first) {
        if ((e = hipMemsetAsync(ctr + CT_OVF, 0, 8, s)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(B.rcnt, 0, (size_t)nreg(p) * 4, s)) != hipSuccess) return e;
    }
    if (m == 0) return hipSuccess;
    const uint32_t CAP1 = part_win1_cap(m), RC = part_region_cap(p, total);
    const bool samp_on = sample;
    if (rec_pass_ok<W>(p)) {
        if (samp_on) {
            const uint32_t RCm = (uint32_t)((uint64_t)RC * m / total);
            if ((e = sample_records<W>(p, recs, m, B.rcnt, s)) != hipSuccess) return e;
            if ((e = sample_mark(p, cap, m, RCm, B, ctr, s)) != hipSuccess) return e;
            if ((e = sample_level2<W>(p, recs, nullptr, m, cap, RCm, m, B, ctr, s)) != hipSuccess) return e;
        }
        if ((e = hipMemsetAsync(B.wcnt, 0, (size_t)NW1 * 4, s)) != hipSuccess) return e;
        if ((e = win1_rec_launch<W>(p, recs, m, CAP1, B.wcnt, B, start_mask, split_mask, part_overflow_cap(total), ctr,
                                    stats, s)) != hipSuccess)
            return e;
        if ((e = win2_launch<W>(p, B, m, RC, B.rcnt, part_overflow_cap(total), ctr, stats, CAP1, B.wcnt, s)) !=
            hipSuccess)
            return e;
        return hipGetLastError();
    }
    uint32_t* samp = samp_on ? B.rcnt : nullptr;
    const unsigned nb = (unsigned)((m + (uint64_t)T1 * PART_TILE - 1) / ((uint64_t)T1 * PART_TILE));
    if (W == 2 && p.K == 51)
        k_part1_convert<W, 13, 51><<<nb, PB, 0, s>>>(p, recs, m, words_tmp, start_mask, split_mask, samp);
    else if (W == 1 && p.K == 19)
        k_part1_convert<W, 5, 19><<<nb, PB, 0, s>>>(p, recs, m, words_tmp, start_mask, split_mask, samp);
    else if (p.P == 13)
        k_part1_convert<W, 13><<<nb, PB, 0, s>>>(p, recs, m, words_tmp, start_mask, split_mask, samp);
    else if (p.P == 5)
        k_part1_convert<W, 5><<<nb, PB, 0, s>>>(p, recs, m, words_tmp, start_mask, split_mask, samp);
    else
        k_part1_convert<W><<<nb, PB, 0, s>>>(p, recs, m, words_tmp, start_mask, split_mask, samp);
    if (samp_on) {
        const uint32_t RCm = (uint32_t)((uint64_t)RC * m / total);
        if ((e = sample_mark(p, cap, m, RCm, B, ctr, s)) != hipSuccess) return e;
        if ((e = sample_level2<W>(p, nullptr, words_tmp, m, cap, RCm, m, B, ctr, s)) != hipSuccess) return e;
    }
    if ((e = hipMemsetAsync(B.wcnt, 0, (size_t)NW1 * 4, s)) != hipSuccess) return e;
    if ((e = win1_launch<W>(p, words_tmp, m, CAP1, B.wcnt, B, part_overflow_cap(total), ctr, stats, s, nullptr, 0,
                            true)) != hipSuccess)
        return e;
    if ((e = win2_launch<W>(p, B, m, RC, B.rcnt, part_overflow_cap(total), ctr, stats, CAP1, B.wcnt, s)) != hipSuccess)
        return e;
    return hipGetLastError();
}

hipError_t launch_part_stage_recs(const KParams& p, const uint8_t* recs, uint64_t m, uint64_t total, bool first,
                                  const PartBuffers& b, uint64_t* words_tmp, uint64_t* start_mask,
                                  uint64_t* split_mask, unsigned long long* ctr, unsigned long long* stats,
                                  hipStream_t s, bool sample, uint64_t cap) {
    return p.W == 1 ? part_stage_recs<1>(p, recs, m, total, first, b, words_tmp, start_mask, split_mask, ctr, stats, s,
                                         sample, cap)
                    : part_stage_recs<2>(p, recs, m, total, first, b, words_tmp, start_mask, split_mask, ctr, stats, s,
                                         sample, cap);
}

hipError_t launch_part_finish(const KParams& p, uint64_t total, TableView t, bool table_empty,
                              const PartBuffers& b, unsigned long long* ctr, unsigned long long* stats,
                              hipStream_t s) {
    return p.W == 1 ? build_launch<1>(p, total, t, table_empty, b, ctr, stats, s)
                    : build_launch<2>(p, total, t, table_empty, b, ctr, stats, s);
}

hipError_t launch_part_insert(const KParams& p, const uint8_t* recs, const uint64_t* words, uint64_t n,
                              TableView t, bool table_empty, const PartBuffers& b,
                              uint64_t* start_mask, uint64_t* split_mask, unsigned long long* ctr,
                              unsigned long long* stats, hipStream_t s, hipEvent_t after_records,
                              uint64_t* wsplits, uint64_t wsplits_cap, hipEvent_t before_build,
                              hipEvent_t after_hot) {
    if (n == 0) return hipSuccess;
    if (recs) {
        return p.W == 1 ? part_insert<1, true>(p, recs, nullptr, n, t, table_empty, b, start_mask, split_mask, ctr,
                                               stats, s, after_records, nullptr, 0, before_build, after_hot)
                        : part_insert<2, true>(p, recs, nullptr, n, t, table_empty, b, start_mask, split_mask, ctr,
                                               stats, s, after_records, nullptr, 0, before_build, after_hot);
    }
    return p.W == 1 ? part_insert<1, false>(p, nullptr, words, n, t, table_empty, b, nullptr, nullptr, ctr, stats, s,
                                            nullptr, wsplits, wsplits_cap, before_build)
                    : part_insert<2, false>(p, nullptr, words, n, t, table_empty, b, nullptr, nullptr, ctr, stats, s,
                                            nullptr, wsplits, wsplits_cap, before_build);
}

}  // namespace kh
