// kh_device.hpp — device helpers shared by the kernel translation units (not part of the ABI):
// block scan + 3-kernel exclusive scan, slot load, CAS insert, and the read-only probe.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "kh_codec.hpp"
#include "kh_kernels.hpp"

namespace kh {

static constexpr int BLOCK = 256;
static constexpr int SCAN_ITEMS = 8;
static constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;  // 2048 elements per block
static constexpr int WALK_GRAB = 64;                   // start k-mers per wave batch (one per lane)
// batches a wave reserves per work-queue atomic: the queue head is ONE global counter, and
// same-address atomics serialise (~11 ns each): C5's 21M short contigs pulled 64 at a time made
// 328K of them, ~3.7 ms of the walk. C5 walk kernel 4.80 ms at 1 batch, 3.27 at 8, 2.99 at 32
// (but C3 1.18 -> 1.85 ms at 32: long contigs leave a wave's reserved batches to one straggler)
static constexpr int WALK_BATCHES = 8;
static constexpr int MAX_R = 17;                       // K <= 60 -> PACKED <= 15 -> R <= 17

// Launch-side dispatch to the compile-time shape (specialize<KT>): f(integral_constant<KT>).
template <int W, class F>
inline auto with_kt(int K, F&& f) {
    if constexpr (W == 2) {
        if (K == 51) return f(std::integral_constant<int, 51>{});
    } else {
        if (K == 19) return f(std::integral_constant<int, 19>{});
    }
    return f(std::integral_constant<int, 0>{});
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
static inline uint64_t hmin(uint64_t a, uint64_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// One slot of a global list per lane that wants one, with ONE atomicAdd per wave on the list's
// counter (a hot region spilling thousands of words per wave would otherwise serialise on a single
// address). Call with every lane of the wave that reached this point; returns the lane's slot.
__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long* counter, bool want) {
    const uint64_t m = __ballot(want);
    if (!m) return 0ull;
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned long long base = 0;
    if ((int)lane_id() == leader) base = atomicAdd(counter, (unsigned long long)__popcll(m));
    base = __shfl(base, leader, 64);
    return base + mbcnt64(m);
}

// atomicAdd(&cnt[key], 1) for every lane that wants it. The lanes sharing the first lane's key are
// served by one atomic (a hot region's words arrive whole waves at a time: ~1 atomic per wave
// instead of 64 on one address); the others issue their own, all in flight at once (distinct
// random keys: one round trip, not one per key).
__device__ __forceinline__ uint32_t wave_count_add(uint32_t* cnt, uint32_t key, bool want) {
    const uint64_t act = __ballot(want);
    if (!act) return 0u;
    const int leader = __ffsll((unsigned long long)act) - 1;
    const uint32_t lk = __shfl(key, leader, 64);
    const uint64_t grp = __ballot(want && key == lk);
    const bool in_grp = (grp >> lane_id()) & 1ull;
    uint32_t old = 0;
    if ((int)lane_id() == leader) old = atomicAdd(&cnt[lk], (uint32_t)__popcll(grp));
    old = __shfl(old, leader, 64);
    if (in_grp) return old + mbcnt64(grp);
    return want ? atomicAdd(&cnt[key], 1u) : 0u;
}

// Quad (4-lane) exchanges by DPP: the walkers' transposed block probes (k_walk_q, k_mw_run).
template <int CTRL>
__device__ __forceinline__ uint32_t qperm32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int J>
__device__ __forceinline__ uint64_t qbcast64(uint64_t v) {  // value of quad lane J
    constexpr int C = J * 0x55;  // quad_perm [J,J,J,J]
    return ((uint64_t)qperm32<C>((uint32_t)(v >> 32)) << 32) | qperm32<C>((uint32_t)v);
}
__device__ __forceinline__ uint32_t qor32(uint32_t v) {
    v |= qperm32<0xB1>(v);  // [1,0,3,2]
    v |= qperm32<0x4E>(v);  // [2,3,0,1]
    return v;
}
static constexpr uint64_t WQ_REC = 1ull << 63;  // walker's next load is a head record (index below)
static constexpr uint64_t WQ_IDLE = ~0ull;

// Rank of each wanting lane among all lanes (of any wave) that add to cnt[key]: one atomic per
// distinct key in the wave (a loop over the wave's keys), so few keys (the route's owner ranks,
// one at P = 1) cost no same-address LDS atomic storm.
__device__ __forceinline__ uint32_t wave_rank_all(uint32_t* cnt, uint32_t key, bool want) {
    uint64_t act = __ballot(want);
    uint32_t r = 0;
    while (act) {  // uniform
        const int leader = __ffsll((unsigned long long)act) - 1;
        const uint32_t lk = __shfl(key, leader, 64);
        const uint64_t grp = __ballot(want && key == lk);
        uint32_t old = 0;
        if ((int)lane_id() == leader) old = atomicAdd(&cnt[lk], (uint32_t)__popcll(grp));
        old = __shfl(old, leader, 64);
        if ((grp >> lane_id()) & 1ull) r = old + mbcnt64(grp);
        act &= ~grp;
    }
    return r;
}

// ---------------------------------------------------------------------------------------------
// Block-wide exclusive scan of one uint64 per thread (256 threads = 4 waves of 64).
// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global loads/stores (HIP's __syncthreads also drains vmcnt, which serialises a tile's stores
// with the next tile's loads and kills any prefetch).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t& total) {
    __shared__ uint64_t wsum[BLOCK / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    lds_barrier();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < BLOCK / 64; ++i) {
        if (i < w) pre += wsum[i];
        tot += wsum[i];
    }
    lds_barrier();
    total = tot;
    return pre + x - v;
}

struct PopcF {
    const uint64_t* mask;
    __device__ uint64_t operator()(uint64_t i) const { return (uint64_t)__popcll(mask[i]); }
};

struct ContigBytesF {
    const uint32_t* len;
    uint64_t K;
    __device__ uint64_t operator()(uint64_t i) const { return K + (uint64_t)len[i]; }
};

// The tile's elements are read and written in striped order (element j * BLOCK + thread), so each
// load / store instruction covers consecutive addresses; the scan order is restored through LDS.
// (A thread's own 8 consecutive elements, 8 loads / stores 32-64 B apart per lane: C5's 21.8M-contig
// offsets scan 0.19 ms.)
template <class F>
__global__ __launch_bounds__(BLOCK) void k_scan_reduce(F f, uint64_t m, uint64_t* bsum) {
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_TILE + threadIdx.x;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j)
        if (b0 + (uint64_t)j * BLOCK < m) s += f(b0 + (uint64_t)j * BLOCK);
    uint64_t tot;
    block_excl_scan(s, tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// One block: exclusive scan of the nb block sums in place, starting at *base (if given);
// *base (if given) and *total_out (if given) receive base + sum.
template <int D>
__global__ __launch_bounds__(BLOCK) void k_scan_top(uint64_t* bsum, uint64_t nb,
                                                    unsigned long long* base,
                                                    unsigned long long* total_out) {
    uint64_t carry = base ? (uint64_t)*base : 0ull;
    for (uint64_t c0 = 0; c0 < nb; c0 += SCAN_TILE) {
        const uint64_t i0 = c0 + (uint64_t)threadIdx.x * SCAN_ITEMS;
        uint64_t v[SCAN_ITEMS];
        uint64_t s = 0;
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j) {
            v[j] = (i0 + j < nb) ? bsum[i0 + j] : 0ull;
            s += v[j];
        }
        uint64_t tot;
        uint64_t pre = block_excl_scan(s, tot) + carry;
#pragma unroll
        for (int j = 0; j < SCAN_ITEMS; ++j) {
            if (i0 + j < nb) bsum[i0 + j] = pre;
            pre += v[j];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) {
        if (base) *base = carry;
        if (total_out) *total_out = carry;
    }
}

struct IdentityIdx {
    __device__ uint64_t operator()(uint64_t i) const { return i; }
};

// out[o(i)] = exclusive prefix of f over [0, i): the scan order and the storage layout differ
// when a consumer wants its offsets contiguous (e.g. per block instead of per bin).
template <class F, class O = IdentityIdx>
__global__ __launch_bounds__(BLOCK) void k_scan_apply(F f, uint64_t m, const uint64_t* bsum,
                                                      uint64_t* out, O o = O()) {
    __shared__ uint64_t t[SCAN_TILE + SCAN_TILE / 32];  // + 1 word per 32: the transposed reads spread over banks
    auto at = [](uint32_t i) { return i + (i >> 5); };
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {  // striped, coalesced loads
        const uint32_t i = (uint32_t)j * BLOCK + threadIdx.x;
        t[at(i)] = base + i < m ? f(base + i) : 0ull;
    }
    lds_barrier();
    uint64_t v[SCAN_ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {  // this thread's consecutive elements
        v[j] = t[at(threadIdx.x * SCAN_ITEMS + j)];
        s += v[j];
    }
    uint64_t tot;
    uint64_t pre = block_excl_scan(s, tot) + bsum[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        t[at(threadIdx.x * SCAN_ITEMS + j)] = pre;
        pre += v[j];
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {  // striped, coalesced stores
        const uint32_t i = (uint32_t)j * BLOCK + threadIdx.x;
        if (base + i < m) out[o(base + i)] = t[at(i)];
    }
}


template <class F, class O = IdentityIdx>
static hipError_t scan_exclusive(F f, uint64_t m, uint64_t* out, uint64_t* scratch,
                                 unsigned long long* base, unsigned long long* total,
                                 hipStream_t s, O o = O()) {
    if (m == 0) return hipSuccess;
    const uint64_t nb = (m + SCAN_TILE - 1) / SCAN_TILE;
    k_scan_reduce<F><<<dim3((unsigned)nb), dim3(BLOCK), 0, s>>>(f, m, scratch);
    k_scan_top<0><<<1, BLOCK, 0, s>>>(scratch, nb, base, total);
    k_scan_apply<F, O><<<dim3((unsigned)nb), dim3(BLOCK), 0, s>>>(f, m, scratch, out, o);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Insert. One record per lane; a block stages 256 records (256*R contiguous bytes, 16-B aligned)
// through LDS with dwordx4 loads so the 15-byte (k=51) / 7-byte (k=19) records are read fully
// coalesced, then parses them from LDS.
//
// W=2 publish protocol (no 128-bit CAS on gfx950): CAS word0 (hi bits + ext) from EMPTY, then
// atomically store word1 (lo bits). A prober whose word0 matches ours must see word1 before it
// can decide; it re-reads word1 with an atomic (coherent across XCD L2s) on its next loop
// iteration — never spinning inside the branch, so a writer lane in the same wave always
// completes its store first.
// Probing reads slots with plain loads and spends an atomic only on a slot that looked EMPTY
// (a stale EMPTY just makes the CAS fail and return the live word; a live word never changes,
// so a plain read of one is never wrong). Word1 is published with a write-through (sc1) store.
template <int W>
__device__ __forceinline__ void load_slot(const uint64_t* slots, uint64_t s, uint64_t& w0,
                                          uint64_t& w1) {
    if (W == 2) {
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(slots + 2 * s);
        w0 = v.x;
        w1 = v.y;
    } else {
        w0 = slots[s];
        w1 = 0;
    }
}

// ---- record loads straight from global memory (aligned 16-B loads, parse in registers) ----
// Record parse straight from global memory, no LDS staging (records of R <= 16 bytes, K <= 56):
// lane i loads the aligned 16-B chunk holding record i's first byte and, when the record runs
// past it, the next one; the 15-B record is funnel-shifted out of the 32-B window in registers.
// Consecutive lanes read overlapping chunks, so a wave's loads coalesce into ~R*64/16 requests.
__device__ __forceinline__ uint64_t funnel64(uint64_t lo, uint64_t hi, uint32_t sh) {  // sh in [0,64)
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

__device__ __forceinline__ void load_record_regs(const uint8_t* __restrict__ recs, uint64_t i, uint32_t R,
                                                 uint64_t& x0, uint64_t& x1) {
    const uint64_t a = i * R;
    const uint32_t o = (uint32_t)(a & 15u);
    const ulonglong2 c0 = *reinterpret_cast<const ulonglong2*>(recs + (a - o));
    ulonglong2 c1 = make_ulonglong2(0, 0);
    if (o + R > 16u) c1 = *reinterpret_cast<const ulonglong2*>(recs + (a - o) + 16);
    uint64_t w0 = c0.x, w1 = c0.y, w2 = c1.x;
    if (o >= 8u) {
        w0 = w1;
        w1 = w2;
        w2 = c1.y;
    }
    const uint32_t sh = (o & 7u) * 8u;
    x0 = funnel64(w0, w1, sh);
    x1 = funnel64(w1, w2, sh);
}

// bytes 0..15 of a record (little-endian in x0, x1) -> key and extension codes (parse_record)
__device__ __forceinline__ void parse_record_regs(uint64_t x0, uint64_t x1, const KParams& p, Key& k,
                                                  uint32_t& ext) {
    const unsigned __int128 be = ((unsigned __int128)__builtin_bswap64(x0) << 64) | __builtin_bswap64(x1);
    const unsigned __int128 B = (be >> (8 * (16 - p.P))) >> (2 * p.pad);
    k.lo = (uint64_t)B & LO_MASK;
    k.hi = (uint64_t)(B >> 62);
    const unsigned __int128 xx = ((unsigned __int128)x1 << 64) | x0;
    const uint32_t e = (uint32_t)(xx >> (8 * p.P)) & 0xFFFFu;
    ext = base_code((uint8_t)e) | (base_code((uint8_t)(e >> 8)) << 3);
}

// Probe load of a read-only table with the non-temporal hint, for walkers that read whole 64-B
// blocks (a random block of a multi-GB table is not re-read before eviction; C3 walk 6.00 ->
// 5.72 ms). Slot-by-slot probing keeps plain loads: its next probe reads the same line (the
// migrating walker with the hint: 5.9 -> 7.6 ms).
template <int W>
__device__ __forceinline__ void load_slot_nt(const uint64_t* slots, uint64_t s, uint64_t& w0, uint64_t& w1) {
    if (W == 2) {
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        const u64x2 v = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(slots + 2 * s));
        w0 = v.x;
        w1 = v.y;
    } else {
        w0 = __builtin_nontemporal_load(slots + s);
        w1 = 0;
    }
}

// w0: the slot's word0 (may carry j*); home: its home slot (home_of)
template <int W>
__device__ __forceinline__ void insert_one(Key k, unsigned long long w0, uint64_t home, const KParams& p,
                                           uint64_t* slots, uint64_t cap, unsigned long long* stats) {
    unsigned long long* S = reinterpret_cast<unsigned long long*>(slots);
    const unsigned long long w1 = k.lo;
    const uint64_t want0 = slot_keybits(w0, p);
    uint64_t s = home;
    uint64_t probes = 0;
    uint32_t spins = 0;
    uint64_t c0, c1;
    load_slot<W>(slots, s, c0, c1);
    while (true) {
        if (c0 == EMPTY) {
            const unsigned long long old = atomicCAS(&S[W * s], (unsigned long long)EMPTY, w0);
            if (old == EMPTY) {
                if (W == 2)
                    __hip_atomic_store(&S[2 * s + 1], w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
            c0 = old;
            c1 = EMPTY;  // unknown: re-read coherently below if needed
        }
        if (slot_keybits(c0, p) == want0) {
            if (W == 1) {
                atomicAdd(&stats[ST_DUP], 1ull);
                return;
            }
            if (c1 == EMPTY)
                c1 = atomicCAS(&S[2 * s + 1], (unsigned long long)EMPTY, (unsigned long long)EMPTY);
            if (c1 == EMPTY) {
                if (++spins > (1u << 26)) {
                    atomicAdd(&stats[ST_SPIN], 1ull);
                    return;
                }
                continue;  // word1 not yet published: re-read it on the next iteration
            }
            if (c1 == w1) {
                atomicAdd(&stats[ST_DUP], 1ull);
                return;
            }
        }
        if (++probes >= cap) {
            atomicAdd(&stats[ST_FULL], 1ull);
            return;
        }
        s = (s + 1 == cap) ? 0 : s + 1;
        load_slot<W>(slots, s, c0, c1);
    }
}

// Probe: returns true and the slot's word0 if the key is present. Table is read-only here
// (written by an earlier kernel), so plain 8/16-byte loads are coherent. Both words feed the
// hit test unconditionally so the compiler keeps ONE dwordx4 per probe (a short-circuit on
// word0 made it split the slot into two dependent dwordx2 round trips).
template <int W>
__device__ __forceinline__ bool probe(Key k, const KParams& p, const uint64_t* __restrict__ slots,
                                      uint64_t cap, uint64_t& w0_out) {
    uint64_t s = home_of(place(k, p), cap, p);
    const uint64_t want0 = (W == 1) ? k.lo : k.hi;
    for (uint64_t probes = 0; probes < cap; ++probes) {
        uint64_t w0, w1;
        load_slot<W>(slots, s, w0, w1);
        const bool empty = w0 == EMPTY;
        const bool hit = !empty & (slot_keybits(w0, p) == want0) & ((W == 1) | (w1 == k.lo));
        if (hit | empty) {
            w0_out = w0;
            return hit;
        }
        s = (s + 1 == cap) ? 0 : s + 1;
    }
    return false;
}

// ---------------------------------------------------------------------------------------------
// Characters are produced 4 at a time (little-endian u32) and stored as aligned dwords: the
// leading/trailing bytes of a run that does not start/end on a dword boundary are byte stores,
// the inside is funnel-shifted (alignbyte) whole dwords. Byte-per-char stores made the two
// materialisation kernels ~1 ms at C3 (296 MB of text).
__device__ __forceinline__ uint32_t codes4_chars(uint32_t c8) {  // 4 2-bit codes, code 0 in bits 0-1
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) r |= ((0x54474341u >> (8 * ((c8 >> (2 * b)) & 3u))) & 0xFFu) << (8 * b);
    return r;
}

template <class Gen>
__device__ __forceinline__ void store_chars(char* dst, uint32_t n, Gen gen) {
    const uint32_t a = (4u - (uint32_t)((uintptr_t)dst & 3u)) & 3u;
    uint32_t cur = gen(0);
    const uint32_t lead = a < n ? a : n;
    for (uint32_t b = 0; b < lead; ++b) dst[b] = (char)(cur >> (8 * b));
    if (n <= a) return;
    uint32_t i = 0;
    for (; a + 4 * i + 4 <= n; ++i) {
        const uint32_t nxt = gen(i + 1);
        const uint32_t v = a ? __builtin_amdgcn_alignbyte(nxt, cur, a) : cur;
        *reinterpret_cast<uint32_t*>(dst + a + 4 * i) = v;
        cur = nxt;
    }
    for (uint32_t x = a + 4 * i; x < n; ++x) dst[x] = (char)(gen(x >> 2) >> (8 * (x & 3)));
}

// ---------------------------------------------------------------------------------------------
// Owner-major view of a [blocks][ranks] histogram for the exclusive scan.
struct HistF {
    const uint64_t* hist;
    uint64_t nb;
    uint32_t P;
    __device__ uint64_t operator()(uint64_t i) const { return hist[(i % nb) * P + i / nb]; }
};

template <int Unused = 0>
__global__ void k_route_counts(const uint64_t* off, uint64_t nb, uint32_t P,
                               const unsigned long long* total, uint64_t* counts) {
    const uint32_t q = threadIdx.x;
    if (q < P) {
        const uint64_t a = off[(uint64_t)q * nb];
        const uint64_t b = (q + 1 < P) ? off[(uint64_t)(q + 1) * nb] : (uint64_t)*total;
        counts[q] = b - a;
    }
    if (q == 0) counts[P] = (uint64_t)*total;
}

// Generic two-kernel owner grouping. Op must provide:
//   int owner(uint64_t i)             -> rank in [0,P) or -1 to skip (read-only)
//   void emit(uint64_t i, int q, uint64_t dst)   (may mutate per-item state; called once)
template <class Op>
__global__ __launch_bounds__(BLOCK) void k_group_hist(Op op, uint64_t n, uint32_t P, uint64_t* hist) {
    __shared__ uint32_t h[MAX_RANKS];
    for (uint32_t q = threadIdx.x; q < P; q += BLOCK) h[q] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * ROUTE_TILE;
    for (uint32_t j = threadIdx.x; j < ROUTE_TILE; j += BLOCK) {
        const uint64_t i = b0 + j;
        if (i < n) {
            const int q = op.owner(i);
            if (q >= 0) atomicAdd(&h[q], 1u);
        }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < P; q += BLOCK) hist[(uint64_t)blockIdx.x * P + q] = h[q];
}

template <class Op>
__global__ __launch_bounds__(BLOCK) void k_group_scatter(Op op, uint64_t n, uint32_t P,
                                                         const uint64_t* off, uint64_t nb) {
    __shared__ uint32_t h[MAX_RANKS];
    for (uint32_t q = threadIdx.x; q < P; q += BLOCK) h[q] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * ROUTE_TILE;
    for (uint32_t j = threadIdx.x; j < ROUTE_TILE; j += BLOCK) {
        const uint64_t i = b0 + j;
        int q = -1;
        if (i < n) q = op.owner(i);
        uint64_t dst = 0;
        if (q >= 0) dst = off[(uint64_t)q * nb + blockIdx.x] + atomicAdd(&h[q], 1u);
        if (i < n) op.emit(i, q, dst);
    }
}

template <class Op>
static inline hipError_t group_by_owner(Op op, uint64_t n, uint32_t P, uint64_t* hist, uint64_t* off,
                                 uint64_t* scratch, uint64_t* counts, unsigned long long* total,
                                 hipStream_t s) {
    const uint64_t nb = route_blocks(n);
    if (nb == 0) {
        hipError_t e = hipMemsetAsync(counts, 0, (P + 1) * 8, s);
        return e;
    }
    k_group_hist<Op><<<(unsigned)nb, BLOCK, 0, s>>>(op, n, P, hist);
    hipError_t e = scan_exclusive(HistF{hist, nb, P}, nb * P, off, scratch,
                                  (unsigned long long*)nullptr, total, s);
    if (e != hipSuccess) return e;
    k_route_counts<0><<<1, MAX_RANKS, 0, s>>>(off, nb, P, total, counts);
    k_group_scatter<Op><<<(unsigned)nb, BLOCK, 0, s>>>(op, n, P, off, nb);
    return hipGetLastError();
}

// multiprocessor count of the current device (per device: tables on several GPUs in one process)
inline int cu_count() {
    static int ncu[64] = {0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return 256;
    int v = __atomic_load_n(&ncu[dev], __ATOMIC_RELAXED);
    if (!v) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        __atomic_store_n(&ncu[dev], v, __ATOMIC_RELAXED);
    }
    return v;
}

}  // namespace kh
