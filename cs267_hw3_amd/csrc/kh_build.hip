// kh_build.hip — atomic-free bulk build of the open-addressing k-mer table (gfx950).
//
// Replaces one-CAS-per-key global inserts (bound at ~20 G random CAS/s on MI355X, measured by
// tools/membench) with streaming passes:
//   pass 1   group the batch by the top 9 bits of key_hash         512 bins
//   pass 2   then by the next 8 bits, within each pass-1 bucket     256 bins
//            (per-block LDS histograms + one exclusive scan per pass; each 4096-item tile is
//             counting-sorted by bin in LDS first so waves write contiguous runs)
//   build    one workgroup per region (top 17 hash bits) builds its slot range (~cap/2^17 slots,
//            ~49 KB at 200M k-mers) in LDS with LDS CAS linear probing, then writes the slice
//            out with coalesced 16-B stores
//   overflow keys whose probe run leaves their slice take the global CAS path afterwards, so
//            every key satisfies the linear-probing invariant "all slots from home to position
//            are occupied"
// Placement differs from the CAS path; find()/the walk depend only on the invariant, so outputs
// are identical (tests run both paths).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "kh_device.hpp"

namespace kh {

static constexpr int PB = 256;                    // threads per radix block
static constexpr int PITEMS = PART_TILE / PB;     // inputs per thread per tile (16)
static constexpr int B1 = 9, B2 = 8;              // radix bits per pass
static constexpr int NB1 = 1 << B1, NB2 = 1 << B2;
static constexpr int RBITS = B1 + B2;             // region = top 17 hash bits
static constexpr uint32_t NREG = 1u << RBITS;
static constexpr int BUILD_THREADS = 512;
static constexpr int T1 = 2;                      // consecutive tiles per pass-1 block
static constexpr uint32_t S1 = 8;                 // pass-1 windows (atomic counters) per bucket
static constexpr uint32_t NW1 = NB1 * S1;
// splitter buffer of k_win1 in the dynamic-LDS tail: (4 KB - 2 KB gpos - wsum - counter) / 16 B
static constexpr uint32_t WIN_SPLIT_LCAP = 120;
static_assert(PART_TILE * 18 + 3 * 512 * 4 + 8 + WIN_SPLIT_LCAP * 16 + 8 <= PART_TILE * 16 + PART_TILE * 2 + 512 * 16,
              "k_win1 LDS tail");
static constexpr uint64_t LDS_BYTES = 160 * 1024;
// radix-pass LDS: sorted items (2 words) + bin ids + hist/start (u32) + per-bin bases (u64) = 80 KiB
static constexpr size_t SORT_LDS = (size_t)PART_TILE * 16 + PART_TILE * 2 + 2 * NB1 * 4 + NB1 * 8;
// the windowed passes (k_win1 / k_win2) sort tiles of WIN_TILE words: 8192 doubles the runs each
// bin gets per tile (C3 pass 1: 16 words = 256 B instead of 128 B) in 152 KiB of LDS
static constexpr int WIN_TILE = 8192;
constexpr size_t sort_lds(int tile) { return (size_t)tile * 16 + tile * 2 + 2 * NB1 * 4 + NB1 * 8; }
static_assert(sort_lds(WIN_TILE) + 64 <= 160 * 1024, "k_win LDS");
static int win_tile() {
    const char* e = getenv("KH_WTILE");
    return (e && *e) ? atoi(e) : WIN_TILE;
}
static uint64_t win_blocks1(uint64_t n, int tile) { return (n + (uint64_t)T1 * tile - 1) / ((uint64_t)T1 * tile); }
static uint64_t win_G(uint64_t n, int tile) {
    const uint64_t tiles_per_bucket = (n / NB1 + tile - 1) / tile + 1;
    return (tiles_per_bucket + 1) / 2;
}

PartPlan part_plan(uint64_t n) {
    PartPlan pl;
    pl.n = n;
    pl.nb1 = (n + (uint64_t)T1 * PART_TILE - 1) / ((uint64_t)T1 * PART_TILE);
    const uint64_t tiles_per_bucket = (n / NB1 + PART_TILE - 1) / PART_TILE + 1;
    pl.G = (tiles_per_bucket + 1) / 2;
    if (pl.G < 1) pl.G = 1;
    return pl;
}

uint64_t part_hist_words(const PartPlan& pl) {
    const uint64_t a = pl.nb1 * NB1, b = (uint64_t)NB1 * NB2 * pl.G;
    return (a > b ? a : b) + 1;
}

uint64_t part_scratch_words(const PartPlan& pl) { return scan_scratch_words(part_hist_words(pl)) + 2; }

uint64_t part_overflow_cap(uint64_t n) { return n / 4 + 65536; }

uint32_t part_region_cap(uint64_t n) {
    const double mu = (double)n / NREG;
    return (uint32_t)(mu + 10.0 * sqrt(mu) + 16.0);
}

uint32_t part_win1_cap(uint64_t n) {
    const double mu = (double)n / NW1;
    return (uint32_t)(mu + 10.0 * sqrt(mu) + 64.0);
}

uint64_t part_buf1_words(const KParams& p, uint64_t n) {
    const uint64_t w = (uint64_t)NW1 * part_win1_cap(n);
    return (w > n ? w : n) * p.W;
}

uint64_t part_buf2_words(const KParams& p, uint64_t n) {
    const uint64_t w = (uint64_t)NREG * part_region_cap(n);
    return (w > n ? w : n) * p.W;
}

// Pass-1 / pass-2 variants (KH_P1 = convert | rec, KH_P2 = scan | res); defaults below.
// Pass-1 variant (KH_P1): 0 fused = k_part1_fused (windows + atomics, no histogram pass),
// 1 convert = records -> words + histogram, then the exact scatter (words input: histogram +
// scatter), 2 rec = histogram and scatter both parse the records, 3 direct = record parse from
// registers inside the windowed pass, 4 convfused = records -> words (k_part1_convert without
// its histogram) then the windowed pass on the words. Defaults (C3, MI355X): records ->
// convfused (1.45 + 1.91 ms; convert 1.45 + scans 0.42 + scatter 2.09; fused/direct parse in
// the sort kernel 5.5-5.7); 5 recwin = the windowed pass reading the records itself (coalesced
// 16-B blocks, records gathered by cross-lane shuffles; k with 13 or 5 packed bytes, else 4):
// 2.56 ms vs 1.21 + 1.65-1.82 at C3, the default for records; words -> fused.
static int p1_mode(bool rec) {
    const char* e = getenv("KH_P1");
    if (!e || !*e) return rec ? 5 : 0;
    if (!strcmp(e, "fused")) return 0;
    if (!strcmp(e, "direct")) return 3;
    if (!strcmp(e, "convfused")) return 4;
    if (!strcmp(e, "recwin")) return 5;
    return !strcmp(e, "rec") ? 2 : 1;
}
static bool p2_res() {
    const char* e = getenv("KH_P2");
    return e ? !strcmp(e, "res") : true;
}

static uint64_t region_max_slots(uint64_t cap) { return cap / NREG + 1; }

bool region_slots_fit(const KParams& p, uint64_t cap) {
    return region_max_slots(cap) <= LDS_BYTES / (8ull * p.W);
}

bool part_usable(const KParams& p, uint64_t cap, uint64_t n) {
    return n >= (1ull << 20) && region_slots_fit(p, cap) && cap >= (uint64_t)NREG * 8;
}

template <int W>
__device__ __forceinline__ uint64_t words_hash(uint64_t w0, uint64_t w1, const KParams& p) {
    return key_hash(slot_key(w0, w1, p));
}

// ---- tile loading -------------------------------------------------------------------------------
// Loads up to PART_TILE inputs starting at `base` into registers (item j of thread t is input
// base + j*PB + t). Records are staged through LDS CH at a time (`stage` >= CH*R bytes): every
// thread issues its 16-B loads for the whole chunk at once, so a chunk costs one memory latency;
// start bits are ballot-written to start_mask when given.
template <int W, bool REC, int CH>
__device__ __forceinline__ void load_tile(const KParams& p, const uint8_t* recs, const uint64_t* words,
                                          uint64_t base, uint64_t end, uint64_t* start_mask,
                                          uint8_t* stage, uint64_t (&a)[PITEMS], uint64_t (&b)[PITEMS],
                                          uint64_t* split_mask = nullptr) {
    if (REC) {
        constexpr int JPC = CH / PB;  // items per thread per chunk
#pragma unroll
        for (int c = 0; c < PITEMS / JPC; ++c) {
            const uint64_t cb = base + (uint64_t)c * CH;
            const uint32_t cnt = cb < end ? (uint32_t)min((uint64_t)CH, end - cb) : 0u;
            if (cnt) {  // uniform
                // all of this thread's 16-B loads in flight at once, then the LDS stores (a
                // load->store loop with a runtime trip count serialised one round trip per vector)
                constexpr int MAXV = (CH * 17 / 16 + PB - 1) / PB;
                const uint8_t* src = recs + cb * p.R;
                const uint32_t bytes = cnt * p.R, nvec = bytes >> 4;
                uint4 r[MAXV];
#pragma unroll
                for (int q = 0; q < MAXV; ++q) {
                    const uint32_t v = threadIdx.x + (uint32_t)q * PB;
                    if (v < nvec) r[q] = reinterpret_cast<const uint4*>(src)[v];
                }
                __syncthreads();
#pragma unroll
                for (int q = 0; q < MAXV; ++q) {
                    const uint32_t v = threadIdx.x + (uint32_t)q * PB;
                    if (v < nvec) reinterpret_cast<uint4*>(stage)[v] = r[q];
                }
                for (uint32_t x = (nvec << 4) + threadIdx.x; x < bytes; x += PB) stage[x] = src[x];
                __syncthreads();
            }
#pragma unroll
            for (int jj = 0; jj < JPC; ++jj) {
                const int j = c * JPC + jj;
                const uint32_t li = (uint32_t)jj * PB + threadIdx.x;  // index inside the chunk
                const bool valid = li < cnt;
                Key k{0, 0};
                uint32_t ext = 0;
                if (valid) parse_record(stage + li * p.R, p, k, ext);
                if (start_mask && cnt) {
                    const bool is_start = valid && ext_bwd(ext) == EXT_F;
                    const uint64_t bal = __ballot(is_start);
                    const uint64_t wb = cb + (uint64_t)jj * PB + (threadIdx.x & ~63u);
                    if ((threadIdx.x & 63) == 0 && wb < end) start_mask[wb >> 6] = bal;
                    if (split_mask) {
                        const uint64_t sb = __ballot(valid && !is_start && is_splitter(key_hash(k), p));
                        if ((threadIdx.x & 63) == 0 && wb < end) split_mask[wb >> 6] = sb;
                    }
                }
                a[j] = valid ? slot_w0(k, ext, p) : EMPTY;
                b[j] = (valid && W == 2) ? k.lo : 0;
            }
        }
        __syncthreads();
    } else {
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) {
            const uint64_t i = base + (uint64_t)j * PB + threadIdx.x;
            a[j] = EMPTY;
            b[j] = 0;
            if (i < end) {
                a[j] = words[i * W];
                b[j] = (W == 2) ? words[i * W + 1] : 0;
            }
        }
    }
}

// Item j of thread t = words[base + j*PB + t] (EMPTY past end): 16-B loads, fully coalesced.
// Loads are unconditional (index clamped to `last`, a valid index of the buffer) and the value
// selected afterwards, so all PITEMS loads issue back to back without branches or waits.
template <int W>
__device__ __forceinline__ void load_words(const uint64_t* __restrict__ words, uint64_t base, uint64_t end,
                                           uint64_t last, uint64_t (&a)[PITEMS], uint64_t (&b)[PITEMS]) {
#pragma unroll
    for (int j = 0; j < PITEMS; ++j) {
        const uint64_t i = base + (uint64_t)j * PB + threadIdx.x;
        const uint64_t ii = i < end ? i : last;
        uint64_t x0, x1 = 0;
        if (W == 2) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(words + 2 * ii);
            x0 = v.x;
            x1 = v.y;
        } else {
            x0 = words[ii];
        }
        a[j] = i < end ? x0 : EMPTY;
        b[j] = i < end ? x1 : 0;
    }
}

// Same from the S1 pass-1 windows of bucket bk (pre = window prefix sums): virtual index v.
template <int W>
__device__ __forceinline__ void load_words_win(const uint64_t* __restrict__ buf1, uint32_t bk, uint32_t CAP1,
                                               const uint32_t (&pre)[S1 + 1], uint64_t base, uint64_t end,
                                               uint64_t (&a)[PITEMS], uint64_t (&b)[PITEMS]) {
#pragma unroll
    for (int j = 0; j < PITEMS; ++j) {
        const uint32_t v = (uint32_t)(base + (uint64_t)j * PB + threadIdx.x);
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
            const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(buf1 + 2 * i);
            x0 = x.x;
            x1 = x.y;
        } else {
            x0 = buf1[i];
        }
        a[j] = ok ? x0 : EMPTY;
        b[j] = ok ? x1 : 0;
    }
}

// Block-wide exclusive scan of NB (<= 512) LDS counters into start[]; returns the total.
template <int NB>
__device__ __forceinline__ uint32_t scan_bins(const uint32_t* hist, uint32_t* start) {
    constexpr int PER = (NB + PB - 1) / PB;
    uint32_t v[PER];
    uint64_t s = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int i = threadIdx.x * PER + q;
        v[q] = i < NB ? hist[i] : 0;
        s += v[q];
    }
    uint64_t tot;
    uint64_t pre = block_excl_scan(s, tot);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const int i = threadIdx.x * PER + q;
        if (i < NB) start[i] = (uint32_t)pre;
        pre += v[q];
    }
    lds_barrier();
    return (uint32_t)tot;
}

// Counting-sort the tile's items by bin in LDS, then write them to out at gbase[bin] + rank
// (gbase in LDS), so consecutive lanes store consecutive addresses of one bin.
// sorted_write in two halves: sorted_place leaves the tile in LDS (a/b/bin dead afterwards, so a
// caller can issue the next tile's loads into them), sorted_out writes it and advances nothing.
template <int W, int NB>
__device__ __forceinline__ uint32_t sorted_place(const uint64_t (&a)[PITEMS], const uint64_t (&b)[PITEMS],
                                                 const uint32_t (&bin)[PITEMS], uint64_t* items,
                                                 uint16_t* sbin, uint32_t* hist, uint32_t* start) {
    for (int i = threadIdx.x; i < NB; i += PB) hist[i] = 0;
    lds_barrier();
    uint32_t rank[PITEMS];
#pragma unroll
    for (int j = 0; j < PITEMS; ++j) rank[j] = (a[j] != EMPTY) ? atomicAdd(&hist[bin[j]], 1u) : 0u;
    lds_barrier();
    const uint32_t total = scan_bins<NB>(hist, start);
#pragma unroll
    for (int j = 0; j < PITEMS; ++j) {
        if (a[j] != EMPTY) {
            const uint32_t pos = start[bin[j]] + rank[j];
            items[pos * W] = a[j];
            if (W == 2) items[pos * W + 1] = b[j];
            sbin[pos] = (uint16_t)bin[j];
        }
    }
    return total;
}

template <int W>
__device__ __forceinline__ void sorted_out(uint32_t total, const uint64_t* items, const uint16_t* sbin,
                                           const uint32_t* start, const uint64_t* gbase, uint64_t* out) {
#pragma unroll 4
    for (uint32_t t = threadIdx.x; t < total; t += PB) {
        const uint32_t q = sbin[t];
        const uint64_t g = gbase[q] + (t - start[q]);
        if (W == 2) {
            *reinterpret_cast<ulonglong2*>(out + g * 2) = make_ulonglong2(items[2 * t], items[2 * t + 1]);
        } else {
            out[g] = items[t];
        }
    }
}

template <int W, int NB>
__device__ __forceinline__ void sorted_write(const uint64_t (&a)[PITEMS], const uint64_t (&b)[PITEMS],
                                             const uint32_t (&bin)[PITEMS], uint64_t* items,
                                             uint16_t* sbin, uint32_t* hist, uint32_t* start,
                                             const uint64_t* gbase, uint64_t* out) {
    for (int i = threadIdx.x; i < NB; i += PB) hist[i] = 0;
    lds_barrier();
    uint32_t rank[PITEMS];
#pragma unroll
    for (int j = 0; j < PITEMS; ++j) rank[j] = (a[j] != EMPTY) ? atomicAdd(&hist[bin[j]], 1u) : 0u;
    lds_barrier();
    const uint32_t total = scan_bins<NB>(hist, start);
#pragma unroll
    for (int j = 0; j < PITEMS; ++j) {
        if (a[j] != EMPTY) {
            const uint32_t pos = start[bin[j]] + rank[j];
            items[pos * W] = a[j];
            if (W == 2) items[pos * W + 1] = b[j];
            sbin[pos] = (uint16_t)bin[j];
        }
    }
    lds_barrier();
    for (uint32_t t = threadIdx.x; t < total; t += PB) {
        const uint32_t q = sbin[t];
        const uint64_t g = gbase[q] + (t - start[q]);
        if (W == 2) {
            *reinterpret_cast<ulonglong2*>(out + g * 2) = make_ulonglong2(items[2 * t], items[2 * t + 1]);
        } else {
            out[g] = items[t];
        }
    }
    lds_barrier();
}

// ---- pass 1: bin = top 9 hash bits --------------------------------------------------------------
// Record input: parse the reference records once, one per thread per 256-record sub-tile (the next
// sub-tile's 16-B loads are in flight while this one is parsed), emit internal words in input
// order, count bins, and write the start bits. The pass-1 scatter then reads words only.
template <int PK>
__device__ __forceinline__ void parse_record_regs_t(uint64_t x0, uint64_t x1, int pad, Key& k, uint32_t& ext);

template <int W, int PK = 0>
__global__ __launch_bounds__(PB) void k_part1_convert(KParams p, const uint8_t* __restrict__ recs,
                                                      uint64_t n, uint64_t* words_out, uint64_t* hist1,
                                                      uint64_t* start_mask, uint64_t* split_mask) {
    __shared__ uint32_t h[NB1];
    __shared__ __attribute__((aligned(16))) uint8_t stage[2][PB * 17 + 16];
    for (int i = threadIdx.x; i < NB1; i += PB) h[i] = 0;
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
        const uint64_t hk = key_hash(k);
        if (split_mask) {
            const uint64_t sb = __ballot(valid && !is_start && is_splitter(hk, p));
            if ((threadIdx.x & 63) == 0 && wb < b1) split_mask[wb >> 6] = sb;
        }
        if (valid) {
            const uint64_t w0 = slot_w0(k, ext, p), i = sub + threadIdx.x;
            if (W == 2) {
                *reinterpret_cast<ulonglong2*>(words_out + i * 2) = make_ulonglong2(w0, k.lo);
            } else {
                words_out[i] = w0;
            }
            if (hist1) atomicAdd(&h[hk >> (64 - B1)], 1u);
        }
    }
    if (!hist1) return;  // words only (the windowed pass 1 needs no histogram)
    __syncthreads();
    for (int i = threadIdx.x; i < NB1; i += PB) hist1[(uint64_t)blockIdx.x * NB1 + i] = h[i];
}

// Pass 1 fused with the parse: one read of the records, no histogram pass, no word copy.
// Bucket b (top 9 hash bits) is S1 fixed windows of CAP1 words in buf1; block x writes to window
// x % S1 of each bucket, reserving its tile's run there with one atomicAdd per (tile, bucket).
// S1 counters per bucket keep each counter at ~1/S1 of the tiles (same-address device atomics
// serialise at the memory side). Records are staged 256 at a time through LDS (the
// next sub-tile's 16-B loads in flight while this one is parsed); items stay in registers until
// the tile is counting-sorted by bucket in LDS and written out as contiguous runs.
template <int W, bool REC>
__global__ __launch_bounds__(PB) void k_part1_fused(KParams p, const uint8_t* __restrict__ recs,
                                                    const uint64_t* __restrict__ words, uint64_t n,
                                                    uint32_t CAP1, uint32_t* wcnt, uint64_t* buf1,
                                                    uint64_t* start_mask, uint64_t* split_mask,
                                                    uint64_t* ovf, uint64_t ovf_cap,
                                                    unsigned long long* ctr, unsigned long long* stats) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;                                              // PART_TILE * 2 words
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + PART_TILE * 2);  // PART_TILE
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + PART_TILE);      // NB1
    uint32_t* start = hist + NB1;                                        // NB1
    uint32_t* gpos = start + NB1;                                        // NB1
    const uint32_t sub = blockIdx.x % S1;
    const uint32_t R = (uint32_t)p.R;
    for (int tt = 0; tt < T1; ++tt) {
        const uint64_t base = ((uint64_t)blockIdx.x * T1 + tt) * PART_TILE;
        if (base >= n) break;  // uniform
        const uint64_t end = min(base + (uint64_t)PART_TILE, n);
        uint64_t a[PITEMS], b[PITEMS];
        uint32_t bin[PITEMS];
        if (REC) {
            uint8_t* stage = reinterpret_cast<uint8_t*>(items);  // 2 x 256 records, aliases items
            uint4 r0 = make_uint4(0, 0, 0, 0), r1 = r0;
            auto fetch = [&](uint64_t s0) {
                if (s0 >= end) return;
                const uint32_t nvec = (uint32_t)(min((uint64_t)PB, end - s0) * R) >> 4;
                const uint4* src = reinterpret_cast<const uint4*>(recs + s0 * R);
                if (threadIdx.x < nvec) r0 = src[threadIdx.x];
                if (threadIdx.x + PB < nvec) r1 = src[threadIdx.x + PB];
            };
            fetch(base);
#pragma unroll
            for (int j = 0; j < PITEMS; ++j) {
                const uint64_t s0 = base + (uint64_t)j * PB;
                const uint32_t cnt = s0 < end ? (uint32_t)min((uint64_t)PB, end - s0) : 0u;
                const uint32_t bytes = cnt * R, nvec = bytes >> 4;
                uint8_t* st = stage + (j & 1) * (PB * MAX_R);
                if (threadIdx.x < nvec) reinterpret_cast<uint4*>(st)[threadIdx.x] = r0;
                if (threadIdx.x + PB < nvec) reinterpret_cast<uint4*>(st)[threadIdx.x + PB] = r1;
                for (uint32_t x = (nvec << 4) + threadIdx.x; x < bytes; x += PB) st[x] = recs[s0 * R + x];
                if (j + 1 < PITEMS) fetch(s0 + PB);
                lds_barrier();
                const bool valid = threadIdx.x < cnt;
                Key k{0, 0};
                uint32_t ext = 0;
                if (valid) parse_record(st + threadIdx.x * R, p, k, ext);
                const uint64_t hk = key_hash(k);
                if (cnt) {  // uniform
                    const bool is_start = valid && ext_bwd(ext) == EXT_F;
                    const uint64_t bal = __ballot(is_start);
                    const uint64_t sb = __ballot(valid && !is_start && is_splitter(hk, p));
                    const uint64_t wb = s0 + (threadIdx.x & ~63u);
                    if ((threadIdx.x & 63) == 0 && wb < end) {
                        if (start_mask) start_mask[wb >> 6] = bal;
                        if (split_mask) split_mask[wb >> 6] = sb;
                    }
                }
                a[j] = valid ? slot_w0(k, ext, p) : EMPTY;
                b[j] = (valid && W == 2) ? k.lo : 0;
                bin[j] = (uint32_t)(hk >> (64 - B1));
            }
            lds_barrier();  // stage reads done before the sort reuses the space
        } else {
#pragma unroll
            for (int j = 0; j < PITEMS; ++j) {
                const uint64_t i = base + (uint64_t)j * PB + threadIdx.x;
                a[j] = EMPTY;
                b[j] = 0;
                if (i < end) {
                    if (W == 2) {
                        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(words + 2 * i);
                        a[j] = v.x;
                        b[j] = v.y;
                    } else {
                        a[j] = words[i];
                    }
                }
                bin[j] = (uint32_t)(words_hash<W>(a[j], b[j], p) >> (64 - B1));
            }
        }
        for (int i = threadIdx.x; i < NB1; i += PB) hist[i] = 0;
        lds_barrier();
        uint32_t rank[PITEMS];
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) rank[j] = (a[j] != EMPTY) ? atomicAdd(&hist[bin[j]], 1u) : 0u;
        lds_barrier();
        const uint32_t total = scan_bins<NB1>(hist, start);
        for (int i = threadIdx.x; i < NB1; i += PB)
            gpos[i] = hist[i] ? atomicAdd(&wcnt[i * S1 + sub], hist[i]) : 0u;
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) {
            if (a[j] != EMPTY) {
                const uint32_t pos = start[bin[j]] + rank[j];
                items[pos * W] = a[j];
                if (W == 2) items[pos * W + 1] = b[j];
                sbin[pos] = (uint16_t)bin[j];
            }
        }
        lds_barrier();
        for (uint32_t x = threadIdx.x; x < total; x += PB) {
            const uint32_t q = sbin[x];
            const uint32_t w = gpos[q] + (x - start[q]);
            const uint64_t v0 = items[W * x], v1 = (W == 2) ? items[W * x + 1] : 0;
            if (w < CAP1) {
                const uint64_t g = (uint64_t)(q * S1 + sub) * CAP1 + w;
                if (W == 2) {
                    *reinterpret_cast<ulonglong2*>(buf1 + g * 2) = make_ulonglong2(v0, v1);
                } else {
                    buf1[g] = v0;
                }
            } else {
                const unsigned long long idx = atomicAdd(&ctr[CT_OVF], 1ull);
                if (idx < ovf_cap) {
                    ovf[idx * W] = v0;
                    if (W == 2) ovf[idx * W + 1] = v1;
                } else {
                    atomicAdd(&stats[ST_FULL], 1ull);
                }
            }
        }
        lds_barrier();
    }
}

// same with the packed size PK known at compile time: constant shifts, no SALU per record
template <int PK>
__device__ __forceinline__ void parse_record_regs_t(uint64_t x0, uint64_t x1, int pad, Key& k, uint32_t& ext) {
    const unsigned __int128 be = ((unsigned __int128)__builtin_bswap64(x0) << 64) | __builtin_bswap64(x1);
    const unsigned __int128 B = (be >> (8 * (16 - PK))) >> (2 * pad);
    k.lo = (uint64_t)B & LO_MASK;
    k.hi = (uint64_t)(B >> 62);
    const unsigned __int128 xx = ((unsigned __int128)x1 << 64) | x0;
    const uint32_t e = (uint32_t)(xx >> (8 * PK)) & 0xFFFFu;
    ext = base_code((uint8_t)e) | (base_code((uint8_t)(e >> 8)) << 3);
}

template <int W, int PK = 0>
__global__ __launch_bounds__(PB) void k_part1_direct(KParams p, const uint8_t* __restrict__ recs, uint64_t n,
                                                     uint32_t CAP1, uint32_t* wcnt, uint64_t* buf1,
                                                     uint64_t* start_mask, uint64_t* split_mask,
                                                     uint64_t* ovf, uint64_t ovf_cap,
                                                     unsigned long long* ctr, unsigned long long* stats) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;                                              // PART_TILE * 2 words
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + PART_TILE * 2);  // PART_TILE
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + PART_TILE);      // NB1
    uint32_t* start = hist + NB1;                                        // NB1
    uint32_t* gpos = start + NB1;                                        // NB1
    const uint32_t sub = blockIdx.x % S1;
    const uint32_t R = (uint32_t)p.R;
    for (int tt = 0; tt < T1; ++tt) {
        const uint64_t base = ((uint64_t)blockIdx.x * T1 + tt) * PART_TILE;
        if (base >= n) break;  // uniform
        uint64_t a[PITEMS], b[PITEMS];
        uint32_t bin[PITEMS];
        uint64_t x0[PITEMS], x1[PITEMS];
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) {
            const uint64_t i = base + (uint64_t)j * PB + threadIdx.x;
            x0[j] = x1[j] = 0;
            if (i < n) load_record_regs(recs, i, PK ? (uint32_t)(PK + 2) : R, x0[j], x1[j]);
        }
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) {
            const uint64_t s0 = base + (uint64_t)j * PB;
            const uint64_t i = s0 + threadIdx.x;
            const bool valid = i < n;
            Key k{0, 0};
            uint32_t ext = 0;
            if (valid) {
                if constexpr (PK != 0)
                    parse_record_regs_t<PK>(x0[j], x1[j], p.pad, k, ext);
                else
                    parse_record_regs(x0[j], x1[j], p, k, ext);
            }
            const uint64_t hk = key_hash(k);
            if (s0 < n) {  // uniform
                const bool is_start = valid && ext_bwd(ext) == EXT_F;
                const uint64_t bal = __ballot(is_start);
                const uint64_t sb = __ballot(valid && !is_start && is_splitter(hk, p));
                const uint64_t wb = s0 + (threadIdx.x & ~63u);
                if ((threadIdx.x & 63) == 0 && wb < n) {
                    if (start_mask) start_mask[wb >> 6] = bal;
                    if (split_mask) split_mask[wb >> 6] = sb;
                }
            }
            a[j] = valid ? slot_w0(k, ext, p) : EMPTY;
            b[j] = (valid && W == 2) ? k.lo : 0;
            bin[j] = (uint32_t)(hk >> (64 - B1));
        }
        for (int i = threadIdx.x; i < NB1; i += PB) hist[i] = 0;
        lds_barrier();
        uint32_t rank[PITEMS];
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) rank[j] = (a[j] != EMPTY) ? atomicAdd(&hist[bin[j]], 1u) : 0u;
        lds_barrier();
        const uint32_t total = scan_bins<NB1>(hist, start);
        for (int i = threadIdx.x; i < NB1; i += PB)
            gpos[i] = hist[i] ? atomicAdd(&wcnt[i * S1 + sub], hist[i]) : 0u;
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) {
            if (a[j] != EMPTY) {
                const uint32_t pos = start[bin[j]] + rank[j];
                items[pos * W] = a[j];
                if (W == 2) items[pos * W + 1] = b[j];
                sbin[pos] = (uint16_t)bin[j];
            }
        }
        lds_barrier();
#pragma unroll 4
        for (uint32_t x = threadIdx.x; x < total; x += PB) {
            const uint32_t q = sbin[x];
            const uint32_t w = gpos[q] + (x - start[q]);
            const uint64_t v0 = items[W * x], v1 = (W == 2) ? items[W * x + 1] : 0;
            if (w < CAP1) {
                const uint64_t g = (uint64_t)(q * S1 + sub) * CAP1 + w;
                if (W == 2) {
                    *reinterpret_cast<ulonglong2*>(buf1 + g * 2) = make_ulonglong2(v0, v1);
                } else {
                    buf1[g] = v0;
                }
            } else {
                const unsigned long long idx = atomicAdd(&ctr[CT_OVF], 1ull);
                if (idx < ovf_cap) {
                    ovf[idx * W] = v0;
                    if (W == 2) ovf[idx * W + 1] = v1;
                } else {
                    atomicAdd(&stats[ST_FULL], 1ull);
                }
            }
        }
        lds_barrier();
    }
}

template <int W, bool REC>
__global__ __launch_bounds__(PB) void k_part1_hist(KParams p, const uint8_t* recs, const uint64_t* words,
                                                   uint64_t n, uint64_t* hist1, uint64_t* start_mask,
                                                   uint64_t* split_mask) {
    __shared__ uint32_t h[NB1];
    __shared__ __attribute__((aligned(16))) uint8_t stage[REC ? 1024 * 17 : 16];
    for (int i = threadIdx.x; i < NB1; i += PB) h[i] = 0;
    __syncthreads();
    for (int tt = 0; tt < T1; ++tt) {
        const uint64_t base = ((uint64_t)blockIdx.x * T1 + tt) * PART_TILE;
        if (base >= n) break;  // uniform
        uint64_t a[PITEMS], b[PITEMS];
        load_tile<W, REC, 1024>(p, recs, words, base, min(base + PART_TILE, n), start_mask, stage, a, b,
                                split_mask);
#pragma unroll
        for (int j = 0; j < PITEMS; ++j)
            if (a[j] != EMPTY) atomicAdd(&h[words_hash<W>(a[j], b[j], p) >> (64 - B1)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NB1; i += PB) hist1[(uint64_t)blockIdx.x * NB1 + i] = h[i];
}

template <int W, bool REC>
__global__ __launch_bounds__(PB) void k_part1_scatter(KParams p, const uint8_t* recs,
                                                      const uint64_t* words, uint64_t n,
                                                      const uint64_t* off1, uint64_t nb1,
                                                      uint64_t* buf1) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;                                              // PART_TILE * 2 words
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + PART_TILE * 2);  // PART_TILE
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + PART_TILE);      // NB1
    uint32_t* start = hist + NB1;                                        // NB1
    uint64_t* gbase = reinterpret_cast<uint64_t*>(start + NB1);          // NB1 (8-B aligned)
    for (int i = threadIdx.x; i < NB1; i += PB) gbase[i] = off1[(uint64_t)blockIdx.x * NB1 + i];
    __syncthreads();
    if (!REC) {
        // words: the next tile's loads are issued before this tile is sorted and written, and
        // tiles are separated by LDS-only barriers, so loads, LDS work and stores overlap
        uint64_t a[PITEMS], b[PITEMS];
        const uint64_t b0 = (uint64_t)blockIdx.x * T1 * PART_TILE;
        load_words<W>(words, b0, min(b0 + PART_TILE, n), b0 < n ? b0 : 0, a, b);
        for (int tt = 0; tt < T1; ++tt) {
            const uint64_t base = b0 + (uint64_t)tt * PART_TILE;
            if (base >= n) break;  // uniform
            uint32_t bin[PITEMS];
#pragma unroll
            for (int j = 0; j < PITEMS; ++j) bin[j] = (uint32_t)(words_hash<W>(a[j], b[j], p) >> (64 - B1));
            const uint32_t total = sorted_place<W, NB1>(a, b, bin, items, sbin, hist, start);
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t nbase = base + PART_TILE;
            load_words<W>(words, nbase, (tt + 1 < T1) ? min(nbase + PART_TILE, n) : nbase, base, a, b);
            lds_barrier();
            sorted_out<W>(total, items, sbin, start, gbase, buf1);
            lds_barrier();
            for (int i = threadIdx.x; i < NB1; i += PB) gbase[i] += hist[i];
            lds_barrier();
        }
        return;
    }
    for (int tt = 0; tt < T1; ++tt) {
        const uint64_t base = ((uint64_t)blockIdx.x * T1 + tt) * PART_TILE;
        if (base >= n) break;  // uniform
        uint64_t a[PITEMS], b[PITEMS];
        load_tile<W, REC, PART_TILE>(p, recs, words, base, min(base + PART_TILE, n), nullptr,
                                     reinterpret_cast<uint8_t*>(items), a, b);
        uint32_t bin[PITEMS];
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) bin[j] = (uint32_t)(words_hash<W>(a[j], b[j], p) >> (64 - B1));
        sorted_write<W, NB1>(a, b, bin, items, sbin, hist, start, gbase, buf1);
        for (int i = threadIdx.x; i < NB1; i += PB) gbase[i] += hist[i];
        __syncthreads();
    }
}

// pass-1 offsets stored block-major: [block][bin]
struct Off1Idx {
    uint64_t nb;
    __device__ uint64_t operator()(uint64_t i) const { return (i % nb) * NB1 + i / nb; }
};

struct Hist1F {
    const uint64_t* hist;
    uint64_t nb;
    __device__ uint64_t operator()(uint64_t i) const { return hist[(i % nb) * NB1 + i / nb]; }
};

// ---- pass 2: bin = next 8 hash bits, within each pass-1 bucket ----------------------------------
// bucket b starts at the offset of (block 0, bin b) = off1[b] in the block-major layout
__device__ __forceinline__ void bucket_range(const uint64_t* off1, uint64_t nb1, uint64_t n, uint32_t b,
                                             uint64_t& s, uint64_t& e) {
    (void)nb1;
    s = off1[b];
    e = (b + 1 < (uint32_t)NB1) ? off1[b + 1] : n;
}

template <int W>
__global__ __launch_bounds__(PB) void k_part2_hist(KParams p, const uint64_t* buf1, uint64_t n,
                                                   const uint64_t* off1, uint64_t nb1, uint64_t G,
                                                   uint64_t* hist2) {
    __shared__ uint32_t h[NB2];
    for (int i = threadIdx.x; i < NB2; i += PB) h[i] = 0;
    __syncthreads();
    const uint32_t bk = blockIdx.x / (uint32_t)G, g = blockIdx.x % (uint32_t)G;
    uint64_t s, e;
    bucket_range(off1, nb1, n, bk, s, e);
    for (uint64_t t = s + (uint64_t)g * PART_TILE; t < e; t += G * PART_TILE) {
        uint64_t a[PITEMS], b[PITEMS];
        load_tile<W, false, PART_TILE>(p, nullptr, buf1, t, min(t + PART_TILE, e), nullptr, nullptr, a, b);
#pragma unroll
        for (int j = 0; j < PITEMS; ++j)
            if (a[j] != EMPTY)
                atomicAdd(&h[(words_hash<W>(a[j], b[j], p) >> (64 - RBITS)) & (NB2 - 1)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NB2; i += PB) hist2[(uint64_t)blockIdx.x * NB2 + i] = h[i];
}

template <int W>
__global__ __launch_bounds__(PB) void k_part2_scatter(KParams p, const uint64_t* buf1, uint64_t n,
                                                      const uint64_t* off1, uint64_t nb1, uint64_t G,
                                                      const uint64_t* off2, uint64_t* buf2) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + PART_TILE * 2);
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + PART_TILE);
    uint32_t* start = hist + NB1;
    uint64_t* gbase = reinterpret_cast<uint64_t*>(start + NB1);
    const uint32_t bk = blockIdx.x / (uint32_t)G, g = blockIdx.x % (uint32_t)G;
    uint64_t s, e;
    bucket_range(off1, nb1, n, bk, s, e);
    for (int i = threadIdx.x; i < NB2; i += PB) gbase[i] = off2[((uint64_t)bk * G + g) * NB2 + i];
    __syncthreads();
    for (uint64_t t = s + (uint64_t)g * PART_TILE; t < e; t += G * PART_TILE) {
        uint64_t a[PITEMS], b[PITEMS];
        load_tile<W, false, PART_TILE>(p, nullptr, buf1, t, min(t + PART_TILE, e), nullptr, nullptr, a, b);
        uint32_t bin[PITEMS];
#pragma unroll
        for (int j = 0; j < PITEMS; ++j)
            bin[j] = (uint32_t)(words_hash<W>(a[j], b[j], p) >> (64 - RBITS)) & (NB2 - 1);
        sorted_write<W, NB2>(a, b, bin, items, sbin, hist, start, gbase, buf2);
        // advance the running per-bin bases by this tile's counts (hist still holds them)
        for (int i = threadIdx.x; i < NB2; i += PB) gbase[i] += hist[i];
        __syncthreads();
    }
}

// Pass 2 without a histogram pass: region r owns a fixed window of RC words of buf2
// ([r*RC, r*RC + RC)); each tile counting-sorts its items by region in LDS and reserves its run in
// every region it touches with ONE atomicAdd on that region's counter (256 per 4096-item tile,
// ~95 per counter at C3, no hot address). Items past a full window go to the overflow list (the
// global CAS path); RC = mean + 10 sigma + 16, so that never happens on hashed keys.
template <int W, bool WIN>
__global__ __launch_bounds__(PB) void k_part2_res(KParams p, const uint64_t* buf1, uint64_t n,
                                                  const uint64_t* off1, uint64_t G, uint32_t RC,
                                                  uint32_t* rcnt, uint64_t* buf2, uint64_t* ovf,
                                                  uint64_t ovf_cap, unsigned long long* ctr,
                                                  unsigned long long* stats, uint32_t CAP1,
                                                  const uint32_t* wcnt) {
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + PART_TILE * 2);
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + PART_TILE);
    uint32_t* start = hist + NB1;
    uint32_t* gpos = start + NB1;  // reserved position of this tile's run in each region window
    const uint32_t bk = blockIdx.x / (uint32_t)G, g = blockIdx.x % (uint32_t)G;
    uint64_t s, e;
    // bucket bk = the S1 windows of k_part1_fused (CAP1 != 0), concatenated, or a contiguous range
    uint32_t pre[S1 + 1];
    if (WIN) {
        pre[0] = 0;
#pragma unroll
        for (uint32_t j = 0; j < S1; ++j) pre[j + 1] = pre[j] + min(wcnt[bk * S1 + j], CAP1);
        s = 0;
        e = pre[S1];
    } else {
        bucket_range(off1, 0, n, bk, s, e);
    }
    uint64_t a[PITEMS], b[PITEMS];
#define KH_P2_LOAD(t)                                                                              \
    do {                                                                                           \
        const uint64_t t_ = (t);                                                                   \
        const uint64_t e_ = t_ < e ? min(t_ + PART_TILE, e) : t_;                                  \
        if (WIN)                                                                                   \
            load_words_win<W>(buf1, bk, CAP1, pre, t_, e_, a, b);                                  \
        else                                                                                       \
            load_words<W>(buf1, t_, e_, s, a, b);                                                  \
    } while (0)
    KH_P2_LOAD(s + (uint64_t)g * PART_TILE);
    for (uint64_t t = s + (uint64_t)g * PART_TILE; t < e; t += G * PART_TILE) {
        uint32_t bin[PITEMS];
#pragma unroll
        for (int j = 0; j < PITEMS; ++j)
            bin[j] = (uint32_t)(words_hash<W>(a[j], b[j], p) >> (64 - RBITS)) & (NB2 - 1);
        for (int i = threadIdx.x; i < NB2; i += PB) hist[i] = 0;
        lds_barrier();
        uint32_t rank[PITEMS];
#pragma unroll
        for (int j = 0; j < PITEMS; ++j) rank[j] = (a[j] != EMPTY) ? atomicAdd(&hist[bin[j]], 1u) : 0u;
        lds_barrier();
        const uint32_t total = scan_bins<NB2>(hist, start);
        for (int i = threadIdx.x; i < NB2; i += PB)
            gpos[i] = hist[i] ? atomicAdd(&rcnt[(bk << B2) | i], hist[i]) : 0u;

#pragma unroll
        for (int j = 0; j < PITEMS; ++j) {
            if (a[j] != EMPTY) {
                const uint32_t pos = start[bin[j]] + rank[j];
                items[pos * W] = a[j];
                if (W == 2) items[pos * W + 1] = b[j];
                sbin[pos] = (uint16_t)bin[j];
            }
        }
        __builtin_amdgcn_sched_barrier(0);  // keep the next tile's loads below the placement
        KH_P2_LOAD(t + G * PART_TILE);  // next tile in flight while this one is written
        lds_barrier();
#pragma unroll 4
        for (uint32_t x = threadIdx.x; x < total; x += PB) {
            const uint32_t q = sbin[x];
            const uint32_t w = gpos[q] + (x - start[q]);
            const uint64_t v0 = items[W * x], v1 = (W == 2) ? items[W * x + 1] : 0;
            if (w < RC) {
                const uint64_t gidx = (uint64_t)((bk << B2) | q) * RC + w;
                if (W == 2) {
                    *reinterpret_cast<ulonglong2*>(buf2 + gidx * 2) = make_ulonglong2(v0, v1);
                } else {
                    buf2[gidx] = v0;
                }
            } else {
                const unsigned long long idx = atomicAdd(&ctr[CT_OVF], 1ull);
                if (idx < ovf_cap) {
                    ovf[idx * W] = v0;
                    if (W == 2) ovf[idx * W + 1] = v1;
                } else {
                    atomicAdd(&stats[ST_FULL], 1ull);
                }
            }
        }
        lds_barrier();
    }
}
#undef KH_P2_LOAD

// pass-2 offsets stored [bucket][block-in-bucket][bin]
struct Off2Idx {
    uint32_t G;
    __device__ uint64_t operator()(uint64_t i) const {
        const uint32_t x = (uint32_t)i, per = (uint32_t)NB2 * G;
        const uint32_t bk = x / per, rem = x % per, f = rem / G, g = rem % G;
        return ((uint64_t)bk * G + g) * NB2 + f;
    }
};

// order (pass-1 bucket, pass-2 bin, block-in-bucket)
struct Hist2F {
    const uint64_t* hist;
    uint32_t G;
    __device__ uint64_t operator()(uint64_t i) const {
        const uint32_t x = (uint32_t)i, per = (uint32_t)NB2 * G;
        const uint32_t bk = x / per, rem = x % per, f = rem / G, g = rem % G;
        return hist[((uint64_t)bk * G + g) * NB2 + f];
    }
};

// ---- build ------------------------------------------------------------------------------------
// LDS insert with linear probing inside the slice; false = the run left the slice.
template <int W>
__device__ __forceinline__ bool lds_insert(unsigned long long* lt, uint32_t S, uint64_t loc, uint64_t w0,
                                           uint64_t w1, unsigned long long* stats) {
    uint32_t spins = 0;
    while (loc < S) {
        const unsigned long long old = atomicCAS(&lt[W * loc], (unsigned long long)EMPTY, w0);
        if (old == EMPTY) {
            if (W == 2)
                __hip_atomic_store(&lt[2 * loc + 1], (unsigned long long)w1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            return true;
        }
        if ((old >> 6) == (w0 >> 6)) {
            if (W == 1) {
                atomicAdd(&stats[ST_DUP], 1ull);
                return true;
            }
            const unsigned long long o1 =
                __hip_atomic_load(&lt[2 * loc + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (o1 == EMPTY) {  // the claiming lane has not stored word1 yet: retry this slot
                if (++spins > (1u << 24)) {
                    atomicAdd(&stats[ST_SPIN], 1ull);
                    return true;
                }
                continue;
            }
            if (o1 == w1) {
                atomicAdd(&stats[ST_DUP], 1ull);
                return true;
            }
        }
        ++loc;
    }
    return false;
}

template <int W>
__global__ __launch_bounds__(BUILD_THREADS) void k_part_build(KParams p, const uint64_t* buf2, uint64_t n,
                                                              const uint64_t* off2, uint64_t G,
                                                              uint64_t* slots, uint64_t cap, int table_empty,
                                                              uint64_t* ovf, uint64_t ovf_cap,
                                                              unsigned long long* ctr,
                                                              unsigned long long* stats,
                                                              uint32_t RC, const uint32_t* rcnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lt[];
    for (uint32_t r = blockIdx.x; r < NREG; r += gridDim.x) {
        const uint64_t lo = mulhi64((uint64_t)r << (64 - RBITS), cap);
        const uint64_t hi = (r + 1 < NREG) ? mulhi64((uint64_t)(r + 1) << (64 - RBITS), cap) : cap;
        const uint32_t S = (uint32_t)(hi - lo);
        if (W == 2) {
            ulonglong2* l2 = reinterpret_cast<ulonglong2*>(lt);
            const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(slots + lo * 2);
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS)
                l2[i] = table_empty ? make_ulonglong2(EMPTY, EMPTY) : g2[i];
        } else {
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS)
                lt[i] = table_empty ? (unsigned long long)EMPTY : (unsigned long long)slots[lo + i];
        }
        __syncthreads();
        uint64_t b, e;
        if (RC) {  // fixed region windows (k_part2_res)
            b = (uint64_t)r * RC;
            e = b + min(rcnt[r], RC);
        } else {
            b = off2[(uint64_t)(r >> B2) * G * NB2 + (r & (NB2 - 1))];
            e = (r + 1 < NREG) ? off2[(uint64_t)((r + 1) >> B2) * G * NB2 + ((r + 1) & (NB2 - 1))] : n;
        }
        for (uint64_t j = b + threadIdx.x; j < e; j += BUILD_THREADS) {
            uint64_t w0, w1 = 0;
            if (W == 2) {
                const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(buf2 + j * 2);
                w0 = v.x;
                w1 = v.y;
            } else {
                w0 = buf2[j];
            }
            const uint64_t home = home_slot(words_hash<W>(w0, w1, p), cap);
            if (!lds_insert<W>(lt, S, home - lo, w0, w1, stats)) {
                const unsigned long long idx = atomicAdd(&ctr[CT_OVF], 1ull);
                if (idx < ovf_cap) {
                    ovf[idx * W] = w0;
                    if (W == 2) ovf[idx * W + 1] = w1;
                } else {
                    atomicAdd(&stats[ST_FULL], 1ull);
                }
            }
        }
        __syncthreads();
        if (W == 2) {
            ulonglong2* dst = reinterpret_cast<ulonglong2*>(slots + lo * 2);
            const ulonglong2* l2 = reinterpret_cast<const ulonglong2*>(lt);
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) dst[i] = l2[i];
        } else {
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) slots[lo + i] = lt[i];
        }
        __syncthreads();
    }
}

// Build from fixed region windows with the next region's words prefetched: each thread holds up
// to IPT words of the region it inserts and issues the loads of its words of the next region
// before the LDS inserts and the slice write-out, and region hand-offs use LDS-only barriers,
// so a block's window loads, LDS work and slice stores overlap.
template <int W, int IPT>
__global__ __launch_bounds__(BUILD_THREADS) void k_part_build_pf(KParams p, const uint64_t* __restrict__ buf2,
                                                                 uint64_t* slots, uint64_t cap, int table_empty,
                                                                 uint64_t* ovf, uint64_t ovf_cap,
                                                                 unsigned long long* ctr,
                                                                 unsigned long long* stats, uint32_t RC,
                                                                 const uint32_t* __restrict__ rcnt) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lt[];
    uint64_t a[IPT], b[IPT];
    auto load = [&](uint32_t r, uint64_t (&x)[IPT], uint64_t (&y)[IPT]) {
        const uint32_t m = r < NREG ? min(rcnt[r], RC) : 0u;
        const uint64_t base = (uint64_t)(r < NREG ? r : 0) * RC;
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
    load(r, a, b);
    for (; r < NREG; r += gridDim.x) {
        const uint64_t lo = mulhi64((uint64_t)r << (64 - RBITS), cap);
        const uint64_t hi = (r + 1 < NREG) ? mulhi64((uint64_t)(r + 1) << (64 - RBITS), cap) : cap;
        const uint32_t S = (uint32_t)(hi - lo);
        if (W == 2) {
            ulonglong2* l2 = reinterpret_cast<ulonglong2*>(lt);
            const ulonglong2* g2 = reinterpret_cast<const ulonglong2*>(slots + lo * 2);
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS)
                l2[i] = table_empty ? make_ulonglong2(EMPTY, EMPTY) : g2[i];
        } else {
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS)
                lt[i] = table_empty ? (unsigned long long)EMPTY : (unsigned long long)slots[lo + i];
        }
        if (table_empty)
            lds_barrier();
        else
            __syncthreads();
        uint64_t na[IPT], nb[IPT];
        load(r + gridDim.x, na, nb);  // next region's words in flight during this one
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            if (a[j] == EMPTY) continue;
            const uint64_t home = home_slot(words_hash<W>(a[j], b[j], p), cap);
            if (!lds_insert<W>(lt, S, home - lo, a[j], b[j], stats)) {
                const unsigned long long idx = atomicAdd(&ctr[CT_OVF], 1ull);
                if (idx < ovf_cap) {
                    ovf[idx * W] = a[j];
                    if (W == 2) ovf[idx * W + 1] = b[j];
                } else {
                    atomicAdd(&stats[ST_FULL], 1ull);
                }
            }
        }
        lds_barrier();
        if (W == 2) {
            ulonglong2* dst = reinterpret_cast<ulonglong2*>(slots + lo * 2);
            const ulonglong2* l2 = reinterpret_cast<const ulonglong2*>(lt);
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) dst[i] = l2[i];
        } else {
            for (uint32_t i = threadIdx.x; i < S; i += BUILD_THREADS) slots[lo + i] = lt[i];
        }
        lds_barrier();
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            a[j] = na[j];
            b[j] = nb[j];
        }
    }
}

// Region-window build: the prefetching kernel when a window fits IPT words per thread.
template <int W>
static void launch_build_windows(const KParams& p, const PartBuffers& B, uint64_t n, uint64_t G, TableView t,
                                 bool table_empty, uint64_t ovf_cap, unsigned long long* ctr,
                                 unsigned long long* stats, uint32_t RC, const uint32_t* rcnt, size_t lds,
                                 hipStream_t s) {
    const char* e = getenv("KH_BUILD");
    const bool pf = !(e && !strcmp(e, "plain"));
    if (pf && RC <= 4u * BUILD_THREADS) {
        k_part_build_pf<W, 4><<<8192, BUILD_THREADS, lds, s>>>(p, B.buf2, t.slots, t.cap, table_empty ? 1 : 0,
                                                               B.overflow, ovf_cap, ctr, stats, RC, rcnt);
    } else if (pf && RC <= 12u * BUILD_THREADS) {
        k_part_build_pf<W, 12><<<8192, BUILD_THREADS, lds, s>>>(p, B.buf2, t.slots, t.cap, table_empty ? 1 : 0,
                                                                B.overflow, ovf_cap, ctr, stats, RC, rcnt);
    } else {
        k_part_build<W><<<8192, BUILD_THREADS, lds, s>>>(p, B.buf2, n, B.off2, G, t.slots, t.cap,
                                                         table_empty ? 1 : 0, B.overflow, ovf_cap, ctr, stats, RC,
                                                         rcnt);
    }
}

template <int W>
__global__ __launch_bounds__(PB) void k_insert_overflow(KParams p, const uint64_t* ovf, uint64_t ovf_cap,
                                                        const unsigned long long* ctr, uint64_t* slots,
                                                        uint64_t cap, unsigned long long* stats) {
    const uint64_t m = min((uint64_t)ctr[CT_OVF], ovf_cap);
    for (uint64_t i = (uint64_t)blockIdx.x * PB + threadIdx.x; i < m; i += (uint64_t)gridDim.x * PB) {
        const uint64_t w0 = ovf[i * W], w1 = (W == 2) ? ovf[i * W + 1] : 0;
        insert_one<W>(slot_key(w0, w1, p), slot_ext(w0), p, slots, cap, stats);
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
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(words + 2 * ii);
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
            const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(buf1 + 2 * i);
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
template <int W, int TB, int NB, int TILE, class CtrF, class WinF, class NextF>
__device__ __forceinline__ void sort_reserve_write(uint64_t* a, uint64_t* b, const uint32_t* bin, uint64_t* items,
                                                   uint16_t* sbin, uint32_t* hist, uint32_t* start, uint32_t* gpos,
                                                   uint32_t* wsum, CtrF counter, WinF window, uint32_t cap,
                                                   uint64_t* out, uint64_t* ovf, uint64_t ovf_cap,
                                                   unsigned long long* ctr, unsigned long long* stats, NextF next) {
    constexpr int IPT = TILE / TB;
    static_assert(NB <= TB, "one bin per thread");
    if (threadIdx.x < NB) hist[threadIdx.x] = 0;
    lds_barrier();
    uint32_t rank[IPT];
#pragma unroll
    for (int j = 0; j < IPT; ++j) rank[j] = (a[j] != EMPTY) ? atomicAdd(&hist[bin[j]], 1u) : 0u;
    lds_barrier();
    const uint32_t hv = threadIdx.x < NB ? hist[threadIdx.x] : 0u;
    uint32_t total;
    const uint32_t st = block_scan_u32<TB>(hv, total, wsum);
    if (threadIdx.x < NB) {
        start[threadIdx.x] = st;
        gpos[threadIdx.x] = hv ? atomicAdd(counter(threadIdx.x), hv) : 0u;
    }
    lds_barrier();
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
        if (a[j] != EMPTY) {
            const uint32_t pos = start[bin[j]] + rank[j];
            items[pos * W] = a[j];
            if (W == 2) items[pos * W + 1] = b[j];
            sbin[pos] = (uint16_t)bin[j];
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    next();  // the next tile's loads are in flight while this one is written
    lds_barrier();
#pragma unroll 4
    for (uint32_t x = threadIdx.x; x < total; x += TB) {
        const uint32_t q = sbin[x];
        const uint32_t w = gpos[q] + (x - start[q]);
        const uint64_t v0 = items[W * x], v1 = (W == 2) ? items[W * x + 1] : 0;
        if (w < cap) {
            const uint64_t g = window(q) + w;
            if (W == 2) {
                *reinterpret_cast<ulonglong2*>(out + g * 2) = make_ulonglong2(v0, v1);
            } else {
                out[g] = v0;
            }
        } else {
            const unsigned long long idx = atomicAdd(&ctr[CT_OVF], 1ull);
            if (idx < ovf_cap) {
                ovf[idx * W] = v0;
                if (W == 2) ovf[idx * W + 1] = v1;
            } else {
                atomicAdd(&stats[ST_FULL], 1ull);
            }
        }
    }
    lds_barrier();
}

// pass 1 on words: bucket = top 9 hash bits, S1 windows per bucket (window blockIdx % S1)
template <int W, int TB, bool COLLECT, int TILE>
__global__ __launch_bounds__(TB) void k_win1(KParams p, const uint64_t* __restrict__ words, uint64_t n,
                                             uint32_t CAP1, uint32_t* wcnt, uint64_t* buf1, uint64_t* ovf,
                                             uint64_t ovf_cap, unsigned long long* ctr,
                                             unsigned long long* stats, uint64_t* splits = nullptr,
                                             uint64_t splits_cap = 0) {
    constexpr int IPT = TILE / TB;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + TILE * 2);
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + TILE);
    uint32_t* start = hist + NB1;
    uint32_t* gpos = start + NB1;
    // block-scan partials in static LDS: 80 KB + a few bytes keeps these kernels at one block
    // (8 waves) per CU, measured faster than two (C3: pass 1 1.79-1.89 vs 1.98 ms, pass 2
    // 1.61-1.67 vs 1.69); the splitter buffer (COLLECT) uses the dynamic region's unused tail
    __shared__ uint32_t wsum[TB / 64];
    uint32_t* scount = gpos + NB1;
    uint64_t* sbuf = reinterpret_cast<uint64_t*>(scount + 2);
    const uint32_t sub = blockIdx.x % S1;
    const uint64_t b0 = (uint64_t)blockIdx.x * T1 * TILE;
    uint64_t a[IPT], b[IPT];
    if (COLLECT && threadIdx.x == 0) *scount = 0;
    load_words_tb<W, TB, TILE>(words, b0, min(b0 + TILE, n), b0 < n ? b0 : 0, a, b);
    for (int tt = 0; tt < T1; ++tt) {
        const uint64_t base = b0 + (uint64_t)tt * TILE;
        if (base >= n) break;  // uniform
        uint32_t bin[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t h = words_hash<W>(a[j], b[j], p);
            bin[j] = (uint32_t)(h >> (64 - B1));
            // splitter k-mers this shard owns (they head migrating-walk segments, kh_mseg.hip)
            if (COLLECT && a[j] != EMPTY && ext_bwd(slot_ext(a[j])) != EXT_F && is_splitter(h, p)) {
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

// pass 1 on records (KH_P1=recwin, k with a compile-time packed size PK): the windowed pass 1
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

template <int W, int TB, int TILE, int PK>
__global__ __launch_bounds__(TB) void k_win1_rec(KParams p, const uint8_t* __restrict__ recs, uint64_t n,
                                                 uint32_t CAP1, uint32_t* wcnt, uint64_t* buf1,
                                                 uint64_t* start_mask, uint64_t* split_mask, uint64_t* ovf,
                                                 uint64_t ovf_cap, unsigned long long* ctr,
                                                 unsigned long long* stats) {
    constexpr int IPT = TILE / TB;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + TILE * 2);
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + TILE);
    uint32_t* start = hist + NB1;
    uint32_t* gpos = start + NB1;
    __shared__ uint32_t wsum[TB / 64];
    const uint32_t sub = blockIdx.x % S1;
    // persistent blocks: tile t, t + gridDim.x, ...; the next tile's loads are always in flight
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    // a wave's 64 records are one contiguous run of 64 * R bytes: lane l loads the run's l-th
    // aligned 16-B block (coalesced, no straddling), and each lane later gathers the two blocks
    // holding its record by cross-lane shuffles
    constexpr uint32_t R = PK + 2;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t nbytes = n * (uint64_t)R;
    uint64_t a[IPT], b[IPT];  // raw 16-B blocks until parsed, then the words
    auto load = [&](uint64_t base, uint64_t end) {
#pragma unroll
        for (int j = 0; j < IPT; ++j) {
            const uint64_t r0 = base + (uint64_t)j * TB + (threadIdx.x & ~63u);  // the wave's first record
            const uint64_t g = ((r0 * R) & ~15ull) + 16ull * lane;
            a[j] = b[j] = 0;
            if (r0 < end && lane < 62 && g < nbytes) {
                const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(recs + g);
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
                if (valid) parse_record_regs_t<PK>(funnel64(w0, w1, sh), funnel64(w1, w2, sh), p.pad, k, ext);
            }
            const uint64_t hk = key_hash(k);
            if (s0 < n) {  // uniform: one start / splitter word per 64 consecutive records
                const bool is_start = valid && ext_bwd(ext) == EXT_F;
                const uint64_t bal = __ballot(is_start);
                const uint64_t sb = __ballot(valid && !is_start && is_splitter(hk, p));
                const uint64_t wb = s0 + (threadIdx.x & ~63u);
                if ((threadIdx.x & 63) == 0 && wb < n) {
                    if (start_mask) start_mask[wb >> 6] = bal;
                    if (split_mask) split_mask[wb >> 6] = sb;
                }
            }
            a[j] = valid ? slot_w0(k, ext, p) : EMPTY;
            b[j] = (valid && W == 2) ? k.lo : 0;
            bin[j] = (uint32_t)(hk >> (64 - B1));
        }
        const uint64_t nt = t + gridDim.x, nbase = nt * TILE;
        sort_reserve_write<W, TB, NB1, TILE>(
            a, b, bin, items, sbin, hist, start, gpos, wsum,
            [&](uint32_t q) { return &wcnt[q * S1 + sub]; },
            [&](uint32_t q) { return (uint64_t)(q * S1 + sub) * CAP1; }, CAP1, buf1, ovf, ovf_cap, ctr, stats,
            [&]() { load(nbase, nt < ntiles ? min(nbase + TILE, n) : nbase); });
    }
}

// pass 2: next 8 hash bits within bucket bk, into the region windows (RC words each)
template <int W, int TB, bool WIN, int TILE>
__global__ __launch_bounds__(TB) void k_win2(KParams p, const uint64_t* __restrict__ buf1, uint64_t n,
                                             const uint64_t* off1, uint64_t G, uint32_t RC, uint32_t* rcnt,
                                             uint64_t* buf2, uint64_t* ovf, uint64_t ovf_cap,
                                             unsigned long long* ctr, unsigned long long* stats, uint32_t CAP1,
                                             const uint32_t* wcnt) {
    constexpr int IPT = TILE / TB;
    extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
    uint64_t* items = smem;
    uint16_t* sbin = reinterpret_cast<uint16_t*>(smem + TILE * 2);
    uint32_t* hist = reinterpret_cast<uint32_t*>(sbin + TILE);
    uint32_t* start = hist + NB1;
    uint32_t* gpos = start + NB1;
    __shared__ uint32_t wsum[TB / 64];  // static: one block per CU (see k_win1)
    const uint32_t bk = blockIdx.x / (uint32_t)G, g = blockIdx.x % (uint32_t)G;
    uint64_t s, e;
    uint32_t pre[S1 + 1];
    if (WIN) {
        pre[0] = 0;
#pragma unroll
        for (uint32_t j = 0; j < S1; ++j) pre[j + 1] = pre[j] + min(wcnt[bk * S1 + j], CAP1);
        s = 0;
        e = pre[S1];
    } else {
        bucket_range(off1, 0, n, bk, s, e);
    }
    uint64_t a[IPT], b[IPT];
    auto load = [&](uint64_t t) {
        const uint64_t e_ = t < e ? min(t + TILE, e) : t;
        if (WIN)
            load_words_win_tb<W, TB, TILE>(buf1, bk, CAP1, pre, t, e_, a, b);
        else
            load_words_tb<W, TB, TILE>(buf1, t, e_, s, a, b);
    };
    load(s + (uint64_t)g * TILE);
    for (uint64_t t = s + (uint64_t)g * TILE; t < e; t += G * TILE) {
        uint32_t bin[IPT];
#pragma unroll
        for (int j = 0; j < IPT; ++j)
            bin[j] = (uint32_t)(words_hash<W>(a[j], b[j], p) >> (64 - RBITS)) & (NB2 - 1);
        sort_reserve_write<W, TB, NB2, TILE>(
            a, b, bin, items, sbin, hist, start, gpos, wsum,
            [&](uint32_t q) { return &rcnt[(bk << B2) | q]; },
            [&](uint32_t q) { return (uint64_t)((bk << B2) | q) * RC; }, RC, buf2, ovf, ovf_cap, ctr, stats,
            [&]() { load(t + G * TILE); });
    }
}

static int win_tb() {
    const char* e = getenv("KH_TB");
    return (e && *e) ? atoi(e) : 512;
}

template <class K>
static hipError_t allow_lds(K kernel, size_t bytes) {
    return hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

// windowed pass 1 / pass 2 launches at tile size TILE (KH_WTILE = 4096 | 8192)
template <int W, int TILE>
static hipError_t win1_launch_t(const KParams& p, const uint64_t* words, uint64_t n, uint32_t CAP1, uint32_t* wcnt,
                                const PartBuffers& B, uint64_t ovf_cap, unsigned long long* ctr,
                                unsigned long long* stats, hipStream_t s, uint64_t* wsplits, uint64_t wsplits_cap) {
    constexpr size_t L = sort_lds(TILE);
    const unsigned nb = (unsigned)win_blocks1(n, TILE);
    hipError_t e;
    if (wsplits) {
        if ((e = allow_lds(k_win1<W, 512, true, TILE>, L)) != hipSuccess) return e;
        k_win1<W, 512, true, TILE><<<nb, 512, L, s>>>(p, words, n, CAP1, wcnt, B.buf1, B.overflow, ovf_cap, ctr,
                                                      stats, wsplits, wsplits_cap);
    } else {
        if ((e = allow_lds(k_win1<W, 512, false, TILE>, L)) != hipSuccess) return e;
        k_win1<W, 512, false, TILE><<<nb, 512, L, s>>>(p, words, n, CAP1, wcnt, B.buf1, B.overflow, ovf_cap, ctr,
                                                       stats);
    }
    return hipSuccess;
}
template <int W>
static hipError_t win1_launch(const KParams& p, const uint64_t* words, uint64_t n, uint32_t CAP1, uint32_t* wcnt,
                              const PartBuffers& B, uint64_t ovf_cap, unsigned long long* ctr,
                              unsigned long long* stats, hipStream_t s, uint64_t* wsplits, uint64_t wsplits_cap) {
    return win_tile() == PART_TILE
               ? win1_launch_t<W, PART_TILE>(p, words, n, CAP1, wcnt, B, ovf_cap, ctr, stats, s, wsplits, wsplits_cap)
               : win1_launch_t<W, WIN_TILE>(p, words, n, CAP1, wcnt, B, ovf_cap, ctr, stats, s, wsplits, wsplits_cap);
}
template <int W, int PK, int TILE>
static hipError_t win1_rec_launch_t(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t CAP1,
                                    uint32_t* wcnt, const PartBuffers& B, uint64_t* start_mask,
                                    uint64_t* split_mask, uint64_t ovf_cap, unsigned long long* ctr,
                                    unsigned long long* stats, hipStream_t s) {
    constexpr size_t L = sort_lds(TILE);
    hipError_t e;
    if ((e = allow_lds(k_win1_rec<W, 512, TILE, PK>, L)) != hipSuccess) return e;
    // persistent: a few blocks per CU slot (one 152-KiB block fits a CU), a multiple of S1
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
    }
    const char* gb = getenv("KH_RWIN_BLOCKS");
    uint64_t grid = gb ? (uint64_t)atoi(gb) : (uint64_t)ncu;
    grid = (grid + S1 - 1) / S1 * S1;
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    if (grid > ntiles) grid = (ntiles + S1 - 1) / S1 * S1;
    if (grid == 0) grid = S1;
    k_win1_rec<W, 512, TILE, PK><<<(unsigned)grid, 512, L, s>>>(
        p, recs, n, CAP1, wcnt, B.buf1, start_mask, split_mask, B.overflow, ovf_cap, ctr, stats);
    return hipSuccess;
}
template <int W>
static hipError_t win1_rec_launch(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t CAP1,
                                  uint32_t* wcnt, const PartBuffers& B, uint64_t* start_mask, uint64_t* split_mask,
                                  uint64_t ovf_cap, unsigned long long* ctr, unsigned long long* stats,
                                  hipStream_t s) {
    constexpr int PK = W == 2 ? 13 : 5;
    const char* t = getenv("KH_RTILE");
    if (t && atoi(t) == PART_TILE)
        return win1_rec_launch_t<W, PK, PART_TILE>(p, recs, n, CAP1, wcnt, B, start_mask, split_mask, ovf_cap,
                                                   ctr, stats, s);
    return win1_rec_launch_t<W, PK, WIN_TILE>(p, recs, n, CAP1, wcnt, B, start_mask, split_mask, ovf_cap, ctr,
                                              stats, s);
}
template <int W, bool WIN, int TILE>
static hipError_t win2_launch_t(const KParams& p, const PartBuffers& B, uint64_t n, uint32_t RC, uint32_t* rcnt,
                                uint64_t ovf_cap, unsigned long long* ctr, unsigned long long* stats, uint32_t CAP1,
                                const uint32_t* wcnt, hipStream_t s) {
    constexpr size_t L = sort_lds(TILE);
    uint64_t G = win_G(n, TILE);
    if (const char* e = getenv("KH_WIN2_G")) G = (uint64_t)atoi(e) > 0 ? (uint64_t)atoi(e) : G;
    hipError_t e;
    if ((e = allow_lds(k_win2<W, 512, WIN, TILE>, L)) != hipSuccess) return e;
    k_win2<W, 512, WIN, TILE><<<(unsigned)(NB1 * G), 512, L, s>>>(p, B.buf1, n, B.off1, G, RC, rcnt, B.buf2,
                                                                  B.overflow, ovf_cap, ctr, stats, CAP1, wcnt);
    return hipSuccess;
}
template <int W, bool WIN>
static hipError_t win2_launch(const KParams& p, const PartBuffers& B, uint64_t n, uint32_t RC, uint32_t* rcnt,
                              uint64_t ovf_cap, unsigned long long* ctr, unsigned long long* stats, uint32_t CAP1,
                              const uint32_t* wcnt, hipStream_t s) {
    return win_tile() == PART_TILE
               ? win2_launch_t<W, WIN, PART_TILE>(p, B, n, RC, rcnt, ovf_cap, ctr, stats, CAP1, wcnt, s)
               : win2_launch_t<W, WIN, WIN_TILE>(p, B, n, RC, rcnt, ovf_cap, ctr, stats, CAP1, wcnt, s);
}

template <int W, bool REC>
static hipError_t part_insert(const KParams& p, const uint8_t* recs, const uint64_t* words, uint64_t n,
                              TableView t, bool table_empty, const PartBuffers& B, uint64_t* start_mask,
                              uint64_t* split_mask,
                              unsigned long long* ctr, unsigned long long* stats, hipStream_t s,
                              hipEvent_t after_records = nullptr, uint64_t* wsplits = nullptr,
                              uint64_t wsplits_cap = 0) {
    static bool attrs = false;  // per template instance
    hipError_t e;
    if (!attrs) {
        if ((e = allow_lds(k_part1_scatter<W, false>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part2_scatter<W>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part1_scatter<W, true>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part2_res<W, true>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part2_res<W, false>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part1_fused<W, true>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part1_fused<W, false>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part1_direct<W>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part1_direct<W, 13>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part1_direct<W, 5>, SORT_LDS)) != hipSuccess) return e;
        if ((e = allow_lds(k_part_build<W>, LDS_BYTES)) != hipSuccess) return e;
        if ((e = allow_lds(k_part_build_pf<W, 4>, LDS_BYTES)) != hipSuccess) return e;
        if ((e = allow_lds(k_part_build_pf<W, 12>, LDS_BYTES)) != hipSuccess) return e;
        attrs = true;
    }
    const PartPlan pl = part_plan(n);
    const unsigned nb1 = (unsigned)pl.nb1;
    int mode1 = p1_mode(REC);
    if (mode1 == 3 && (!REC || p.R > 16)) mode1 = REC ? 1 : 0;  // direct parse: records of <= 16 B
    if (mode1 == 4 && !REC) mode1 = 0;
    const bool direct1 = mode1 == 3;
    if (mode1 == 5 && !(REC && ((p.P == 13 && W == 2) || (p.P == 5 && W == 1)))) mode1 = REC ? 4 : 0;
    if (mode1 == 4) {  // records -> words (input order) in buf2, then the windowed pass 1 on them
        if (p.P == 13 && W == 2)
            k_part1_convert<W, 13><<<nb1, PB, 0, s>>>(p, recs, n, B.buf2, nullptr, start_mask, split_mask);
        else if (p.P == 5 && W == 1)
            k_part1_convert<W, 5><<<nb1, PB, 0, s>>>(p, recs, n, B.buf2, nullptr, start_mask, split_mask);
        else
            k_part1_convert<W><<<nb1, PB, 0, s>>>(p, recs, n, B.buf2, nullptr, start_mask, split_mask);
        words = B.buf2;
        if (after_records) {  // start / splitter bits are complete: the caller's compaction may start
            if ((e = hipEventRecord(after_records, s)) != hipSuccess) return e;
            after_records = nullptr;
        }
    }
    const bool fused1 = mode1 == 0 || direct1 || mode1 == 4 || mode1 == 5, rec1 = REC && mode1 == 2;
    const bool res2 = fused1 || p2_res();
    if ((e = hipMemsetAsync(ctr + CT_OVF, 0, 8, s)) != hipSuccess) return e;
    uint32_t CAP1 = 0;
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(B.hist1);
    if (fused1) {
        CAP1 = part_win1_cap(n);
        if ((e = hipMemsetAsync(wcnt, 0, (size_t)NW1 * 4, s)) != hipSuccess) return e;
        if (mode1 == 5) {
            if ((e = win1_rec_launch<W>(p, recs, n, CAP1, wcnt, B, start_mask, split_mask, part_overflow_cap(n),
                                        ctr, stats, s)) != hipSuccess)
                return e;
        } else if (direct1 && p.P == 13 && W == 2 && !getenv("KH_NOMASK"))
            k_part1_direct<W, 13><<<nb1, PB, SORT_LDS, s>>>(p, recs, n, CAP1, wcnt, B.buf1, start_mask, split_mask,
                                                           B.overflow, part_overflow_cap(n), ctr, stats);
        else if (direct1 && p.P == 5 && W == 1)
            k_part1_direct<W, 5><<<nb1, PB, SORT_LDS, s>>>(p, recs, n, CAP1, wcnt, B.buf1, start_mask, split_mask,
                                                          B.overflow, part_overflow_cap(n), ctr, stats);
        else if (direct1 && getenv("KH_NOMASK"))
            k_part1_direct<W, 13><<<nb1, PB, SORT_LDS, s>>>(p, recs, n, CAP1, wcnt, B.buf1, nullptr, nullptr,
                                                           B.overflow, part_overflow_cap(n), ctr, stats);
        else if (direct1)
            k_part1_direct<W><<<nb1, PB, SORT_LDS, s>>>(p, recs, n, CAP1, wcnt, B.buf1, start_mask, split_mask,
                                                       B.overflow, part_overflow_cap(n), ctr, stats);
        else if ((mode1 == 4 || (mode1 == 0 && !REC)) && win_tb() == 512)
        {
            if ((e = win1_launch<W>(p, words, n, CAP1, wcnt, B, part_overflow_cap(n), ctr, stats, s, wsplits,
                                    wsplits_cap)) != hipSuccess)
                return e;
        }
        else if (mode1 == 4)
            k_part1_fused<W, false><<<nb1, PB, SORT_LDS, s>>>(p, nullptr, words, n, CAP1, wcnt, B.buf1, nullptr,
                                                               nullptr, B.overflow, part_overflow_cap(n), ctr,
                                                               stats);
        else
            k_part1_fused<W, REC><<<nb1, PB, SORT_LDS, s>>>(p, recs, words, n, CAP1, wcnt, B.buf1, start_mask,
                                                             split_mask, B.overflow, part_overflow_cap(n), ctr,
                                                             stats);
    } else if (REC && !rec1) {
        // records -> words (input order) in buf2, which pass 2 only writes after pass 1 is done
        k_part1_convert<W><<<nb1, PB, 0, s>>>(p, recs, n, B.buf2, B.hist1, start_mask, split_mask);
        words = B.buf2;
    } else if (rec1) {
        // parse the records twice (histogram pass, then the scatter) instead of writing and
        // re-reading a word copy of them: 3.0 GB less HBM traffic at C3
        k_part1_hist<W, true><<<nb1, PB, 0, s>>>(p, recs, nullptr, n, B.hist1, start_mask, split_mask);
    } else {
        k_part1_hist<W, false><<<nb1, PB, 0, s>>>(p, nullptr, words, n, B.hist1, nullptr, nullptr);
    }
    if (after_records && (e = hipEventRecord(after_records, s)) != hipSuccess) return e;
    if (!fused1) {
        e = scan_exclusive(Hist1F{B.hist1, pl.nb1}, pl.nb1 * NB1, B.off1, B.scratch,
                           (unsigned long long*)nullptr, (unsigned long long*)nullptr, s, Off1Idx{pl.nb1});
        if (e != hipSuccess) return e;
        if (rec1)
            k_part1_scatter<W, true><<<nb1, PB, SORT_LDS, s>>>(p, recs, nullptr, n, B.off1, pl.nb1, B.buf1);
        else
            k_part1_scatter<W, false><<<nb1, PB, SORT_LDS, s>>>(p, nullptr, words, n, B.off1, pl.nb1, B.buf1);
    }
    const unsigned nb2 = (unsigned)(NB1 * pl.G);
    uint32_t RC = 0;
    uint32_t* rcnt = reinterpret_cast<uint32_t*>(B.hist2);
    if (res2) {
        RC = part_region_cap(n);
        if ((e = hipMemsetAsync(rcnt, 0, (size_t)NREG * 4, s)) != hipSuccess) return e;
        if (win_tb() == 512 && CAP1) {
            if ((e = win2_launch<W, true>(p, B, n, RC, rcnt, part_overflow_cap(n), ctr, stats, CAP1, wcnt, s)) !=
                hipSuccess)
                return e;
        } else if (win_tb() == 512) {  // pass-1 exact offsets: the grid of part_plan
            if ((e = allow_lds(k_win2<W, 512, false, PART_TILE>, SORT_LDS)) != hipSuccess) return e;
            k_win2<W, 512, false, PART_TILE><<<nb2, 512, SORT_LDS, s>>>(p, B.buf1, n, B.off1, pl.G, RC, rcnt,
                                                                        B.buf2, B.overflow, part_overflow_cap(n),
                                                                        ctr, stats, 0, nullptr);
        } else if (CAP1)
            k_part2_res<W, true><<<nb2, PB, SORT_LDS, s>>>(p, B.buf1, n, B.off1, pl.G, RC, rcnt, B.buf2,
                                                          B.overflow, part_overflow_cap(n), ctr, stats, CAP1,
                                                          wcnt);
        else
            k_part2_res<W, false><<<nb2, PB, SORT_LDS, s>>>(p, B.buf1, n, B.off1, pl.G, RC, rcnt, B.buf2,
                                                           B.overflow, part_overflow_cap(n), ctr, stats, 0,
                                                           nullptr);
    } else {
        k_part2_hist<W><<<nb2, PB, 0, s>>>(p, B.buf1, n, B.off1, pl.nb1, pl.G, B.hist2);
        e = scan_exclusive(Hist2F{B.hist2, (uint32_t)pl.G}, (uint64_t)NB1 * NB2 * pl.G, B.off2, B.scratch,
                           (unsigned long long*)nullptr, (unsigned long long*)nullptr, s,
                           Off2Idx{(uint32_t)pl.G});
        if (e != hipSuccess) return e;
        k_part2_scatter<W><<<nb2, PB, SORT_LDS, s>>>(p, B.buf1, n, B.off1, pl.nb1, pl.G, B.off2, B.buf2);
    }
    const size_t lds = (size_t)region_max_slots(t.cap) * W * 8;
    if (RC)
        launch_build_windows<W>(p, B, n, pl.G, t, table_empty, part_overflow_cap(n), ctr, stats, RC, rcnt, lds, s);
    else
        k_part_build<W><<<8192, BUILD_THREADS, lds, s>>>(p, B.buf2, n, B.off2, pl.G, t.slots, t.cap,
                                                         table_empty ? 1 : 0, B.overflow,
                                                         part_overflow_cap(n), ctr, stats, RC, rcnt);
    k_insert_overflow<W><<<1024, PB, 0, s>>>(p, B.overflow, part_overflow_cap(n), ctr, t.slots, t.cap,
                                             stats);
    return hipGetLastError();
}


// Staged build (sharded insert): words arrive in chunks (one per all-to-all chunk). Each chunk is
// partitioned at once (pass 1 into its own windows, pass 2 appending to the region windows of a
// build sized for `total` words) while the next chunk is still on the wire; one build at the end.
template <int W>
static hipError_t part_stage(const KParams& p, const uint64_t* words, uint64_t m, uint64_t total, bool first,
                             const PartBuffers& B, unsigned long long* ctr, unsigned long long* stats,
                             hipStream_t s, uint64_t* wsplits, uint64_t wsplits_cap) {
    hipError_t e;
    if ((e = allow_lds(k_part1_fused<W, false>, SORT_LDS)) != hipSuccess) return e;
    if ((e = allow_lds(k_part2_res<W, true>, SORT_LDS)) != hipSuccess) return e;
    uint32_t* wcnt = reinterpret_cast<uint32_t*>(B.hist1);
    uint32_t* rcnt = reinterpret_cast<uint32_t*>(B.hist2);
    if (first) {
        if ((e = hipMemsetAsync(ctr + CT_OVF, 0, 8, s)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(rcnt, 0, (size_t)NREG * 4, s)) != hipSuccess) return e;
    }
    if (m == 0) return hipSuccess;
    const PartPlan pl = part_plan(m);
    const uint32_t CAP1 = part_win1_cap(m), RC = part_region_cap(total);
    if ((e = hipMemsetAsync(wcnt, 0, (size_t)NW1 * 4, s)) != hipSuccess) return e;
    if (win_tb() == 512) {
        if ((e = win1_launch<W>(p, words, m, CAP1, wcnt, B, part_overflow_cap(total), ctr, stats, s, wsplits,
                                wsplits_cap)) != hipSuccess)
            return e;
        if ((e = win2_launch<W, true>(p, B, m, RC, rcnt, part_overflow_cap(total), ctr, stats, CAP1, wcnt, s)) !=
            hipSuccess)
            return e;
        return hipGetLastError();
    }
    k_part1_fused<W, false><<<(unsigned)pl.nb1, PB, SORT_LDS, s>>>(p, nullptr, words, m, CAP1, wcnt, B.buf1,
                                                                  nullptr, nullptr, B.overflow,
                                                                  part_overflow_cap(total), ctr, stats);
    k_part2_res<W, true><<<(unsigned)(NB1 * pl.G), PB, SORT_LDS, s>>>(p, B.buf1, m, B.off1, pl.G, RC, rcnt, B.buf2,
                                                                      B.overflow, part_overflow_cap(total), ctr,
                                                                      stats, CAP1, wcnt);
    return hipGetLastError();
}

template <int W>
static hipError_t part_finish(const KParams& p, uint64_t total, TableView t, bool table_empty, const PartBuffers& B,
                              unsigned long long* ctr, unsigned long long* stats, hipStream_t s) {
    hipError_t e;
    if ((e = allow_lds(k_part_build<W>, LDS_BYTES)) != hipSuccess) return e;
    if ((e = allow_lds(k_part_build_pf<W, 4>, LDS_BYTES)) != hipSuccess) return e;
    if ((e = allow_lds(k_part_build_pf<W, 12>, LDS_BYTES)) != hipSuccess) return e;
    const uint32_t RC = part_region_cap(total);
    const uint32_t* rcnt = reinterpret_cast<const uint32_t*>(B.hist2);
    const size_t lds = (size_t)region_max_slots(t.cap) * W * 8;
    launch_build_windows<W>(p, B, total, 1, t, table_empty, part_overflow_cap(total), ctr, stats, RC, rcnt, lds, s);
    k_insert_overflow<W><<<1024, PB, 0, s>>>(p, B.overflow, part_overflow_cap(total), ctr, t.slots, t.cap, stats);
    return hipGetLastError();
}

hipError_t launch_part_stage(const KParams& p, const uint64_t* words, uint64_t m, uint64_t total, bool first,
                             const PartBuffers& b, unsigned long long* ctr, unsigned long long* stats,
                             hipStream_t s, uint64_t* wsplits, uint64_t wsplits_cap) {
    return p.W == 1 ? part_stage<1>(p, words, m, total, first, b, ctr, stats, s, wsplits, wsplits_cap)
                    : part_stage<2>(p, words, m, total, first, b, ctr, stats, s, wsplits, wsplits_cap);
}

hipError_t launch_part_finish(const KParams& p, uint64_t total, TableView t, bool table_empty,
                              const PartBuffers& b, unsigned long long* ctr, unsigned long long* stats,
                              hipStream_t s) {
    return p.W == 1 ? part_finish<1>(p, total, t, table_empty, b, ctr, stats, s)
                    : part_finish<2>(p, total, t, table_empty, b, ctr, stats, s);
}

bool part_words_collect_splits() { return win_tb() == 512; }

hipError_t launch_part_insert(const KParams& p, const uint8_t* recs, const uint64_t* words, uint64_t n,
                              TableView t, bool table_empty, const PartBuffers& b,
                              uint64_t* start_mask, uint64_t* split_mask, unsigned long long* ctr,
                              unsigned long long* stats, hipStream_t s, hipEvent_t after_records,
                              uint64_t* wsplits, uint64_t wsplits_cap) {
    if (n == 0) return hipSuccess;
    if (recs) {
        return p.W == 1 ? part_insert<1, true>(p, recs, nullptr, n, t, table_empty, b, start_mask, split_mask, ctr,
                                               stats, s, after_records)
                        : part_insert<2, true>(p, recs, nullptr, n, t, table_empty, b, start_mask, split_mask, ctr,
                                               stats, s, after_records);
    }
    return p.W == 1 ? part_insert<1, false>(p, nullptr, words, n, t, table_empty, b, nullptr, nullptr, ctr, stats, s,
                                            nullptr, wsplits, wsplits_cap)
                    : part_insert<2, false>(p, nullptr, words, n, t, table_empty, b, nullptr, nullptr, ctr, stats, s,
                                            nullptr, wsplits, wsplits_cap);
}

}  // namespace kh
