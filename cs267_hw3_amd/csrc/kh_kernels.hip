// kh_kernels.hip — hand-written gfx950 kernels for the k-mer table and the contig walker.
//
// Path (reference -> here):
//   hash_map.hpp:55-80 insert_all / stock HashMap::insert  -> k_insert (LDS-staged record tiles,
//                                                             64-bit CAS open addressing)
//   kmer_hash.cpp:27-31 start-node collection            -> start bit per record (wave ballot) +
//                                                             order-preserving compaction
//   hash_map.hpp:83-107 find                              -> k_find (batched)
//   kmer_hash.cpp:38-55 assemble_contigs                  -> k_walk (persistent per-lane walkers,
//                                                             wave-batched work queue)
//   read_kmers.hpp:81-92 extract_contig + output_results  -> k_write_heads / k_write_chunks
// Everything is integer work bound by HBM random access; there is no MFMA on this path.
#include <hip/hip_runtime.h>

#include "kh_kernels.hpp"

namespace kh {

static constexpr int BLOCK = 256;
static constexpr int SCAN_ITEMS = 8;
static constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;  // 2048 elements per block
static constexpr int WALK_GRAB = 64;                   // start k-mers per work-queue pull
static constexpr int MAX_R = 17;                       // K <= 60 -> PACKED <= 15 -> R <= 17

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
static inline uint64_t hmin(uint64_t a, uint64_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ---------------------------------------------------------------------------------------------
// Block-wide exclusive scan of one uint64 per thread (256 threads = 4 waves of 64).
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
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < BLOCK / 64; ++i) {
        if (i < w) pre += wsum[i];
        tot += wsum[i];
    }
    __syncthreads();
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

template <class F>
__global__ __launch_bounds__(BLOCK) void k_scan_reduce(F f, uint64_t m, uint64_t* bsum) {
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j)
        if (b0 + j < m) s += f(b0 + j);
    uint64_t tot;
    block_excl_scan(s, tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// One block: exclusive scan of the nb block sums in place, starting at *base (if given);
// *base (if given) and *total_out (if given) receive base + sum.
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

template <class F>
__global__ __launch_bounds__(BLOCK) void k_scan_apply(F f, uint64_t m, const uint64_t* bsum,
                                                      uint64_t* out) {
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint64_t v[SCAN_ITEMS];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        v[j] = (b0 + j < m) ? f(b0 + j) : 0ull;
        s += v[j];
    }
    uint64_t tot;
    uint64_t pre = block_excl_scan(s, tot) + bsum[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        if (b0 + j < m) out[b0 + j] = pre;
        pre += v[j];
    }
}

uint64_t scan_scratch_words(uint64_t m) { return (m + SCAN_TILE - 1) / SCAN_TILE + 1; }

template <class F>
static hipError_t scan_exclusive(F f, uint64_t m, uint64_t* out, uint64_t* scratch,
                                 unsigned long long* base, unsigned long long* total,
                                 hipStream_t s) {
    if (m == 0) return hipSuccess;
    const uint64_t nb = (m + SCAN_TILE - 1) / SCAN_TILE;
    k_scan_reduce<F><<<dim3((unsigned)nb), dim3(BLOCK), 0, s>>>(f, m, scratch);
    k_scan_top<<<1, BLOCK, 0, s>>>(scratch, nb, base, total);
    k_scan_apply<F><<<dim3((unsigned)nb), dim3(BLOCK), 0, s>>>(f, m, scratch, out);
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
template <int W>
__device__ __forceinline__ void insert_one(Key k, uint32_t ext, const KParams& p, uint64_t* slots,
                                           uint64_t cap, unsigned long long* stats) {
    unsigned long long* S = reinterpret_cast<unsigned long long*>(slots);
    const unsigned long long w0 = slot_w0(k, ext, p);
    const unsigned long long w1 = k.lo;
    uint64_t s = home_slot(key_hash(k), cap);
    uint64_t probes = 0;
    uint32_t spins = 0;
    while (true) {
        const unsigned long long old = atomicCAS(&S[W * s], (unsigned long long)EMPTY, w0);
        if (old == EMPTY) {
            if (W == 2) atomicExch(&S[2 * s + 1], w1);
            return;
        }
        if ((old >> 6) == (w0 >> 6)) {
            if (W == 1) {
                atomicAdd(&stats[ST_DUP], 1ull);
                return;
            }
            const unsigned long long o1 =
                atomicCAS(&S[2 * s + 1], (unsigned long long)EMPTY, (unsigned long long)EMPTY);
            if (o1 == EMPTY) {
                if (++spins > (1u << 26)) {
                    atomicAdd(&stats[ST_SPIN], 1ull);
                    return;
                }
                continue;  // word1 not yet published: retry this slot next iteration
            }
            if (o1 == w1) {
                atomicAdd(&stats[ST_DUP], 1ull);
                return;
            }
        }
        if (++probes >= cap) {
            atomicAdd(&stats[ST_FULL], 1ull);
            return;
        }
        s = (s + 1 == cap) ? 0 : s + 1;
    }
}

template <int W>
__global__ __launch_bounds__(BLOCK) void k_insert(KParams p, const uint8_t* __restrict__ recs,
                                                  uint64_t n, uint64_t* slots, uint64_t cap,
                                                  uint64_t* start_mask,
                                                  unsigned long long* stats) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[BLOCK * MAX_R];
    const uint32_t R = (uint32_t)p.R;
    const uint64_t ntiles = (n + BLOCK - 1) / BLOCK;
    for (uint64_t ti = blockIdx.x; ti < ntiles; ti += gridDim.x) {
        const uint64_t base = ti * BLOCK;
        const uint32_t cnt = (uint32_t)min((uint64_t)BLOCK, n - base);
        const uint32_t bytes = cnt * R;
        const uint8_t* src = recs + base * R;
        const uint32_t nvec = bytes >> 4;
        for (uint32_t v = threadIdx.x; v < nvec; v += BLOCK)
            reinterpret_cast<uint4*>(tile)[v] = reinterpret_cast<const uint4*>(src)[v];
        for (uint32_t b = (nvec << 4) + threadIdx.x; b < bytes; b += BLOCK) tile[b] = src[b];
        __syncthreads();
        const bool valid = threadIdx.x < cnt;
        Key k{0, 0};
        uint32_t ext = 0;
        if (valid) parse_record(tile + threadIdx.x * R, p, k, ext);
        __syncthreads();  // tile is reused by the next iteration
        const bool is_start = valid && ext_bwd(ext) == EXT_F;
        const uint64_t bal = __ballot(is_start);
        const uint64_t wbase = base + (threadIdx.x & ~63u);
        if ((threadIdx.x & 63) == 0 && wbase < n) start_mask[wbase >> 6] = bal;
        if (valid) {
            if (ext_bwd(ext) == EXT_BAD || ext_fwd(ext) == EXT_BAD) atomicAdd(&stats[ST_BAD_EXT], 1ull);
            insert_one<W>(k, ext, p, slots, cap, stats);
        }
    }
}

hipError_t launch_insert(const KParams& p, const uint8_t* recs, uint64_t n, TableView t,
                         uint64_t* start_mask, unsigned long long* stats, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t ntiles = (n + BLOCK - 1) / BLOCK;
    const unsigned grid = (unsigned)hmin(ntiles, 256ull * 32);
    if (p.W == 1)
        k_insert<1><<<grid, BLOCK, 0, s>>>(p, recs, n, t.slots, t.cap, start_mask, stats);
    else
        k_insert<2><<<grid, BLOCK, 0, s>>>(p, recs, n, t.slots, t.cap, start_mask, stats);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Start-node compaction in record order (kmer_hash.cpp:27-31 push_back order).
template <int W>
__global__ __launch_bounds__(BLOCK) void k_scatter_starts(KParams p, const uint8_t* recs, uint64_t n,
                                                          const uint64_t* mask,
                                                          const uint64_t* mask_off,
                                                          uint64_t* starts) {
    const uint64_t nw = (n + 63) >> 6;
    for (uint64_t w = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; w < nw;
         w += (uint64_t)gridDim.x * BLOCK) {
        uint64_t m = mask[w];
        uint64_t o = mask_off[w];
        while (m) {
            const int b = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const uint64_t i = (w << 6) + (uint64_t)b;
            Key k;
            uint32_t ext;
            parse_record(recs + i * (uint64_t)p.R, p, k, ext);
            starts[o * W] = slot_w0(k, ext, p);
            if (W == 2) starts[o * W + 1] = k.lo;
            ++o;
        }
    }
}

hipError_t launch_collect_starts(const KParams& p, const uint8_t* recs, uint64_t n,
                                 const uint64_t* start_mask, uint64_t* mask_offsets,
                                 uint64_t* scratch, uint64_t* starts, unsigned long long* ctr,
                                 hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t nw = (n + 63) >> 6;
    hipError_t e = scan_exclusive(PopcF{start_mask}, nw, mask_offsets, scratch, &ctr[CT_N_STARTS],
                                  (unsigned long long*)nullptr, s);
    if (e != hipSuccess) return e;
    const unsigned grid = (unsigned)hmin((nw + BLOCK - 1) / BLOCK, 4096);
    if (p.W == 1)
        k_scatter_starts<1><<<grid, BLOCK, 0, s>>>(p, recs, n, start_mask, mask_offsets, starts);
    else
        k_scatter_starts<2><<<grid, BLOCK, 0, s>>>(p, recs, n, start_mask, mask_offsets, starts);
    return hipGetLastError();
}

template <int W>
__global__ __launch_bounds__(BLOCK) void k_load_starts(KParams p, const uint8_t* recs, uint64_t n,
                                                       uint64_t* starts) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * BLOCK) {
        Key k;
        uint32_t ext;
        parse_record(recs + i * (uint64_t)p.R, p, k, ext);
        starts[i * W] = slot_w0(k, ext, p);
        if (W == 2) starts[i * W + 1] = k.lo;
    }
}

__global__ void k_set_ctr(unsigned long long* ctr, int idx, unsigned long long v) { ctr[idx] = v; }

hipError_t launch_load_starts(const KParams& p, const uint8_t* recs, uint64_t n, uint64_t* starts,
                              unsigned long long* ctr, hipStream_t s) {
    if (n) {
        const unsigned grid = (unsigned)hmin((n + BLOCK - 1) / BLOCK, 4096);
        if (p.W == 1)
            k_load_starts<1><<<grid, BLOCK, 0, s>>>(p, recs, n, starts);
        else
            k_load_starts<2><<<grid, BLOCK, 0, s>>>(p, recs, n, starts);
    }
    k_set_ctr<<<1, 1, 0, s>>>(ctr, CT_N_STARTS, (unsigned long long)n);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Probe: returns true and the slot's word0 if the key is present. Table is read-only here
// (written by an earlier kernel), so plain 8/16-byte loads are coherent.
template <int W>
__device__ __forceinline__ bool probe(Key k, const KParams& p, const uint64_t* __restrict__ slots,
                                      uint64_t cap, uint64_t& w0_out) {
    uint64_t s = home_slot(key_hash(k), cap);
    const uint64_t want0 = (W == 1) ? k.lo : k.hi;
    for (uint64_t probes = 0; probes < cap; ++probes) {
        uint64_t w0, w1 = 0;
        if (W == 2) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(slots + 2 * s);
            w0 = v.x;
            w1 = v.y;
        } else {
            w0 = slots[s];
        }
        if (w0 == EMPTY) return false;
        if ((w0 >> 6) == want0 && (W == 1 || w1 == k.lo)) {
            w0_out = w0;
            return true;
        }
        s = (s + 1 == cap) ? 0 : s + 1;
    }
    return false;
}

template <int W>
__global__ __launch_bounds__(BLOCK) void k_find(KParams p, const uint8_t* keys, uint64_t n,
                                                const uint64_t* slots, uint64_t cap, uint8_t* out,
                                                uint8_t* found) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * BLOCK) {
        const Key k = key_from_packed(keys + i * (uint64_t)p.P, p);
        uint64_t w0 = 0;
        const bool f = probe<W>(k, p, slots, cap, w0);
        uint8_t* o = out + i * (uint64_t)p.R;
        if (f) {
            write_record(o, k, slot_ext(w0), p);
        } else {
            for (int j = 0; j < p.R; ++j) o[j] = 0;
        }
        found[i] = f ? 1 : 0;
    }
}

hipError_t launch_find(const KParams& p, const uint8_t* keys, uint64_t n, TableView t, uint8_t* out,
                       uint8_t* found, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)hmin((n + BLOCK - 1) / BLOCK, 8192);
    if (p.W == 1)
        k_find<1><<<grid, BLOCK, 0, s>>>(p, keys, n, t.slots, t.cap, out, found);
    else
        k_find<2><<<grid, BLOCK, 0, s>>>(p, keys, n, t.slots, t.cap, out, found);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Walker (kmer_hash.cpp:41-53). Each lane owns one contig at a time: append the forward base,
// shift it into the key (next_kmer), probe, repeat until fwd == 'F'. Finished lanes refill from
// a work queue that the wave pulls WALK_GRAB start k-mers at a time (one atomic per pull instead
// of one per contig). Appended bases are packed 2 bits each into 256-base chunks allocated on
// demand; k_write_chunks turns them into characters at the contig's final offset.
template <int W>
__global__ __launch_bounds__(BLOCK) void k_walk(KParams p, const uint64_t* __restrict__ slots,
                                                uint64_t cap, WalkBuffers wb,
                                                unsigned long long* ctr,
                                                unsigned long long* stats) {
    const uint32_t lane = lane_id();
    uint64_t q_next = 0, q_end = 0;  // wave-uniform queue window
    bool active = false, done = false;
    uint64_t c = 0;
    Key k{0, 0};
    uint32_t fwd = 0;
    uint32_t steps = 0;  // bases appended so far (= k-mers in contig - 1)
    uint32_t chunk = 0;
    uint64_t buf = 0;
    while (true) {
        const bool need = !active && !done;
        const uint64_t m = __ballot(need);
        if (m) {
            const uint32_t cnt = (uint32_t)__popcll(m);
            const uint32_t rank = mbcnt64(m);
            const uint64_t avail = q_end - q_next;
            uint64_t nbase = 0;
            if (cnt > avail) {
                unsigned long long g = 0;
                if (lane == 0) g = atomicAdd(&ctr[CT_WALK_NEXT], (unsigned long long)WALK_GRAB);
                nbase = __shfl(g, 0, 64);
            }
            const uint64_t mine = (rank < avail) ? q_next + rank : nbase + (rank - avail);
            if (cnt > avail) {
                q_next = nbase + (cnt - avail);
                q_end = nbase + WALK_GRAB;
            } else {
                q_next += cnt;
            }
            if (need) {
                if (mine >= wb.n_starts) {
                    done = true;
                } else {
                    c = mine;
                    const uint64_t w0 = wb.starts[c * W];
                    const uint64_t w1 = (W == 2) ? wb.starts[c * W + 1] : 0;
                    k = slot_key(w0, w1, p);
                    fwd = ext_fwd(slot_ext(w0));
                    steps = 0;
                    buf = 0;
                    active = true;
                }
            }
        }
        if (!__any(active)) break;
        if (active) {
            bool finish = false;
            if (fwd == EXT_F) {
                finish = true;
            } else if (fwd > 3) {
                atomicAdd(&stats[ST_BAD_EXT], 1ull);
                finish = true;
            } else {
                if ((steps & (CHUNK_BASES - 1)) == 0) {
                    chunk = (uint32_t)atomicAdd(&ctr[CT_CHUNK_NEXT], 1ull);
                    if (chunk < wb.chunk_cap) {
                        wb.chunk_owner[chunk] = (uint32_t)c;
                        wb.chunk_seq[chunk] = steps / CHUNK_BASES;
                    } else {
                        atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
                    }
                }
                buf |= (uint64_t)fwd << (2 * (steps & 31));
                if ((steps & 31) == 31) {
                    if (chunk < wb.chunk_cap)
                        wb.chunk_data[(uint64_t)chunk * CHUNK_WORDS + ((steps >> 5) & 7)] = buf;
                    buf = 0;
                }
                ++steps;
                k = key_next(k, fwd, p);
                uint64_t w0 = 0;
                if (probe<W>(k, p, slots, cap, w0)) {
                    fwd = ext_fwd(slot_ext(w0));
                    if (steps > wb.max_steps) {
                        atomicAdd(&stats[ST_CYCLE], 1ull);
                        finish = true;
                    }
                } else {
                    atomicAdd(&stats[ST_MISSING], 1ull);
                    finish = true;
                }
            }
            if (finish) {
                wb.contig_len[c] = steps + 1;
                if ((steps & 31) && chunk < wb.chunk_cap)
                    wb.chunk_data[(uint64_t)chunk * CHUNK_WORDS + ((steps >> 5) & 7)] = buf;
                active = false;
            }
        }
    }
}

hipError_t launch_walk(const KParams& p, TableView t, const WalkBuffers& wb, unsigned long long* ctr,
                       unsigned long long* stats, int grid_blocks, hipStream_t s) {
    if (wb.n_starts == 0) return hipSuccess;
    uint64_t want = (wb.n_starts + BLOCK - 1) / BLOCK;
    unsigned grid = (unsigned)hmin(want, (uint64_t)(grid_blocks > 0 ? grid_blocks : 2048));
    if (p.W == 1)
        k_walk<1><<<grid, BLOCK, 0, s>>>(p, t.slots, t.cap, wb, ctr, stats);
    else
        k_walk<2><<<grid, BLOCK, 0, s>>>(p, t.slots, t.cap, wb, ctr, stats);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Materialisation: contig c occupies bytes [off[c], off[c] + K + len[c]) =
//   K chars of the start k-mer, len[c]-1 appended forward bases, '\n'.
template <int W>
__global__ __launch_bounds__(BLOCK) void k_write_heads(KParams p, const uint64_t* starts, uint64_t nc,
                                                       const uint32_t* len, const uint64_t* off,
                                                       char* out) {
    for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < nc;
         c += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t w0 = starts[c * W];
        const uint64_t w1 = (W == 2) ? starts[c * W + 1] : 0;
        const Key k = slot_key(w0, w1, p);
        char* o = out + off[c];
        for (int i = 0; i < p.K; ++i) o[i] = (char)code_char(key_base(k, i, p));
        o[p.K + len[c] - 1] = '\n';
    }
}

__global__ __launch_bounds__(BLOCK) void k_write_chunks(int K, const uint64_t* chunk_data,
                                                        const uint32_t* owner, const uint32_t* seq,
                                                        const unsigned long long* ctr,
                                                        uint64_t chunk_cap, const uint32_t* len,
                                                        const uint64_t* off, char* out) {
    // The chunk count is only known on the device (walker allocation head), so the grid is sized
    // for the capacity and bounded here.
    const uint64_t nchunks = min((uint64_t)ctr[CT_CHUNK_NEXT], chunk_cap);
    const uint64_t nwords = nchunks * CHUNK_WORDS;
    for (uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < nwords;
         t += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t ch = t / CHUNK_WORDS;
        const uint32_t w = (uint32_t)(t % CHUNK_WORDS);
        const uint32_t c = owner[ch];
        const uint64_t j0 = (uint64_t)seq[ch] * CHUNK_BASES + (uint64_t)w * 32;
        const uint64_t app = (uint64_t)len[c] - 1;
        if (j0 >= app) continue;
        const uint32_t cntb = (uint32_t)min<uint64_t>(32, app - j0);
        const uint64_t word = chunk_data[t];
        char* o = out + off[c] + K + j0;
        for (uint32_t i = 0; i < cntb; ++i) o[i] = (char)code_char((uint32_t)(word >> (2 * i)) & 3u);
    }
}

hipError_t launch_materialize(const KParams& p, const WalkBuffers& wb, uint64_t* offsets,
                              uint64_t* scratch, char* out, unsigned long long* ctr, hipStream_t s) {
    const uint64_t nc = wb.n_starts;
    if (nc == 0) return hipSuccess;
    hipError_t e = scan_exclusive(ContigBytesF{wb.contig_len, (uint64_t)p.K}, nc, offsets, scratch,
                                  (unsigned long long*)nullptr, &ctr[CT_OUT_BYTES], s);
    if (e != hipSuccess) return e;
    const unsigned gh = (unsigned)hmin((nc + BLOCK - 1) / BLOCK, 8192);
    if (p.W == 1)
        k_write_heads<1><<<gh, BLOCK, 0, s>>>(p, wb.starts, nc, wb.contig_len, offsets, out);
    else
        k_write_heads<2><<<gh, BLOCK, 0, s>>>(p, wb.starts, nc, wb.contig_len, offsets, out);
    const unsigned gc =
        (unsigned)hmin((wb.chunk_cap * CHUNK_WORDS + BLOCK - 1) / BLOCK, 8192);
    k_write_chunks<<<gc, BLOCK, 0, s>>>(p.K, wb.chunk_data, wb.chunk_owner, wb.chunk_seq, ctr,
                                        wb.chunk_cap, wb.contig_len, offsets, out);
    return hipGetLastError();
}

}  // namespace kh
