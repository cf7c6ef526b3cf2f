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

#include "kh_device.hpp"
#include "kh_kernels.hpp"

namespace kh {

uint64_t scan_scratch_words(uint64_t m) { return (m + SCAN_TILE - 1) / SCAN_TILE + 1; }

template <int W>
__global__ __launch_bounds__(BLOCK) void k_insert(KParams p, const uint8_t* __restrict__ recs,
                                                  uint64_t n, uint64_t* slots, uint64_t cap,
                                                  uint64_t* start_mask, uint64_t* split_mask,
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
        if (split_mask) {
            const uint64_t sb = __ballot(valid && !is_start && is_splitter(k, p));
            if ((threadIdx.x & 63) == 0 && wbase < n) split_mask[wbase >> 6] = sb;
        }
        if (valid) {
            if (ext_bwd(ext) == EXT_BAD || ext_fwd(ext) == EXT_BAD) atomicAdd(&stats[ST_BAD_EXT], 1ull);
            insert_one<W>(k, slot_w0(k, ext, p), home_of(place(k, p), cap, p), p, slots, cap, stats);
        }
    }
}

hipError_t launch_insert(const KParams& p, const uint8_t* recs, uint64_t n, TableView t,
                         uint64_t* start_mask, uint64_t* split_mask, unsigned long long* stats, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t ntiles = (n + BLOCK - 1) / BLOCK;
    const unsigned grid = (unsigned)hmin(ntiles, 256ull * 32);
    if (p.W == 1)
        k_insert<1><<<grid, BLOCK, 0, s>>>(p, recs, n, t.slots, t.cap, start_mask, split_mask, stats);
    else
        k_insert<2><<<grid, BLOCK, 0, s>>>(p, recs, n, t.slots, t.cap, start_mask, split_mask, stats);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Start-node compaction in record order (kmer_hash.cpp:27-31 push_back order).
template <int W>
__global__ __launch_bounds__(BLOCK) void k_scatter_starts(KParams p, const uint8_t* recs, uint64_t n,
                                                          const uint64_t* mask,
                                                          const uint64_t* mask_off,
                                                          uint64_t* starts) {
    // 64 mask words per wave (one per lane). Sparse (C3: ~1 start per 100 records): each lane
    // parses the set bits of its own word. Dense (C5: every start k-mer at the front of the
    // records): the wave takes the words one at a time, lane j = record 64w + j, so the record
    // reads coalesce instead of 64 serial byte-wise parses per lane.
    const uint64_t nw = (n + 63) >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (BLOCK / 64);
    auto put = [&](uint64_t i, uint64_t o) {
        Key k;
        uint32_t ext;
        if (p.R <= 16) {  // uniform: two aligned 16-B loads instead of R byte loads
            uint64_t x0, x1;
            load_record_regs(recs, i, (uint32_t)p.R, x0, x1);
            parse_record_regs(x0, x1, p, k, ext);
        } else {
            parse_record(recs + i * (uint64_t)p.R, p, k, ext);
        }
        starts[o * W] = slot_w0(k, ext, p);
        if (W == 2) starts[o * W + 1] = k.lo;
    };
    for (uint64_t w0 = ((uint64_t)blockIdx.x * (BLOCK / 64) + (threadIdx.x >> 6)) * 64; w0 < nw; w0 += waves * 64) {
        const uint64_t w = w0 + lane;
        const uint64_t m = w < nw ? mask[w] : 0;
        const uint64_t o = w < nw ? mask_off[w] : 0;
        uint32_t c = (uint32_t)__popcll(m);
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) c += __shfl_xor(c, d, 64);
        if (c <= 128) {
            uint64_t mm = m, oo = o;
            while (mm) {
                const int b = __ffsll((unsigned long long)mm) - 1;
                mm &= mm - 1;
                put((w << 6) + (uint64_t)b, oo++);
            }
        } else {
            for (int j = 0; j < 64; ++j) {
                const uint64_t mj = __shfl(m, j, 64);
                const uint64_t oj = __shfl(o, j, 64);
                if ((mj >> lane) & 1) put(((w0 + j) << 6) + lane, oj + (uint64_t)__popcll(mj & ((1ull << lane) - 1)));
            }
        }
    }
}

hipError_t launch_collect_starts(const KParams& p, const uint8_t* recs, uint64_t n,
                                 const uint64_t* start_mask, uint64_t* mask_offsets,
                                 uint64_t* scratch, uint64_t* starts, unsigned long long* ctr,
                                 hipStream_t s, int ctr_idx) {
    if (n == 0) return hipSuccess;
    const uint64_t nw = (n + 63) >> 6;
    hipError_t e = scan_exclusive(PopcF{start_mask}, nw, mask_offsets, scratch, &ctr[ctr_idx],
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
// shift it into the key (next_kmer), probe, repeat until fwd == 'F'.
//
// The loop is a per-lane state machine that issues exactly ONE table load per lane per
// iteration: a lane whose probe hit an occupied foreign slot simply probes the next slot on the
// next iteration instead of looping inside the wave (which made every lane wait for the longest
// probe chain in its wave). Finished lanes refill from a work queue the wave pulls WALK_GRAB start
// k-mers at a time; the batch's start records are preloaded one per lane with a coalesced load
// and handed out by shuffle, so refilling costs no dependent memory round trip. Appended bases are
// packed 2 bits each into 256-base chunks; k_write_chunks turns them into characters at the
// contig's final offset. Contig c owns chunk c outright (its first 256 bases); only longer contigs
// draw further chunks from a counter, so contig starts never contend on one atomic word (a
// per-contig atomicAdd on a single counter capped the walk at ~88 allocations/us).
struct LaneOut {
    uint32_t* contig_len;
    uint64_t* chunk_data;
    uint32_t* chunk_owner;   // only chunks >= n_first are recorded (chunk c < n_first is contig c)
    uint32_t* chunk_seq;
    uint64_t chunk_cap;
    uint64_t n_first;        // = number of contigs
};

// Word w of chunk ch, word-major: word w of every chunk together, so the first words of consecutive
// contigs are adjacent (the line writer reads 8 B per short contig instead of its 64-B chunk; the
// walker's first-word stores of a wave's 64 contigs fill whole lines).
__device__ __forceinline__ uint64_t chunk_word(uint64_t ch, uint32_t w, uint64_t chunk_cap) {
    return (uint64_t)w * chunk_cap + ch;
}

// Append base `b` as base number `steps` of contig c (2 bits, 32 per word, 8 words per chunk).
__device__ __forceinline__ void append_base(const LaneOut& o, uint64_t c, uint32_t b, uint32_t& steps,
                                            uint32_t& chunk, uint64_t& buf, unsigned long long* ctr,
                                            unsigned long long* stats) {
    if (steps == 0) {
        chunk = (uint32_t)c;
    } else if ((steps & (CHUNK_BASES - 1)) == 0) {
        chunk = (uint32_t)(o.n_first + atomicAdd(&ctr[CT_CHUNK_NEXT], 1ull));
        if (chunk < o.chunk_cap) {
            o.chunk_owner[chunk] = (uint32_t)c;
            o.chunk_seq[chunk] = steps / CHUNK_BASES;
        } else {
            atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
        }
    }
    buf |= (uint64_t)b << (2 * (steps & 31));
    if ((steps & 31) == 31) {
        if (chunk < o.chunk_cap) o.chunk_data[chunk_word(chunk, (steps >> 5) & 7, o.chunk_cap)] = buf;
        buf = 0;
    }
    ++steps;
}

// Append m <= 32 - (steps & 31) bases at once (piece: base i at bits 2i), same layout as append_base.
__device__ __forceinline__ void append_run(const LaneOut& o, uint64_t c, uint64_t piece, uint32_t m, uint32_t& steps,
                                           uint32_t& chunk, uint64_t& buf, unsigned long long* ctr,
                                           unsigned long long* stats) {
    if (steps == 0) {
        chunk = (uint32_t)c;
    } else if ((steps & (CHUNK_BASES - 1)) == 0) {
        chunk = (uint32_t)(o.n_first + atomicAdd(&ctr[CT_CHUNK_NEXT], 1ull));
        if (chunk < o.chunk_cap) {
            o.chunk_owner[chunk] = (uint32_t)c;
            o.chunk_seq[chunk] = steps / CHUNK_BASES;
        } else {
            atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
        }
    }
    buf |= piece << (2 * (steps & 31));
    steps += m;
    if ((steps & 31) == 0) {
        if (chunk < o.chunk_cap) o.chunk_data[chunk_word(chunk, ((steps - 1) >> 5) & 7, o.chunk_cap)] = buf;
        buf = 0;
    }
}

// bits [sh, sh + 64) of V = hi * 2^62 + lo
__device__ __forceinline__ uint64_t key_bits64(Key k, uint32_t sh) {
    return sh < 62 ? (k.lo >> sh) | (sh ? k.hi << (62 - sh) : k.hi << 62) : k.hi >> (sh - 62);
}
// reverse the order of the 32 2-bit groups of x
__device__ __forceinline__ uint64_t rev2_64(uint64_t x) {
    const uint64_t r = ((uint64_t)__builtin_bitreverse32((uint32_t)x) << 32) | __builtin_bitreverse32((uint32_t)(x >> 32));
    return ((r >> 1) & 0x5555555555555555ull) | ((r & 0x5555555555555555ull) << 1);
}
// Append the last n bases of k (oldest first): the links of a chain record (kh_build.hip).
__device__ __forceinline__ void append_key_tail(const LaneOut& o, uint64_t c, Key k, uint32_t n, uint32_t& steps,
                                                uint32_t& chunk, uint64_t& buf, unsigned long long* ctr,
                                                unsigned long long* stats) {
    while (n) {
        const uint32_t room = 32u - (steps & 31u);
        const uint32_t m = n < room ? n : room;
        const uint64_t x = key_bits64(k, 2 * (n - m));
        const uint64_t piece = rev2_64(m >= 32 ? x : x & ((1ull << (2 * m)) - 1)) >> (64 - 2 * m);
        append_run(o, c, piece, m, steps, chunk, buf, ctr, stats);
        n -= m;
    }
}

__device__ __forceinline__ void finish_contig(const LaneOut& o, uint64_t c, uint32_t steps, uint32_t chunk,
                                              uint64_t buf) {
    o.contig_len[c] = steps + 1;
    if ((steps & 31) && chunk < o.chunk_cap)
        o.chunk_data[chunk_word(chunk, (steps >> 5) & 7, o.chunk_cap)] = buf;
}

__device__ __forceinline__ uint64_t walk_splits(const WalkBuffers& wb) {
    return wb.n_splits_dev ? (uint64_t)*wb.n_splits_dev : wb.n_splits;
}

// ---------------------------------------------------------------------------------------------
// Quad-transposed walker: one walker per lane, every probe reads the walker's whole 4-slot block
// (64 B at 16-B slots): lane q of a quad loads slot q of the block of each of the quad's 4
// walkers, so a lookup costs ~1.06 random requests instead of ~1.3 for slot-by-slot probes
// (linear-probing displacement crossing a slot). The walk is bound by the number of random line
// requests the memory system serves (~51 G/s whether a request is a 16-B slot or a full 128-B
// line: tools/membench chase16 / chase64q / chase128o). All intra-quad exchange is DPP quad_perm
// (ALU, no LDS): each walker's probe position and key are broadcast to its quad, and the hit
// slot's extension comes back by a quad OR-reduction.
//
// Chains (kh_build.hip region_chains): a looked-up k-mer whose slot carries a head-record index
// is the head of a run of k-mers that share its minimizer; the walker then reads the record
// (one 16-B load) and appends the run's bases in one step — the record holds the run's last
// k-mer (tail) whose low 2*links bits ARE those bases — and continues from the tail's extension.
// A C3 contig (~104 k-mers) costs ~6 such hops of two dependent requests instead of ~104 lookups.
// Every walker starts by looking up its own start k-mer (to find its record).

template <int W, int KT>
__global__ __launch_bounds__(BLOCK) void k_walk_q(KParams p_in, const uint64_t* __restrict__ slots,
                                                  uint64_t cap, WalkBuffers wb,
                                                  unsigned long long* ctr,
                                                  unsigned long long* stats) {
    const KParams p = specialize<KT>(p_in);
    const uint32_t lane = lane_id();
    const uint32_t q = lane & 3, ql = lane & ~3u;
    const uint64_t n_all = wb.n_starts + walk_splits(wb);
    // Deferred splitter segments (wb.split_min): the splitter walkers follow the start walkers in
    // the queue. A wave that reaches them before any contig has stopped at a splitter (seg_long[0],
    // read once per reservation) defers them all: it moves the queue head past the end
    // (atomicMax), sets seg_long[1] and stops taking walkers. Phase 1 then walks the splitter
    // walkers that were not walked (contig_len still 0), and returns at once unless some contig
    // stopped at a splitter after all (plain loads: phase 0 wrote the flags in an earlier kernel).
    // C3 (contigs shorter than the splitter spacing): no splitter walker runs; C5: the long chains
    // stop early, so the splitter walkers run in phase 0 beside the short contigs as before.
    if (wb.phase == 1 && !(wb.seg_long[0] && wb.seg_long[1])) return;
    const uint64_t q_first = wb.phase == 1 ? wb.n_starts : 0;
    uint64_t n = n_all;  // wave-uniform: the last walker this wave may take (+1)
    // the flags are read and written at most once per wave (agent-scope accesses pass the per-XCD
    // L2 and serialise on one address: one per lane cost C3 10 ms)
    bool long_known = wb.phase == 1;
    const LaneOut o{wb.contig_len, wb.chunk_data, wb.chunk_owner, wb.chunk_seq, wb.chunk_cap, n_all};
    const bool chains = p.chain && wb.hcap != 0;
    uint64_t bbase = 0, rbase = 0;
    uint32_t bused = WALK_GRAB, rleft = 0;  // rleft: walkers left in the wave's reservation
    const uint32_t grab_all = WALK_GRAB * (wb.batches ? wb.batches : (uint32_t)WALK_BATCHES);
    bool bdry = false;
    uint64_t bw0 = 0, bw1 = 0;

    bool active = false, done = false, resolved = false;
    bool entry = false;  // looking up the walker's own start k-mer (fwd = the start record's)
    uint64_t c = 0, s = 0, buf = 0, pb = 0;   // pb: 4-slot blocks probed for the current k-mer
    const uint64_t pb_max = (cap >> 2) + 1;   // every block once: the k-mer is absent (a full table)
    uint32_t reg = 0;  // region of the k-mer being looked up (its head records live there)
    Key k{0, 0};
    uint32_t fwd = 0, steps = 0, chunk = 0;
    uint32_t nrec = 0;  // the last record's successor run (head-record index + 1 in its region)
    // k needs its placement this iteration: its home slot for a lookup, or its region for the
    // record the last record named. One place() site for both (and for a new walker's own start
    // k-mer): a wave whose lanes take different paths runs the minimizer scan once, not per path.
    bool do_place = false;
    while (true) {
        while (true) {
            const bool need = !active && !done;
            bool skipped = false;  // phase 1: took a walker phase 0 walked: take another
            const uint64_t m = __ballot(need);
            if (m) {
                const uint32_t cnt = (uint32_t)__popcll(m);
                const uint32_t rank = mbcnt64(m);
                const uint32_t avail = WALK_GRAB - bused;
                const uint32_t src_old = min(bused + rank, (uint32_t)WALK_GRAB - 1);
                const uint64_t o0 = __shfl(bw0, (int)src_old, 64);
                const uint64_t o1 = __shfl(bw1, (int)src_old, 64);
                const uint64_t oc = bbase + src_old;
                uint64_t n0 = 0, n1 = 0, nc = ~0ull;
                if (cnt > avail) {
                    if (!bdry) {
                        if (rleft == 0) {  // reserve WALK_BATCHES batches with one atomic
                            unsigned long long g = 0;
                            if (lane == 0)
                                g = q_first + atomicAdd(&ctr[CT_WALK_NEXT], (unsigned long long)grab_all);
                            rbase = __shfl(g, 0, 64);
                            rleft = grab_all;
                            // (a reservation past the end, after some wave deferred: nothing to check)
                            if (wb.split_min && !long_known && rbase + grab_all > wb.n_starts && rbase < n_all) {
                                long_known = __hip_atomic_load(wb.seg_long, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT) != 0;
                                if (!long_known) {  // defer every splitter walker to phase 1
                                    if (lane == 0 && atomicMax(&ctr[CT_WALK_NEXT], (unsigned long long)n_all) < n_all)
                                        __hip_atomic_store(wb.seg_long + 1, 1u, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
                                    n = wb.n_starts;
                                }
                            }
                        }
                        bbase = rbase;
                        rbase += WALK_GRAB;
                        rleft -= WALK_GRAB;
                        if (bbase >= n) bdry = true;
                        const uint64_t mi = bbase + lane;
                        if (mi < n) {
                            const uint64_t* src = mi < wb.n_starts ? wb.starts + mi * W
                                                                   : wb.splits + (mi - wb.n_starts) * W;
                            bw0 = src[0];
                            bw1 = (W == 2) ? src[1] : 0;
                        }
                        const uint32_t src_new = min(rank - min(rank, avail), (uint32_t)WALK_GRAB - 1);
                        n0 = __shfl(bw0, (int)src_new, 64);
                        n1 = __shfl(bw1, (int)src_new, 64);
                        nc = bbase + src_new;
                    }
                    bused = cnt - avail;
                } else {
                    bused += cnt;
                }
                if (need) {
                    uint64_t cc, x0, x1;
                    if (rank < avail) {
                        cc = oc;
                        x0 = o0;
                        x1 = o1;
                    } else {
                        cc = nc;
                        x0 = n0;
                        x1 = n1;
                    }
                    // phase 1: a splitter walker phase 0 walked (its length is set) is not taken
                    const bool take = cc < n && (wb.phase == 0 || wb.contig_len[cc] == 0);
                    skipped = cc < n && !take;
                    if (take) {
                        c = cc;
                        k = slot_key(x0, x1, p);
                        fwd = ext_fwd(slot_ext(x0));
                        steps = 0;
                        buf = 0;
                        nrec = 0;
                        active = true;
                        entry = chains;
                        resolved = !chains;  // with chains: its own slot tells whether a record covers its run
                        do_place = chains;
                    } else if (!skipped) {
                        done = true;
                    }
                }
            }
            const bool fin = active && resolved && fwd > 3;
            if (fin) {
                if (fwd != EXT_F) atomicAdd(&stats[ST_BAD_EXT], 1ull);
                finish_contig(o, c, steps, chunk, buf);
                active = false;
            }
            if (!__any(fin || skipped)) break;
        }
        if (!__any(active)) break;
        bool stop_long = false;
        if (active && resolved) {
            append_base(o, c, fwd, steps, chunk, buf, ctr, stats);
            k = key_next(k, fwd, p);
            if (is_splitter(k, p) && (c >= wb.n_starts || steps >= wb.split_min)) {
                stop_long = c < wb.n_starts;  // a long contig: splitter segments are needed
                finish_contig(o, c, steps, chunk, buf);
                wb.seg_next[c] = SEG_AT_SPLIT;
                wb.seg_key[2 * c] = k.hi;
                wb.seg_key[2 * c + 1] = k.lo;
                active = false;
            } else {
                do_place = true;
            }
        }
        if (wb.split_min && !long_known && __any(stop_long)) {  // once per wave
            if (lane == 0) __hip_atomic_store(wb.seg_long, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            long_known = true;
        }
        if (do_place) {
            const Place pl = place(k, p);
            reg = pl.r;
            if (nrec) {  // the record named the run that starts at k (k_rec_succ): read it, no probe
                s = WQ_REC | ((uint64_t)reg * wb.hcap + nrec - 1);
                nrec = 0;
            } else {     // look up k: s = its home slot (the hit may carry a head-record index)
                s = home_of(pl, cap, p);
                pb = 0;
            }
            resolved = false;
            do_place = false;
        }
        // -- quad loads: a probe reads 4 slots per lane, one per quad member's block; a record
        //    read loads the same 16 B in all 4 lanes (one request) ------------------------------
        const uint64_t sp = active ? s : WQ_IDLE;
        uint64_t sj[4], w0[4], w1[4];
        sj[0] = qbcast64<0>(sp);
        sj[1] = qbcast64<1>(sp);
        sj[2] = qbcast64<2>(sp);
        sj[3] = qbcast64<3>(sp);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            w0[j] = EMPTY;
            w1[j] = 0;
            if (sj[j] == WQ_IDLE) continue;
            if (sj[j] & WQ_REC) {
                const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(wb.headrec + (sj[j] & ~WQ_REC) * 2);
                w0[j] = v.x;
                w1[j] = v.y;
            } else {
                const uint64_t my = (sj[j] & ~3ull) + q;
                if (my < cap) load_slot_nt<W>(slots, my, w0[j], w1[j]);
            }
        }
        uint64_t kh_[4], kl_[4];
        kh_[0] = qbcast64<0>(k.hi);
        kh_[1] = qbcast64<1>(k.hi);
        kh_[2] = qbcast64<2>(k.hi);
        kh_[3] = qbcast64<3>(k.hi);
        kl_[0] = qbcast64<0>(k.lo);
        kl_[1] = qbcast64<1>(k.lo);
        kl_[2] = qbcast64<2>(k.lo);
        kl_[3] = qbcast64<3>(k.lo);
        uint32_t myfh = 4, myfe = 4, myext = 0;
        uint64_t r0 = 0, r1 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t my = (sj[j] & ~3ull) + q;
            const bool probe_j = sj[j] != WQ_IDLE && !(sj[j] & WQ_REC);
            const bool valid = probe_j && my >= sj[j] && my < cap;
            const bool empty = w0[j] == EMPTY;
            const bool hit = !empty & (slot_keybits(w0[j], p) == ((W == 1) ? kl_[j] : kh_[j])) &
                             ((W == 1) | (w1[j] == kl_[j]));
            const uint32_t bh = (uint32_t)(__ballot(valid && hit) >> ql) & 0xFu;
            const uint32_t be = (uint32_t)(__ballot(valid && empty) >> ql) & 0xFu;
            const uint32_t fh = bh ? (uint32_t)__builtin_ctz(bh) : 4u;
            const uint32_t fe = be ? (uint32_t)__builtin_ctz(be) : 4u;
            // hit slot: ext | found flag | head-record index << 7
            const uint32_t ext =
                qor32(q == fh ? (slot_ext(w0[j]) | 0x40u | ((chains ? slot_hidx(w0[j], p) : 0u) << 7)) : 0u);
            if (q == (uint32_t)j) {
                myfh = fh;
                myfe = fe;
                myext = ext;
                r0 = w0[j];
                r1 = w1[j];
            }
        }
        if (active) {
            if (s & WQ_REC) {
                // head record: jump to the run's tail, appending the bases of its links
                k = slot_key(r0, r1, p);
                fwd = ext_fwd(slot_ext(r0));
                const uint32_t links = rec_links(r0, p);
                nrec = rec_succ(r0, p);
                append_key_tail(o, c, k, links, steps, chunk, buf, ctr, stats);
                resolved = true;
                if (steps > wb.max_steps) {
                    atomicAdd(&stats[ST_CYCLE], 1ull);
                    finish_contig(o, c, steps, chunk, buf);
                    active = false;
                }
            } else if (myfh < myfe) {
                const uint32_t hidx = myext >> 7, tf = ext_fwd(myext & 63u);
                // a start walks from its own record (kmer_hash.cpp:42-44): a record whose run
                // begins with another extension (duplicate key) is not used for it
                if (hidx && !(entry && tf != fwd)) {
                    s = WQ_REC | ((uint64_t)reg * wb.hcap + hidx - 1);
                } else {
                    if (!entry) fwd = tf;
                    resolved = true;
                    if (steps > wb.max_steps) {
                        atomicAdd(&stats[ST_CYCLE], 1ull);
                        finish_contig(o, c, steps, chunk, buf);
                        active = false;
                    }
                }
                entry = false;
            } else if (myfe < 4u || ++pb > pb_max) {
                if (entry) {  // a start k-mer need not be in the table (kh_set_starts)
                    resolved = true;
                    entry = false;
                } else {
                    atomicAdd(&stats[ST_MISSING], 1ull);
                    finish_contig(o, c, steps, chunk, buf);
                    active = false;
                }
            } else {
                const uint64_t nx = (s & ~3ull) + 4;
                s = nx >= cap ? 0 : nx;
            }
        }
    }
}

// Successor of every head record of the last build: the run after the tail starts at
// y = next_kmer(tail); when y's slot carries a head-record index (y heads a run with a record),
// that index goes into the record (rec_succ), so the walker reads y's record straight after this
// one instead of probing y's slot first (one dependent request per run instead of two). Splitters
// need no test here: the walker checks the next k-mer for one before it follows a successor.
// Each wave owns a contiguous range of regions and keeps its 64 lanes busy with a queue over the
// range's records (the per-region counts follow the records, written by the build): a lane reads
// its record, then probes y's 4-slot blocks quad-transposed as the walker does (lane q of a quad
// loads slot q of each member's 64-B block; one request per block instead of one per slot: ~1.3
// requests per lookup slot by slot). Records of consecutive lanes are consecutive 16-B lines.
template <int W, int KT>
__global__ __launch_bounds__(BLOCK) void k_rec_succ(KParams p_in, const uint64_t* __restrict__ slots, uint64_t cap,
                                                    uint64_t* headrec, uint32_t hcap) {
    const KParams p = specialize<KT>(p_in);
    const uint32_t NR = nreg(p);
    const uint32_t* hn = reinterpret_cast<const uint32_t*>(headrec + (uint64_t)NR * hcap * 2);
    const int sh = rec_succ_shift(p);
    const uint32_t lane = lane_id(), q = lane & 3u, ql = lane & ~3u;
    const uint32_t waves = gridDim.x * (BLOCK / 64), wv = blockIdx.x * (BLOCK / 64) + threadIdx.x / 64;
    const uint32_t rpw = (NR + waves - 1) / waves;
    uint32_t r = wv * rpw;                       // wave-uniform queue cursor: region r, record id
    const uint32_t r_end = min(r + rpw, NR);
    uint32_t id = 0;
    // lane state: its record (index + 1, 0 = idle), y, the probe position (WQ_IDLE: record load)
    uint64_t rec = 0, s = WQ_IDLE, x0 = 0, pb = 0;  // pb: 4-slot blocks probed for y
    Key y{0, 0};
    bool fetch = false;
    const uint64_t pb_max = (cap >> 2) + 1;  // every block once: y is absent (a full table)
    while (true) {
        // refill idle lanes from the queue (uniform loop: one region per sub-step)
        uint64_t idle = __ballot(rec == 0);
        while (idle && r < r_end) {
            const uint32_t nr = min(hn[r], hcap);
            if (id >= nr) {
                ++r;
                id = 0;
                continue;
            }
            const uint32_t take = min(nr - id, (uint32_t)__popcll(idle));
            const uint32_t rk = mbcnt64(idle);
            if (rec == 0 && rk < take) {
                rec = (uint64_t)r * hcap + id + rk + 1;
                fetch = true;
            }
            id += take;
            idle = __ballot(rec == 0);
        }
        if (!__any(rec != 0)) break;
        // loads: a fetching lane reads its record; a probing lane's quad reads its block
        const uint64_t sp = (rec && !fetch) ? s : WQ_IDLE;
        uint64_t sj[4], w0[4], w1[4];
        sj[0] = qbcast64<0>(sp);
        sj[1] = qbcast64<1>(sp);
        sj[2] = qbcast64<2>(sp);
        sj[3] = qbcast64<3>(sp);
        ulonglong2 rv = make_ulonglong2(0, 0);
        if (fetch) rv = *reinterpret_cast<const ulonglong2*>(headrec + (rec - 1) * 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            w0[j] = EMPTY;
            w1[j] = 0;
            const uint64_t my = (sj[j] & ~3ull) + q;
            if (sj[j] != WQ_IDLE && my < cap) load_slot_nt<W>(slots, my, w0[j], w1[j]);
        }
        uint64_t kh_[4], kl_[4];
        kh_[0] = qbcast64<0>(y.hi);
        kh_[1] = qbcast64<1>(y.hi);
        kh_[2] = qbcast64<2>(y.hi);
        kh_[3] = qbcast64<3>(y.hi);
        kl_[0] = qbcast64<0>(y.lo);
        kl_[1] = qbcast64<1>(y.lo);
        kl_[2] = qbcast64<2>(y.lo);
        kl_[3] = qbcast64<3>(y.lo);
        uint32_t myfh = 4, myfe = 4, myidx = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t my = (sj[j] & ~3ull) + q;
            const bool valid = sj[j] != WQ_IDLE && my >= sj[j] && my < cap;
            const bool empty = w0[j] == EMPTY;
            const bool hit = !empty & (slot_keybits(w0[j], p) == ((W == 1) ? kl_[j] : kh_[j])) &
                             ((W == 1) | (w1[j] == kl_[j]));
            const uint32_t bh = (uint32_t)(__ballot(valid && hit) >> ql) & 0xFu;
            const uint32_t be = (uint32_t)(__ballot(valid && empty) >> ql) & 0xFu;
            const uint32_t fh = bh ? (uint32_t)__builtin_ctz(bh) : 4u;
            const uint32_t fe = be ? (uint32_t)__builtin_ctz(be) : 4u;
            const uint32_t hx = qor32(q == fh ? slot_hidx(w0[j], p) : 0u);
            if (q == (uint32_t)j) {
                myfh = fh;
                myfe = fe;
                myidx = hx;
            }
        }
        if (rec) {
            bool done = false;
            uint32_t succ = 0;
            if (fetch) {
                x0 = rv.x;
                const uint32_t f = ext_fwd(slot_ext(rv.x));
                if (f <= 3u) {
                    y = key_next(slot_key(rv.x, rv.y, p), f, p);
                    s = home_of(place(y, p), cap, p);
                    pb = 0;
                } else {
                    done = true;  // the run ends its contig: no successor
                }
                fetch = false;
            } else if (myfh < myfe) {
                succ = myidx;
                done = true;
            } else if (myfe < 4u || ++pb > pb_max) {
                done = true;      // y is not in the table (the walker reports it)
            } else {
                const uint64_t nx = (s & ~3ull) + 4;
                s = nx >= cap ? 0 : nx;
            }
            if (done) {
                // one 64-bit store; walkers may read the record concurrently (side stream), which
                // is only allowed when the successor field lies in the upper dword (rec_succ_side)
                __hip_atomic_store(headrec + (rec - 1) * 2, (x0 & ((1ull << sh) - 1)) | ((uint64_t)succ << sh),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                rec = 0;
                s = WQ_IDLE;
            }
        }
    }
}

bool rec_succ_fits(const KParams& p, uint32_t hcap) {
    return p.chain && hcap && rec_succ_shift(p) < 64 && (uint64_t)hcap + 1 < (1ull << (64 - rec_succ_shift(p)));
}

// The resolve may run beside walkers that read records with 16-B vector loads only when the
// successor field lies entirely in the upper dword of word 0: a load that sees half of the
// resolve's 64-bit store then still reads either 0 or the whole index (the lower dword is
// rewritten with its own value). Below that (W=2 at k <= 40) it runs before the walk.
bool rec_succ_side(const KParams& p) { return rec_succ_shift(p) >= 32; }

hipError_t launch_rec_succ(const KParams& p, TableView t, uint64_t* headrec, uint32_t hcap, hipStream_t s,
                           unsigned blocks) {
    if (!rec_succ_fits(p, hcap)) return hipSuccess;
    // a wave per ~16 regions keeps its lanes' record queue full (the waves' ranges are contiguous)
    const unsigned grid = blocks ? blocks : (unsigned)hmin((nreg(p) + BLOCK / 64 - 1) / (BLOCK / 64), 8u * cu_count());
    if (p.W == 1)
        with_kt<1>(p.K, [&](auto kt) { k_rec_succ<1, decltype(kt)::value><<<grid, BLOCK, 0, s>>>(p, t.slots, t.cap, headrec, hcap); });
    else
        with_kt<2>(p.K, [&](auto kt) { k_rec_succ<2, decltype(kt)::value><<<grid, BLOCK, 0, s>>>(p, t.slots, t.cap, headrec, hcap); });
    return hipGetLastError();
}

hipError_t launch_walk(const KParams& p, TableView t, const WalkBuffers& wb, unsigned long long* ctr,
                       unsigned long long* stats, int grid_blocks, hipStream_t s) {
    const uint64_t nw = wb.n_starts + wb.n_splits;
    if (nw == 0) return hipSuccess;
    // two blocks per CU (512 on MI355X): with non-temporal probes fewer walkers in flight contend
    // less (C3 walk 5.71 -> 5.48-5.54 ms vs 2048 blocks, C2 0.67 -> 0.54; 384: 6.10)
    // grid_blocks <= 0: -grid_blocks blocks per CU (0: two). Walker blocks per CU, C3 walk ms:
    // 1: 1.78, 2: 1.32, 3: 1.24, 4: 1.37, 5: 1.50 (load 0.5); at load 0.85 three are slower than two
    // (2.39 vs 2.27: longer probe runs, more requests in flight contend); C2 (k=19) 0.37 vs 0.35
    const int bpc = grid_blocks < 0 ? -grid_blocks : 2;
    const unsigned grid = (unsigned)hmin((nw + BLOCK - 1) / BLOCK,
                                         (uint64_t)(grid_blocks > 0 ? grid_blocks : bpc * cu_count()));
    // queue batches per reservation: WALK_BATCHES where every wave gets many reservations, fewer
    // where a reservation of 8 x 64 walkers would leave most waves idle (the start walkers of a few
    // long contigs, C2: 12.7K of them, took 25 waves)
    WalkBuffers w = wb;
    if (w.batches == 0) {
        const uint64_t nq = !wb.split_min ? nw : wb.phase == 0 ? wb.n_starts : wb.n_splits;
        const uint64_t per = nq / ((uint64_t)WALK_GRAB * grid * (BLOCK / 64) * 4);
        w.batches = (uint32_t)(per < 1 ? 1 : hmin(per, (uint64_t)WALK_BATCHES));
    }
    if (p.W == 1)
        with_kt<1>(p.K, [&](auto kt) { k_walk_q<1, decltype(kt)::value><<<grid, BLOCK, 0, s>>>(p, t.slots, t.cap, w, ctr, stats); });
    else
        with_kt<2>(p.K, [&](auto kt) { k_walk_q<2, decltype(kt)::value><<<grid, BLOCK, 0, s>>>(p, t.slots, t.cap, w, ctr, stats); });
    return hipGetLastError();
}

__global__ __launch_bounds__(BLOCK) void k_fill(FillSet f) {
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    for (int j = 0; j < f.n; ++j) {
        uint32_t* q = reinterpret_cast<uint32_t*>(f.p[j]);
        const uint64_t words = f.bytes[j] / 4;
        const uint32_t v = f.byte[j] * 0x01010101u;
        for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < words; i += stride) q[i] = v;
    }
}

hipError_t launch_fill(const FillSet& f, hipStream_t s) {
    uint64_t most = 0;
    for (int j = 0; j < f.n; ++j) {
        if (f.bytes[j] % 4 || (reinterpret_cast<uintptr_t>(f.p[j]) & 3)) return hipErrorInvalidValue;
        most = f.bytes[j] > most ? f.bytes[j] : most;
    }
    if (!most) return hipSuccess;
    k_fill<<<(unsigned)hmin((most / 4 + BLOCK - 1) / BLOCK, 2048), BLOCK, 0, s>>>(f);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Materialisation: contig c occupies bytes [off[c], off[c] + K + len[c]) =
//   K chars of the start k-mer, len[c]-1 appended forward bases, '\n'.
template <int W>
__global__ __launch_bounds__(BLOCK) void k_write_heads(KParams p, const uint64_t* starts, uint64_t nc,
                                                       const uint32_t* len, const uint64_t* off,
                                                       char* out, uint64_t cap) {
    // 16 lanes per contig: lane l owns the aligned dword at (o & ~3) + 4l of the contig's K head
    // characters (o = its text offset), so a store instruction writes four contigs' heads as
    // contiguous runs; the first and last dword of a head are shared with the neighbouring text
    // (previous line, appended bases) and written byte by byte.
    constexpr uint32_t G = 16;
    static_assert(KMAX + 3 <= 4 * G, "a head spans at most 16 dwords");
    const uint32_t l = threadIdx.x & (G - 1);
    const uint64_t groups = (uint64_t)gridDim.x * (BLOCK / G);
    for (uint64_t c = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) / G; c < nc; c += groups) {
        const uint64_t w0 = starts[c * W];
        const uint64_t w1 = (W == 2) ? starts[c * W + 1] : 0;
        const Key k = slot_key(w0, w1, p);
        const uint64_t o = off[c];
        if (o + (uint64_t)p.K + len[c] > cap) continue;  // past the buffer: not written
        const uint32_t a = (uint32_t)(o & 3u);
        const int c0 = (int)(4 * l) - (int)a;  // first character of this lane's dword
        if (c0 < p.K) {
            uint32_t dw = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int j = c0 + b;
                const uint32_t code = (j >= 0 && j < p.K) ? key_base(k, j, p) : 0u;
                dw |= ((0x54474341u >> (8 * code)) & 0xFFu) << (8 * b);
            }
            char* d = out + (o - a) + 4 * (uint64_t)l;
            if (c0 >= 0 && c0 + 4 <= p.K) {
                *reinterpret_cast<uint32_t*>(d) = dw;
            } else {
                for (int b = 0; b < 4; ++b)
                    if (c0 + b >= 0 && c0 + b < p.K) d[b] = (char)(dw >> (8 * b));
            }
        }
        if (l == 0) out[o + p.K + len[c] - 1] = '\n';
    }
}

// ---- line writer (K >= 16): the text written in output order ---------------------------------
// A wave owns 1 KiB of the text and stores it with 16-B stores, one per lane, so every 64-B line is
// written whole, once, by one instruction. The heads + chunks writers above store each contig's
// head and its bases from two kernels at unaligned byte ranges: at C5 (21M contigs of ~60 bytes)
// nearly every line was written partially twice. Each lane finds the contig holding its first
// byte among the <= 62 contigs that start in the wave's KiB (contigs hold >= K + 1 >= 17 bytes) and
// builds its 16 characters from that contig and the next: head bases from the start k-mer, the
// bases of the contig's own first chunk (the first CHUNK_BASES bases of its first segment), '\n'.
// Bytes past those (longer segments, splitter segments) are left to the chunk writer, which runs
// after it on the same stream over the chunks it does not cover (chunk index >= n_starts).
static constexpr uint32_t LINE_BYTES = 1024;  // text bytes per wave
static constexpr uint32_t LINE_KMIN = 16;

// line_first[b] = the contig holding byte b * LINE_BYTES (b < ceil(min(total, cap) / LINE_BYTES))
__global__ __launch_bounds__(BLOCK) void k_line_first(int K, const uint32_t* clen, uint64_t nc, const uint64_t* off,
                                                      const unsigned long long* ctr, uint64_t cap, uint32_t* first) {
    const uint64_t lim = min((uint64_t)ctr[CT_OUT_BYTES], cap);
    for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < nc; c += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t o = off[c], e = min(o + (uint64_t)K + clen[c], lim);
        for (uint64_t b = (o + LINE_BYTES - 1) / LINE_BYTES; b * LINE_BYTES < e; ++b) first[b] = (uint32_t)c;
    }
}

// 32 bits of the 128-bit value (h:l) from bit s on; s < 0 shifts left (zeros come in)
__device__ __forceinline__ uint32_t bits32(uint64_t h, uint64_t l, int s) {
    if (s <= -32 || s >= 128) return 0u;
    if (s < 0) return (uint32_t)l << (-s);
    if (s >= 64) return (uint32_t)(h >> (s - 64));
    return s == 0 ? (uint32_t)l : (uint32_t)((l >> s) | (h << (64 - s)));
}

template <int W, int KT>
__global__ __launch_bounds__(BLOCK) void k_write_lines(KParams p_in, const uint64_t* __restrict__ starts, uint64_t nc,
                                                       const uint32_t* __restrict__ clen,
                                                       const uint32_t* __restrict__ slen,
                                                       const uint64_t* __restrict__ chunk_data, uint64_t chunk_cap,
                                                       const uint64_t* __restrict__ off,
                                                       const uint32_t* __restrict__ first,
                                                       const unsigned long long* ctr, char* __restrict__ out,
                                                       uint64_t cap, int slen_add) {
    // slen[c] + slen_add = k-mers of contig c's first segment (the migrating walk's origin passes
    // the bases it appended, slen_add = 1)
    const KParams p = specialize<KT>(p_in);
    const uint64_t lim = min((uint64_t)ctr[CT_OUT_BYTES], cap);
    const uint32_t lane = lane_id();
    const uint64_t nblk = (lim + LINE_BYTES - 1) / LINE_BYTES;
    const uint64_t waves = (uint64_t)gridDim.x * (BLOCK / 64);
    const int K = p.K;
    // U blocks per iteration, each stage's loads issued for all U before any is used: a block is a
    // chain of three dependent loads (first -> offsets -> the lane's contig), so one block at a time
    // left the kernel latency-bound (C5: ~160 blocks per wave)
    constexpr int U = 2;  // 4: C5 text 0.95 -> 1.01 ms, C3 0.30 -> 0.32 (profiles/r05/ab/ab_misc.txt)
    for (uint64_t blk0 = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) / 64; blk0 < nblk; blk0 += U * waves) {
        uint64_t c0[U], oj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c0[u] = first[min(blk0 + u * waves, nblk - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) oj[u] = c0[u] + lane < nc ? off[c0[u] + lane] : ~0ull;
        uint64_t x0[U], c[U], on[U];
        int64_t rc[U];
        uint32_t nb[U], hb[U];
        bool live[U], two[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t blk = blk0 + u * waves;
            x0[u] = blk * LINE_BYTES + 16u * lane;
            // the lane's contig: the last of the wave's 64 whose text starts at or before x0
            uint32_t lo = 0;
#pragma unroll
            for (uint32_t st = 32; st > 0; st >>= 1) {
                const uint64_t v = __shfl(oj[u], (int)(lo + st), 64);
                if (v <= x0[u]) lo += st;
            }
            const uint64_t oc = __shfl(oj[u], (int)lo, 64), onx = __shfl(oj[u], (int)min(lo + 1, 63u), 64);
            on[u] = lo < 63 ? onx : ~0ull;  // lo <= 61 for K >= 16
            live[u] = blk < nblk && x0[u] < lim;
            c[u] = c0[u] + lo;
            two[u] = on[u] < x0[u] + 16 && c[u] + 1 < nc;  // the next contig starts inside these 16 bytes
            rc[u] = (int64_t)(x0[u] - oc);
            nb[u] = two[u] ? (uint32_t)(on[u] - x0[u]) : 16u;  // bytes of contig c
            hb[u] = rc[u] >= K ? 0u : (uint32_t)min<int64_t>(K - rc[u], nb[u]);
        }
        // 2-bit codes of the 16 bytes (byte b at bits 2b), then 4 characters per v_perm_b32: the
        // selector bytes are codes (0-3: "ACGT") or 4 ('\n'). Contig c holds bytes [0, nb): head
        // bases [0, hb), then first-chunk bases (bytes past the chunk are the chunk writer's), '\n'
        // at nl; contig c + 1 bytes [nb, 16), all head bases (nb >= 1, 16 - nb < K).
        auto head_low = [&](uint64_t w0, uint64_t w1, int64_t rel0) {  // head base rel0 + b at bits 2b
            const Key k = slot_key(w0, w1, p);
            const uint64_t vl = k.lo | (k.hi << 62), vh = k.hi >> 2;  // V as 128 bits
            uint32_t r = __builtin_bitreverse32(bits32(vh, vl, 2 * (K - 16 - (int)rel0)));
            return ((r >> 1) & 0x55555555u) | ((r & 0x55555555u) << 1);  // 2-bit groups reversed
        };
        uint64_t kc0[U], kc1[U], kn0[U], kn1[U], d0[U], d1[U];
        uint32_t cl[U], sl[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // every load of both blocks before any use
            const uint64_t cc = live[u] ? c[u] : 0, cn = live[u] && two[u] ? c[u] + 1 : cc;
            kc0[u] = starts[cc * W];
            kc1[u] = W == 2 ? starts[cc * W + 1] : 0;
            kn0[u] = starts[cn * W];
            kn1[u] = W == 2 ? starts[cn * W + 1] : 0;
            cl[u] = clen[cc];
            sl[u] = slen[cc];
            const int64_t j0 = rc[u] - K;
            const uint32_t w = j0 > 0 ? (uint32_t)min<int64_t>(j0 / 32, CHUNK_WORDS - 1) : 0u;
            const bool need = live[u] && hb[u] < nb[u] && j0 < CHUNK_BASES;
            d0[u] = need ? chunk_data[chunk_word(cc, w, chunk_cap)] : 0ull;
            d1[u] = need && w + 1 < CHUNK_WORDS ? chunk_data[chunk_word(cc, w + 1, chunk_cap)] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;
            uint32_t codes = hb[u] ? head_low(kc0[u], kc1[u], rc[u]) : 0u;
            if (hb[u] < nb[u]) {  // first-chunk bases j0 + b
                const int64_t A = min<int64_t>((int64_t)sl[u] + slen_add - 1, CHUNK_BASES), j0 = rc[u] - K;
                if (j0 + 16 > 0 && j0 < A) {
                    const uint32_t w = j0 > 0 ? (uint32_t)(j0 / 32) : 0u;
                    const uint32_t bw = bits32(d1[u], d0[u], (int)(2 * (j0 - 32 * (int64_t)w)));
                    const uint32_t mh = hb[u] ? 0xFFFFFFFFu >> (32 - 2 * hb[u]) : 0u;
                    codes = (codes & mh) | (bw & ~mh);
                }
            }
            if (two[u]) {
                const uint32_t mn = 0xFFFFFFFFu << (2 * nb[u]);
                codes = (codes & ~mn) | ((head_low(kn0[u], kn1[u], 0) << (2 * nb[u])) & mn);
            }
            const int64_t nl = (int64_t)K + cl[u] - 1 - rc[u];
            uint32_t v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t x = (codes >> (8 * i)) & 0xFFu;
                uint32_t sel = (x & 3u) | ((x << 6) & 0x300u) | ((x << 12) & 0x30000u) | ((x << 18) & 0x3000000u);
                if (nl >= 4 * i && nl < 4 * i + 4 && nl < nb[u])
                    sel = (sel & ~(0xFFu << (8 * (nl - 4 * i)))) | (4u << (8 * (nl - 4 * i)));
                v[i] = __builtin_amdgcn_perm(0x0A0A0A0Au, 0x54474341u, sel);
            }
            if (x0[u] + 16 <= lim) {
                *reinterpret_cast<uint4*>(out + x0[u]) = make_uint4(v[0], v[1], v[2], v[3]);
            } else {
                for (uint32_t b = 0; x0[u] + b < lim; ++b) out[x0[u] + b] = (char)(v[b >> 2] >> (8 * (b & 3)));
            }
        }
    }
}

// 64 bits of the 128-bit value (h:l) from bit s on, -64 < s < 64; s < 0 shifts left (zeros come in)
__device__ __forceinline__ uint64_t bits64(uint64_t h, uint64_t l, int s) {
    if (s < 0) return l << (-s);
    return s == 0 ? l : (l >> s) | (h << (64 - s));
}

// The line writer at K >= 32: a wave owns 2 KiB of the text and a lane 32 contiguous bytes (two
// 16-B stores). Contigs then hold >= 33 bytes, so a lane's 32 bytes still touch at most two
// contigs (c, and the head of c + 1) and the <= 63 contigs that start in the wave's 2 KiB fit the
// wave's 64 lanes. Per byte this halves what the 16-byte version repeats per lane — the contig
// search, the key unpacks, the record loads — which is what bound it: VALU-bound at C5's
// 60-byte lines (~280 VALU per 16-B lane store). line_first is the 1-KiB table (entry 2b).
static constexpr uint32_t LINE2_BYTES = 2048;
static constexpr int LINE2_KMIN = 32;

template <int W, int KT>
__global__ __launch_bounds__(BLOCK) void k_write_lines32(KParams p_in, const uint64_t* __restrict__ starts, uint64_t nc,
                                                         const uint32_t* __restrict__ clen,
                                                         const uint32_t* __restrict__ slen,
                                                         const uint64_t* __restrict__ chunk_data, uint64_t chunk_cap,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ first,
                                                         const unsigned long long* ctr, char* __restrict__ out,
                                                         uint64_t cap, int slen_add) {
    const KParams p = specialize<KT>(p_in);
    const uint64_t lim = min((uint64_t)ctr[CT_OUT_BYTES], cap);
    const uint32_t lane = lane_id();
    const uint64_t nblk = (lim + LINE2_BYTES - 1) / LINE2_BYTES;
    const uint64_t waves = (uint64_t)gridDim.x * (BLOCK / 64);
    const int K = p.K;
    const uint32_t xr = 32u * lane;  // the lane's first byte, relative to the block
    constexpr int U = 2;
    for (uint64_t blk0 = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) / 64; blk0 < nblk; blk0 += U * waves) {
        uint64_t c0[U], oj[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c0[u] = first[2 * min(blk0 + u * waves, nblk - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u) oj[u] = c0[u] + lane < nc ? off[c0[u] + lane] : ~0ull;
        uint64_t x0[U], c[U];
        int64_t rc[U];
        uint32_t nb[U], hb[U];
        bool live[U], two[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t blk = blk0 + u * waves, B = blk * LINE2_BYTES;
            x0[u] = B + xr;
            // offsets relative to the block as 32-bit (contig c0 starts at or before B: 0; past
            // the contigs: the maximum), so the search shuffles and compares 32-bit values
            const uint64_t rel = oj[u] - B;
            const uint32_t r32 = oj[u] <= B ? 0u : rel > 0x7fffffffull ? 0x7fffffffu : (uint32_t)rel;
            uint32_t lo = 0;
#pragma unroll
            for (uint32_t st = 32; st > 0; st >>= 1) {
                const uint32_t v = (uint32_t)__shfl((int)r32, (int)(lo + st), 64);
                if (v <= xr) lo += st;
            }
            const uint32_t rn = (uint32_t)__shfl((int)r32, (int)min(lo + 1, 63u), 64);
            const uint64_t oc0 = __shfl(oj[u], 0, 64);
            const uint32_t rl = (uint32_t)__shfl((int)r32, (int)lo, 64);
            live[u] = blk < nblk && x0[u] < lim;
            c[u] = c0[u] + lo;
            two[u] = lo < 63 && rn < xr + 32 && c[u] + 1 < nc;  // the next contig starts inside these 32 bytes
            rc[u] = lo ? (int64_t)(xr - rl) : (int64_t)(x0[u] - oc0);
            nb[u] = two[u] ? rn - xr : 32u;  // bytes of contig c
            hb[u] = rc[u] >= K ? 0u : min((uint32_t)(K - rc[u]), nb[u]);
        }
        auto head64 = [&](uint64_t w0, uint64_t w1, int rel0) {  // head base rel0 + b at bits 2b
            const Key k = slot_key(w0, w1, p);
            const uint64_t vl = k.lo | (k.hi << 62), vh = k.hi >> 2;  // V as 128 bits
            return rev2_64(bits64(vh, vl, 2 * (K - 32 - rel0)));
        };
        uint64_t kc0[U], kc1[U], kn0[U], kn1[U], d0[U], d1[U];
        uint32_t cl[U], sl[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // every load of both blocks before any use
            const uint64_t cc = live[u] ? c[u] : 0, cn = live[u] && two[u] ? c[u] + 1 : cc;
            kc0[u] = starts[cc * W];
            kc1[u] = W == 2 ? starts[cc * W + 1] : 0;
            kn0[u] = starts[cn * W];
            kn1[u] = W == 2 ? starts[cn * W + 1] : 0;
            cl[u] = clen[cc];
            sl[u] = slen[cc];
            const int64_t j0 = rc[u] - K;
            const uint32_t w = j0 > 0 ? (uint32_t)min<int64_t>(j0 / 32, CHUNK_WORDS - 1) : 0u;
            const bool need = live[u] && hb[u] < nb[u] && j0 < CHUNK_BASES;
            d0[u] = need ? chunk_data[chunk_word(cc, w, chunk_cap)] : 0ull;
            d1[u] = need && w + 1 < CHUNK_WORDS ? chunk_data[chunk_word(cc, w + 1, chunk_cap)] : 0ull;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!live[u]) continue;
            // the head (rc < K, so rel0 >= 0 and hb >= 1 bytes of it)
            uint64_t codes = hb[u] ? head64(kc0[u], kc1[u], (int)rc[u]) : 0ull;
            if (hb[u] < nb[u]) {  // first-chunk bases j0 + b
                const int64_t A = min<int64_t>((int64_t)sl[u] + slen_add - 1, CHUNK_BASES), j0 = rc[u] - K;
                if (j0 + 32 > 0 && j0 < A) {
                    const uint32_t w = j0 > 0 ? (uint32_t)(j0 / 32) : 0u;
                    const uint64_t bw = bits64(d1[u], d0[u], (int)(2 * (j0 - 32 * (int64_t)w)));
                    const uint64_t mh = hb[u] ? ~0ull >> (64 - 2 * hb[u]) : 0ull;
                    codes = (codes & mh) | (bw & ~mh);
                }
            }
            if (two[u]) {  // 32 - nb < 32 <= K: all of them head bases of contig c + 1
                const uint64_t mn = ~0ull << (2 * nb[u]);
                codes = (codes & ~mn) | ((head64(kn0[u], kn1[u], 0) << (2 * nb[u])) & mn);
            }
            const int64_t nl64 = (int64_t)K + cl[u] - 1 - rc[u];
            // '\n' as selector bit 2 (selector 4 | code picks a byte of 0x0A0A0A0A): one bit per byte
            const uint32_t nlm = (nl64 >= 0 && nl64 < (int64_t)nb[u]) ? 1u << (uint32_t)nl64 : 0u;
            uint32_t v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                // 4 codes (2 bits each) spread to the low bits of 4 selector bytes
                const uint32_t x = (uint32_t)(codes >> (8 * i)) & 0xFFu;
                const uint32_t t = (x | (x << 12)) & 0x000F000Fu;
                const uint32_t nib = (nlm >> (4 * i)) & 0xFu;
                const uint32_t sel = ((t | (t << 6)) & 0x03030303u) | (((nib * 0x00204081u) & 0x01010101u) << 2);
                v[i] = __builtin_amdgcn_perm(0x0A0A0A0Au, 0x54474341u, sel);
            }
            if (x0[u] + 32 <= lim) {
                *reinterpret_cast<uint4*>(out + x0[u]) = make_uint4(v[0], v[1], v[2], v[3]);
                *reinterpret_cast<uint4*>(out + x0[u] + 16) = make_uint4(v[4], v[5], v[6], v[7]);
            } else {
                for (uint32_t b = 0; x0[u] + b < lim; ++b) out[x0[u] + b] = (char)(v[b >> 2] >> (8 * (b & 3)));
            }
        }
    }
}

__global__ __launch_bounds__(BLOCK) void k_write_chunks(int K, const uint64_t* chunk_data,
                                                        const uint32_t* owner, const uint32_t* seq,
                                                        const unsigned long long* ctr,
                                                        uint64_t chunk_cap, uint64_t n_first,
                                                        const uint32_t* len,
                                                        const uint64_t* off, char* out, uint64_t cap,
                                                        uint64_t ch_begin = 0) {
    // Chunks [0, n_first) are the contigs' own first chunks; the extra-chunk count is only known
    // on the device (walker allocation head), so the grid is sized for the capacity and bounded
    // here.
    const uint64_t nchunks = min(n_first + (uint64_t)ctr[CT_CHUNK_NEXT], chunk_cap);
    const uint64_t nwords = nchunks * CHUNK_WORDS;
    for (uint64_t t = ch_begin * CHUNK_WORDS + (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < nwords;
         t += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t ch = t / CHUNK_WORDS;
        const uint32_t w = (uint32_t)(t % CHUNK_WORDS);
        const uint32_t c = ch < n_first ? (uint32_t)ch : owner[ch];
        const uint64_t j0 = (ch < n_first ? 0ull : (uint64_t)seq[ch] * CHUNK_BASES) + (uint64_t)w * 32;
        const uint64_t app = (uint64_t)len[c] - 1;
        if (j0 >= app) continue;
        const uint32_t cntb = (uint32_t)min<uint64_t>(32, app - j0);
        if (off[c] + K + j0 + cntb > cap) continue;
        const uint64_t word = chunk_data[chunk_word(ch, w, chunk_cap)];
        char* o = out + off[c] + K + j0;
        store_chars(o, cntb, [&](uint32_t i) { return codes4_chars((uint32_t)(word >> (8 * i)) & 0xFFu); });
    }
}

// ---------------------------------------------------------------------------------------------
// Text parse (read_kmers.hpp:62-76 + packKmer, packing.hpp:77-92). A block stages 256 lines
// through LDS with aligned 16-B loads (lines are K+4 bytes, unaligned), packs each line's K
// bases in a register pair, and stores its 256 records back with 16-B stores.
static constexpr int TXT_MAX_LINE = KMAX + 4;

__global__ __launch_bounds__(BLOCK) void k_pack_text(KParams p, const char* __restrict__ text, uint64_t n,
                                                     uint8_t* __restrict__ recs, unsigned long long* stats) {
    __shared__ uint4 in_st[(BLOCK * TXT_MAX_LINE + 32) / 16];
    __shared__ uint4 out_st[(BLOCK * 17 + 16) / 16];
    __shared__ uint32_t bad;
    const uint32_t Lb = (uint32_t)p.K + 4, R = (uint32_t)p.R;
    const uint64_t end = n * Lb;  // bytes of complete lines: never read past them
    if (threadIdx.x == 0) bad = 0;
    for (uint64_t sub = (uint64_t)blockIdx.x * BLOCK; sub < n; sub += (uint64_t)gridDim.x * BLOCK) {
        const uint32_t cnt = n - sub < (uint64_t)BLOCK ? (uint32_t)(n - sub) : (uint32_t)BLOCK;
        const int64_t a = (int64_t)(sub * Lb), b = a + (int64_t)cnt * Lb, e = (int64_t)end;
        const uint32_t mis = (uint32_t)((uintptr_t)(text + a) & 15u);
        const int64_t a0 = a - mis;                    // precedes the buffer only when a == 0
        const uint32_t nv = (uint32_t)((b - a0 + 15) / 16);
        __syncthreads();
        for (uint32_t v = threadIdx.x; v < nv; v += BLOCK) {
            const int64_t lo = a0 + (int64_t)v * 16;
            if (lo >= a && lo + 16 <= e) {
                in_st[v] = *reinterpret_cast<const uint4*>(text + lo);
            } else {  // partial vector at either edge of the text: byte loads inside [a, end)
                uint8_t* d = reinterpret_cast<uint8_t*>(&in_st[v]);
                for (int x = 0; x < 16; ++x) d[x] = (lo + x >= a && lo + x < e) ? (uint8_t)text[lo + x] : 0;
            }
        }
        __syncthreads();
        if (threadIdx.x < cnt) {
            const uint8_t* l = reinterpret_cast<const uint8_t*>(in_st) + mis + threadIdx.x * Lb;
            uint64_t hi = 0, lo = 0;  // V = hi:lo, 2 bits per base, base 0 most significant
            uint32_t badl = 0;
            for (int i = 0; i < p.K; ++i) {
                const uint32_t c = base_code(l[i]);
                badl |= c > 3;
                hi = (hi << 2) | (lo >> 62);
                lo = (lo << 2) | (c & 3u);
            }
            if (badl) atomicAdd(&bad, 1u);
            const Key k{(hi << 2) | (lo >> 62), lo & LO_MASK};
            uint8_t* o = reinterpret_cast<uint8_t*>(out_st) + threadIdx.x * R;
            key_to_packed(k, o, p);
            o[p.P] = l[p.K + 1];
            o[p.P + 1] = l[p.K + 2];
        }
        __syncthreads();
        const uint32_t ob = cnt * R, onv = ob >> 4;
        uint8_t* dst = recs + sub * R;  // 16-B aligned: sub is a multiple of 256, recs aligned
        for (uint32_t v = threadIdx.x; v < onv; v += BLOCK) reinterpret_cast<uint4*>(dst)[v] = out_st[v];
        for (uint32_t x = (onv << 4) + threadIdx.x; x < ob; x += BLOCK)
            dst[x] = reinterpret_cast<const uint8_t*>(out_st)[x];
    }
    __syncthreads();
    if (threadIdx.x == 0 && bad) atomicAdd(&stats[ST_BAD_BASE], (unsigned long long)bad);
}

hipError_t launch_pack_text(const KParams& p, const char* text, uint64_t n, uint8_t* recs,
                            unsigned long long* stats, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)hmin((n + BLOCK - 1) / BLOCK, 4096);
    k_pack_text<<<g, BLOCK, 0, s>>>(p, text, n, recs, stats);
    return hipGetLastError();
}

hipError_t launch_contig_offsets(int K, const uint32_t* len, uint64_t nc, uint64_t* offsets,
                                 uint64_t* scratch, unsigned long long* total, hipStream_t s) {
    return scan_exclusive(ContigBytesF{len, (uint64_t)K}, nc, offsets, scratch, (unsigned long long*)nullptr,
                          total, s);
}

hipError_t launch_write_heads(const KParams& p, const uint64_t* starts, uint64_t nc, const uint32_t* len,
                              const uint64_t* offsets, char* out, hipStream_t s, uint64_t cap) {
    if (nc == 0) return hipSuccess;
    const unsigned gh = (unsigned)hmin((nc * 16 + BLOCK - 1) / BLOCK, 65536);  // 16 lanes per contig
    if (p.W == 1)
        k_write_heads<1><<<gh, BLOCK, 0, s>>>(p, starts, nc, len, offsets, out, cap);
    else
        k_write_heads<2><<<gh, BLOCK, 0, s>>>(p, starts, nc, len, offsets, out, cap);
    return hipGetLastError();
}

// The line writer for the contigs' heads, first chunks and newlines (K >= 16, line_first sized
// out_bytes / LINE_BYTES + 2 entries); false: the heads writer instead.
static bool launch_lines(const KParams& p, const WalkBuffers& wb, const uint32_t* clen, const uint64_t* offsets,
                         char* out, const unsigned long long* ctr, hipStream_t s, uint64_t cap, uint32_t* line_first,
                         uint64_t out_bytes, int slen_add = 0) {
    const uint64_t nc = wb.n_starts;
    if (!line_first || p.K < (int)LINE_KMIN) return false;
    const unsigned gf = (unsigned)hmin((nc + BLOCK - 1) / BLOCK, 8192);
    k_line_first<<<gf, BLOCK, 0, s>>>(p.K, clen, nc, offsets, ctr, cap, line_first);
    if (p.K >= LINE2_KMIN) {
        const uint64_t waves2 = (min(out_bytes, cap) + LINE2_BYTES - 1) / LINE2_BYTES;
        const unsigned g2 = (unsigned)hmin((waves2 + BLOCK / 64 - 1) / (BLOCK / 64) + 1, 8192);
        if (p.W == 1)
            with_kt<1>(p.K, [&](auto kt) {
                k_write_lines32<1, decltype(kt)::value><<<g2, BLOCK, 0, s>>>(
                    p, wb.starts, nc, clen, wb.contig_len, wb.chunk_data, wb.chunk_cap, offsets, line_first, ctr, out,
                    cap, slen_add);
            });
        else
            with_kt<2>(p.K, [&](auto kt) {
                k_write_lines32<2, decltype(kt)::value><<<g2, BLOCK, 0, s>>>(
                    p, wb.starts, nc, clen, wb.contig_len, wb.chunk_data, wb.chunk_cap, offsets, line_first, ctr, out,
                    cap, slen_add);
            });
        return true;
    }
    const uint64_t waves = (min(out_bytes, cap) + LINE_BYTES - 1) / LINE_BYTES;
    const unsigned gl = (unsigned)hmin((waves + BLOCK / 64 - 1) / (BLOCK / 64) + 1, 8192);
    if (p.W == 1)
        with_kt<1>(p.K, [&](auto kt) {
            k_write_lines<1, decltype(kt)::value><<<gl, BLOCK, 0, s>>>(p, wb.starts, nc, clen, wb.contig_len, wb.chunk_data,
                                                                      wb.chunk_cap, offsets, line_first, ctr, out, cap,
                                                                      slen_add);
        });
    else
        with_kt<2>(p.K, [&](auto kt) {
            k_write_lines<2, decltype(kt)::value><<<gl, BLOCK, 0, s>>>(p, wb.starts, nc, clen, wb.contig_len, wb.chunk_data,
                                                                      wb.chunk_cap, offsets, line_first, ctr, out, cap,
                                                                      slen_add);
        });
    return true;
}

bool launch_text_lines(const KParams& p, const WalkBuffers& wb, const uint32_t* clen, int slen_add,
                       const uint64_t* offsets, char* out, const unsigned long long* ctr, hipStream_t s, uint64_t cap,
                       uint32_t* line_first, uint64_t out_bytes) {
    return launch_lines(p, wb, clen, offsets, out, ctr, s, cap, line_first, out_bytes, slen_add);
}

hipError_t launch_materialize(const KParams& p, const WalkBuffers& wb, uint64_t* offsets,
                              uint64_t* scratch, char* out, unsigned long long* ctr, hipStream_t s,
                              int phases, uint32_t* line_first, uint64_t out_bytes) {
    const uint64_t nc = wb.n_starts;
    if (nc == 0) return hipSuccess;
    if (phases & MAT_SCAN) {
        hipError_t e = scan_exclusive(ContigBytesF{wb.contig_len, (uint64_t)p.K}, nc, offsets, scratch,
                                      (unsigned long long*)nullptr, &ctr[CT_OUT_BYTES], s);
        if (e != hipSuccess) return e;
    }
    if (!(phases & MAT_WRITE)) return hipSuccess;
    const uint64_t cap = wb.text_cap ? wb.text_cap : ~0ull;
    const bool lines = launch_lines(p, wb, wb.contig_len, offsets, out, ctr, s, cap, line_first, out_bytes);
    if (!lines) {
        const unsigned gh = (unsigned)hmin((nc * 16 + BLOCK - 1) / BLOCK, 65536);  // 16 lanes per contig
        if (p.W == 1)
            k_write_heads<1><<<gh, BLOCK, 0, s>>>(p, wb.starts, nc, wb.contig_len, offsets, out, cap);
        else
            k_write_heads<2><<<gh, BLOCK, 0, s>>>(p, wb.starts, nc, wb.contig_len, offsets, out, cap);
    }
    // chunks the line writer does not cover: every contig's chunks past its first
    const uint64_t cb = lines ? nc : 0;
    const unsigned gc =
        (unsigned)hmin(((wb.chunk_cap - min(cb, wb.chunk_cap)) * CHUNK_WORDS + BLOCK - 1) / BLOCK + 1, 8192);
    k_write_chunks<<<gc, BLOCK, 0, s>>>(p.K, wb.chunk_data, wb.chunk_owner, wb.chunk_seq, ctr,
                                        wb.chunk_cap, nc, wb.contig_len, offsets, out, cap, cb);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Splitter segments (sparse ruling set). With p.split_bits > 0 every k-mer whose hash has
// split_bits low zero bits (and that is not a contig start) heads a segment walked by its own
// lane, and walkers stop before such a k-mer. A contig of L k-mers then costs ~L / 2^split_bits
// dependent steps on its critical path instead of L (C5 chains of 10^6 k-mers;
// C2 chains of ~800 walked by only ~13 K lanes). Afterwards each segment's successor is looked
// up in a small splitter table and each contig's chain of segments is followed once.
// The splitter table holds 2x the walked splitters (+64): sized on the device from the walked count
// (C3: 49K of the 780K collected, whose bound sizes the allocation), so it stays in L2.
__device__ __forceinline__ uint64_t stab_cap(const WalkBuffers& wb, uint64_t cap2) {
    return min(cap2, 2 * walk_splits(wb) + 64);
}
// Deferred splitter segments (wb.split_min): the table is needed only if some contig stopped at a
// splitter (seg_long[0]). Beside the walk it is built when that is already known (C5: the long
// chains stop early), else after the walk if it turned out so (seg_long[2]: built beside; [3]: this
// launch builds it). C3 never builds it (it was the critical path of the walk phase: resolve 0.98
// + table 0.09 ms beside a 0.99-ms walk).
__global__ void k_stab_gate(uint32_t* seg_long, int after) {
    if (threadIdx.x || blockIdx.x) return;
    const uint32_t f = __hip_atomic_load(seg_long, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t go = after ? (f && !seg_long[2]) : f;
    if (!after) seg_long[2] = go;
    seg_long[3] = go;
}
__global__ __launch_bounds__(BLOCK) void k_stab_init(WalkBuffers wb, uint64_t* stab, uint64_t cap2_max) {
    if (wb.split_min && !wb.seg_long[3]) return;
    const uint64_t cap2 = stab_cap(wb, cap2_max);
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < cap2; i += (uint64_t)gridDim.x * BLOCK)
        stab[2 * i] = EMPTY;
}
__global__ __launch_bounds__(BLOCK) void k_stab_build(KParams p, WalkBuffers wb, uint64_t* stab, uint32_t* id,
                                                      uint64_t cap2_max) {
    if (wb.split_min && !wb.seg_long[3]) return;
    const uint64_t* splits = wb.splits;
    const uint64_t nsp = walk_splits(wb);
    const uint64_t cap2 = stab_cap(wb, cap2_max);
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nsp; i += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t w0 = splits[i * p.W], w1 = p.W == 2 ? splits[i * p.W + 1] : 0;
        const Key k = slot_key(w0, w1, p);
        uint64_t s = mulhi64(fmix64(key_hash(k)), cap2);
        while (true) {  // lo < 2^62 is never EMPTY; keys are unique (table invariant)
            const unsigned long long old =
                atomicCAS((unsigned long long*)&stab[2 * s], (unsigned long long)EMPTY, (unsigned long long)k.lo);
            if (old == EMPTY) {
                stab[2 * s + 1] = k.hi;
                id[s] = (uint32_t)i;
                break;
            }
            s = (s + 1 == cap2) ? 0 : s + 1;
        }
    }
}

// The successor of every segment a walker ended before a splitter (SEG_AT_SPLIT + its key), from
// the splitter table, all segments in parallel. Resolving lazily inside k_seg_chain instead (one
// lookup per hop on the contig's serial path) measured C3 -0.03 ms but C2 (~80 segments per
// contig) 0.60 -> 1.00 ms walk bracket (profiles/r05/ab/ab_seg_lazy_link.txt).
__global__ __launch_bounds__(BLOCK) void k_seg_link(WalkBuffers wb, SegBuffers sb, unsigned long long* stats) {
    if (wb.split_min && !*wb.seg_long) return;  // no walker stopped at a splitter
    const uint64_t nseg = wb.n_starts + walk_splits(wb);
    const uint64_t cap2 = stab_cap(wb, sb.cap2);
    // most segments end at 'F' (C5: 21M of 21.8M): a thread tests 4 with one 16-B load (seg_next
    // is 16-B aligned, its allocation rounded up to 4 entries)
    for (uint64_t g4 = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; 4 * g4 < nseg; g4 += (uint64_t)gridDim.x * BLOCK) {
        const uint4 v = reinterpret_cast<const uint4*>(wb.seg_next)[g4];
        if (v.x != SEG_AT_SPLIT && v.y != SEG_AT_SPLIT && v.z != SEG_AT_SPLIT && v.w != SEG_AT_SPLIT) continue;
        for (uint64_t g = 4 * g4; g < min(4 * g4 + 4, nseg); ++g) {
        if (wb.seg_next[g] != SEG_AT_SPLIT) continue;
        const Key k{wb.seg_key[2 * g], wb.seg_key[2 * g + 1]};
        uint64_t s = mulhi64(fmix64(key_hash(k)), cap2);
        uint32_t nx = SEG_NONE;
        for (uint64_t pr = 0; pr < cap2; ++pr) {
            const uint64_t lo = sb.stab[2 * s];
            if (lo == EMPTY) break;
            if (lo == k.lo && sb.stab[2 * s + 1] == k.hi) {
                nx = (uint32_t)(wb.n_starts + sb.stab_id[s]);
                break;
            }
            s = (s + 1 == cap2) ? 0 : s + 1;
        }
        // not a collected splitter: a start k-mer that passes split_test (starts are not collected),
        // reached by another contig's walk (overlapping walks, malformed input: the reference walks
        // on through it, kmer_hash.cpp:44 tests only the forward extension), or a k-mer missing from
        // the table. Both are counted as an overlap: kh_assemble redoes the walk unsegmented, whose
        // walker steps through the start and reports a k-mer that is really missing.
        if (nx == SEG_NONE) atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
        wb.seg_next[g] = nx;
        }
    }
}

// Each contig's chain of segments -> its length and every segment's contig and base offset.
// One thread per contig walks its chain serially for up to SEG_SERIAL segments (C3: 1-3, C2: ~80).
// Longer chains (C5: ~4K segments per 10^6-k-mer chain, 2 ms as one serial walk) raise a flag and
// continue over jump pointers: every segment gets a pointer SEG_JUMP links ahead and the bases of
// those links (k_seg_jump, all segments in parallel); the contig walks the jump pointers only,
// marking the segments it lands on (k_seg_chain_jump); each marked segment fills in the
// SEG_JUMP - 1 segments after it (k_seg_fill). Without the flag those three kernels return at once.
// C5 (chains of ~3.9K segments): 256 serial + 228 jumps of 16 = ~500 dependent hops (seg_chain 0.36 +
// chain_jump 0.27 ms); 128 serial + jumps of 64 (~sqrt of the chain) + 64-hop jump and fill passes: ~320
// (32 / 64 serial hops: C5 -0.08 / 0 ms but C2 1.24 -> 1.44 / 1.46 ms: C2's ~100-segment contigs then
// take the jump passes; profiles/r05/ab/ab_misc.txt)
// Round 6: the serial prefix is SegBuffers::serial — SEG_SERIAL where contigs average many
// segments (C2: ~50 walked splitters per start), SEG_SERIAL_FEW where long chains are rare
// outliers among single-segment contigs (C5: 0.04 per start), whose few chains take the jump
// passes anyway: 128 + 61 + 64 dependent hops become 32 + 61 + 64.
static constexpr uint32_t SEG_SERIAL = 128, SEG_SERIAL_FEW = 32, SEG_JUMP = 64;
__global__ __launch_bounds__(BLOCK) void k_seg_chain(WalkBuffers wb, SegBuffers sb, unsigned long long* stats) {
    const uint64_t nseg = wb.n_starts + walk_splits(wb);
    for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < wb.n_starts; c += (uint64_t)gridDim.x * BLOCK) {
        uint32_t g = (uint32_t)c;
        uint64_t off = 0, hops = 0;
        uint32_t pend = SEG_NONE;
        while (true) {
            // a segment another contig reached first: two walks overlap (malformed input); the
            // segment text would be written once, so kh_assemble redoes the walk unsegmented.
            // Segment links lead to splitter segments only, so the contig's own start segment is
            // reached by this thread alone: a plain store (C5: 21M atomics fewer)
            // (segment c < n_starts is contig c's own start segment at offset 0: not stored)
            if (hops) {
                if (atomicExch(&sb.seg_contig[g], (uint32_t)c) != SEG_NONE) atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
                sb.seg_off[g] = (uint32_t)off;
            }
            off += wb.contig_len[g] - 1;
            g = wb.seg_next[g];
            if (g == SEG_NONE) break;
            if (++hops > nseg || off > wb.max_steps) {  // segments in a cycle
                atomicAdd(&stats[ST_CYCLE], 1ull);
                break;
            }
            if (hops == sb.serial) {  // a long chain: the rest goes over jump pointers
                pend = g;
                *sb.long_flag = 1u;
                break;
            }
        }
        sb.pend[c] = pend;
        sb.clen[c] = (uint32_t)(off + 1);  // pending: the bases before segment pend
    }
}

// (jump pointers and anchors are splitter segments' only: a long chain continues past its start
// segment through splitter segments, and k_seg_chain_jump starts at one)
__global__ __launch_bounds__(BLOCK) void k_seg_jump(WalkBuffers wb, SegBuffers sb) {
    if (!*sb.long_flag) return;
    const uint64_t nseg = wb.n_starts + walk_splits(wb);
    for (uint64_t i = wb.n_starts + (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nseg;
         i += (uint64_t)gridDim.x * BLOCK) {
        uint32_t g = (uint32_t)i, sum = 0;
        for (uint32_t h = 0; h < SEG_JUMP && g != SEG_NONE; ++h) {
            sum += wb.contig_len[g] - 1;
            g = wb.seg_next[g];
        }
        sb.jump[i] = g;
        sb.jsum[i] = sum;
        sb.anchor[i] = 0;
    }
}

__global__ __launch_bounds__(BLOCK) void k_seg_chain_jump(WalkBuffers wb, SegBuffers sb, unsigned long long* stats) {
    if (!*sb.long_flag) return;
    const uint64_t nseg = wb.n_starts + walk_splits(wb);
    for (uint64_t c = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; c < wb.n_starts; c += (uint64_t)gridDim.x * BLOCK) {
        uint32_t g = sb.pend[c];
        if (g == SEG_NONE) continue;
        uint64_t off = sb.clen[c] - 1, hops = 0;
        while (true) {
            if (atomicExch(&sb.seg_contig[g], (uint32_t)c) != SEG_NONE) atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
            sb.seg_off[g] = (uint32_t)off;
            sb.anchor[g] = 1;
            off += sb.jsum[g];
            g = sb.jump[g];
            if (g == SEG_NONE) break;
            if (++hops * SEG_JUMP > nseg || off > wb.max_steps) {  // segments in a cycle
                atomicAdd(&stats[ST_CYCLE], 1ull);
                break;
            }
        }
        sb.clen[c] = (uint32_t)(off + 1);
    }
}

__global__ __launch_bounds__(BLOCK) void k_seg_fill(WalkBuffers wb, SegBuffers sb, unsigned long long* stats) {
    if (!*sb.long_flag) return;
    const uint64_t nseg = wb.n_starts + walk_splits(wb);
    for (uint64_t i = wb.n_starts + (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nseg;
         i += (uint64_t)gridDim.x * BLOCK) {
        if (!sb.anchor[i]) continue;
        uint32_t g = (uint32_t)i;
        const uint32_t c = sb.seg_contig[g];
        uint64_t off = sb.seg_off[g];
        for (uint32_t h = 1; h < SEG_JUMP; ++h) {
            off += wb.contig_len[g] - 1;
            g = wb.seg_next[g];
            if (g == SEG_NONE) break;
            if (atomicExch(&sb.seg_contig[g], c) != SEG_NONE) atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
            sb.seg_off[g] = (uint32_t)off;
        }
    }
}

struct SplitKeepF {
    KParams p;
    const uint64_t* splits;
    int bits;
    __device__ uint64_t operator()(uint64_t i) const {
        const uint64_t w0 = splits[i * p.W], w1 = p.W == 2 ? splits[i * p.W + 1] : 0;
        return split_test(slot_key(w0, w1, p), bits);
    }
};

__global__ __launch_bounds__(BLOCK) void k_filter_splits(SplitKeepF f, uint64_t n, const uint64_t* off, uint64_t* out) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        if (!f(i)) continue;
        for (int w = 0; w < f.p.W; ++w) out[off[i] * f.p.W + w] = f.splits[i * f.p.W + w];
    }
}

hipError_t launch_filter_splits(const KParams& p, const uint64_t* splits, uint64_t n, int bits, uint64_t* off,
                                uint64_t* scratch, uint64_t* out, unsigned long long* count, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(count, 0, 8, s);
    const SplitKeepF f{p, splits, bits};
    hipError_t e = scan_exclusive(f, n, off, scratch, (unsigned long long*)nullptr, count, s);
    if (e != hipSuccess) return e;
    k_filter_splits<<<(unsigned)hmin((n + BLOCK - 1) / BLOCK, 8192), BLOCK, 0, s>>>(f, n, off, out);
    return hipGetLastError();
}

// The splitter table (key -> segment id) and the segment owners' reset: they read only the walked
// splitter list, so they run before or beside the walk (on the resolve's side stream).
hipError_t launch_seg_table(const KParams& p, const WalkBuffers& wb, const SegBuffers& sb, hipStream_t s,
                            bool after) {
    const uint64_t nseg = wb.n_starts + wb.n_splits;
    if (nseg == 0) return hipSuccess;
    if (wb.split_min) k_stab_gate<<<1, 64, 0, s>>>(wb.seg_long, after ? 1 : 0);
    else if (after) return hipSuccess;  // built beside the walk
    k_stab_init<<<(unsigned)hmin((sb.cap2 + BLOCK - 1) / BLOCK, 2048), BLOCK, 0, s>>>(wb, sb.stab, sb.cap2);
    hipError_t e;
    // splitter segments' contigs (a start segment's is itself, never stored)
    if (!after && wb.n_splits &&
        (e = hipMemsetAsync(sb.seg_contig + wb.n_starts, 0xff, wb.n_splits * 4, s)) != hipSuccess)
        return e;
    if (wb.n_splits)
        k_stab_build<<<(unsigned)hmin((wb.n_splits + BLOCK - 1) / BLOCK, 4096), BLOCK, 0, s>>>(
            p, wb, sb.stab, sb.stab_id, sb.cap2);
    return hipGetLastError();
}

// After the walk (and launch_seg_table): links, chains, offsets.
hipError_t launch_segments(const KParams& p, const WalkBuffers& wb, const SegBuffers& sb_in,
                           unsigned long long* stats, hipStream_t s) {
    (void)p;
    SegBuffers sb = sb_in;
    sb.serial = wb.n_splits >= 16 * wb.n_starts ? SEG_SERIAL : SEG_SERIAL_FEW;
    const uint64_t nseg = wb.n_starts + wb.n_splits;
    if (nseg == 0) return hipSuccess;
    hipError_t e;
    const unsigned gs = (unsigned)hmin((nseg + BLOCK - 1) / BLOCK, 8192);
    k_seg_link<<<(unsigned)hmin((nseg / 4 + BLOCK) / BLOCK, 8192), BLOCK, 0, s>>>(wb, sb, stats);
    if (wb.n_starts == 0) return hipGetLastError();
    const unsigned gc = (unsigned)hmin((wb.n_starts + BLOCK - 1) / BLOCK, 8192);
    if ((e = hipMemsetAsync(sb.long_flag, 0, 4, s)) != hipSuccess) return e;
    k_seg_chain<<<gc, BLOCK, 0, s>>>(wb, sb, stats);
    k_seg_jump<<<gs, BLOCK, 0, s>>>(wb, sb);
    k_seg_chain_jump<<<gc, BLOCK, 0, s>>>(wb, sb, stats);
    k_seg_fill<<<gs, BLOCK, 0, s>>>(wb, sb, stats);
    return hipGetLastError();
}

// Chunk words of segment g go to contig seg_contig[g] at base offset seg_off[g].
// Four threads per chunk (words q and q + 4 of it): C3 segments (~100 bases) use ~4 of a chunk's
// 8 words and C5's ~21M contigs of 2-16 k-mers one, so eight threads per chunk (one per word)
// mostly load the segment metadata only to find their word unused.
static constexpr uint32_t WC_TPC = 4;  // 1: C3 materialize 0.38 -> 0.41 ms, C5 unchanged (round 5)
__global__ __launch_bounds__(BLOCK) void k_write_chunks_seg(int K, const uint64_t* chunk_data, const uint32_t* owner,
                                                            const uint32_t* seq, const unsigned long long* ctr,
                                                            uint64_t chunk_cap, uint64_t n_starts,
                                                            const unsigned long long* nsp_dev, uint64_t nsp,
                                                            const uint32_t* seg_len, const uint32_t* seg_contig,
                                                            const uint32_t* seg_off, const uint64_t* off,
                                                            char* out, uint64_t cap, uint64_t ch_begin,
                                                            const uint32_t* seg_long) {
    const uint64_t ns_w = nsp_dev ? (uint64_t)*nsp_dev : nsp;
    const uint64_t nseg = n_starts + ns_w;
    const uint64_t nchunks = min(nseg + (uint64_t)ctr[CT_CHUNK_NEXT], chunk_cap);
    // no contig reached a splitter segment (deferred segments, k_walk_q): their chunks are skipped
    const uint64_t gap = (seg_long && !*seg_long && ch_begin <= n_starts) ? ns_w : 0;
    const uint64_t nt = (nchunks - min(gap, nchunks)) * WC_TPC;
    for (uint64_t t = ch_begin * WC_TPC + (uint64_t)blockIdx.x * BLOCK + threadIdx.x; t < nt;
         t += (uint64_t)gridDim.x * BLOCK) {
        uint64_t ch = t / WC_TPC;
        if (ch >= n_starts) ch += gap;
        const uint32_t q = (uint32_t)(t % WC_TPC);
        const uint32_t g = ch < nseg ? (uint32_t)ch : owner[ch];
        const bool own = g < n_starts;  // a contig's start segment: contig g, offset 0
        const uint32_t c = own ? g : seg_contig[g];
        if (c == SEG_NONE) continue;  // a segment no contig reached
        const uint64_t cb = ch < nseg ? 0ull : (uint64_t)seq[ch] * CHUNK_BASES;
        const uint64_t app = (uint64_t)seg_len[g] - 1;
        if (cb + 32 * q >= app) continue;
        const uint32_t cnt = (uint32_t)min<uint64_t>(CHUNK_BASES, app - cb);
        const uint64_t so = own ? 0ull : (uint64_t)seg_off[g];
        if (off[c] + K + so + cb + cnt > cap) continue;  // past the buffer: not written
        char* o = out + off[c] + K + so + cb;
        for (uint32_t w = q; 32 * w < cnt; w += WC_TPC) {
            const uint64_t word = chunk_data[chunk_word(ch, w, chunk_cap)];
            store_chars(o + 32 * w, min(32u, cnt - 32 * w),
                        [&](uint32_t i) { return codes4_chars((uint32_t)(word >> (8 * i)) & 0xFFu); });
        }
    }
}

hipError_t launch_materialize_seg(const KParams& p, const WalkBuffers& wb, const SegBuffers& sb,
                                  uint64_t* offsets, uint64_t* scratch, char* out, unsigned long long* ctr,
                                  hipStream_t s, int phases, uint32_t* line_first, uint64_t out_bytes) {
    const uint64_t nc = wb.n_starts;
    if (nc == 0) return hipSuccess;
    hipError_t e = hipSuccess;
    if (phases & MAT_SCAN) {
        e = scan_exclusive(ContigBytesF{sb.clen, (uint64_t)p.K}, nc, offsets, scratch,
                           (unsigned long long*)nullptr, &ctr[CT_OUT_BYTES], s);
        if (e != hipSuccess) return e;
    }
    if (!(phases & MAT_WRITE)) return hipSuccess;
    const uint64_t cap = wb.text_cap ? wb.text_cap : ~0ull;
    const bool lines = launch_lines(p, wb, sb.clen, offsets, out, ctr, s, cap, line_first, out_bytes);
    if (!lines && (e = launch_write_heads(p, wb.starts, nc, sb.clen, offsets, out, s, cap)) != hipSuccess) return e;
    // chunks the line writer does not cover: splitter segments' and every segment's past its first
    const uint64_t cb = lines ? nc : 0;
    const unsigned gc = (unsigned)hmin(((wb.chunk_cap - min(cb, wb.chunk_cap)) * WC_TPC + BLOCK - 1) / BLOCK + 1, 8192);
    k_write_chunks_seg<<<gc, BLOCK, 0, s>>>(p.K, wb.chunk_data, wb.chunk_owner, wb.chunk_seq, ctr, wb.chunk_cap,
                                            nc, wb.n_splits_dev, wb.n_splits, wb.contig_len, sb.seg_contig,
                                            sb.seg_off, offsets, out, cap, cb, wb.split_min ? wb.seg_long : nullptr);
    return hipGetLastError();
}

// =============================================================================================
// Sharded multi-GPU path. The key space is split by owner_key (minimizer owner, kh_codec.hpp); records
// are routed to their owner once (insert), then contigs are walked in rounds: every home rank
// emits the next k-mer of each live walker to its owner, owners answer with the ext byte, homes
// apply the answers. The exchange between emit and apply is the caller's (RCCL all-to-all).

template <int W>
__global__ __launch_bounds__(BLOCK) void k_start_mask(KParams p, const uint8_t* __restrict__ recs,
                                                      uint64_t n, uint64_t* start_mask) {
    const uint64_t nw = (n + 63) >> 6;
    for (uint64_t i0 = (uint64_t)blockIdx.x * BLOCK + (threadIdx.x & ~63u); i0 < nw * 64;
         i0 += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t i = i0 + (threadIdx.x & 63);
        const bool st = i < n && recs[i * (uint64_t)p.R + p.P] == 'F';
        const uint64_t bal = __ballot(st);
        if ((threadIdx.x & 63) == 0) start_mask[i0 >> 6] = bal;
    }
}

hipError_t launch_start_mask(const KParams& p, const uint8_t* recs, uint64_t n, uint64_t* start_mask,
                             hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned grid = (unsigned)hmin((n + BLOCK - 1) / BLOCK, 8192);
    k_start_mask<1><<<grid, BLOCK, 0, s>>>(p, recs, n, start_mask);
    return hipGetLastError();
}

// Route = records -> owner-grouped words in two streaming passes over the records (the minimizer
// scan runs once, in the first pass, and is kept per record: it gives the owner rank and the
// j* / order bits the routed words carry into the owner's partition passes). Records are staged
// through LDS with 16-B loads (15-/7-byte records are unaligned for per-lane loads).
__device__ __forceinline__ void stage_records(const uint8_t* recs, uint64_t sub, uint32_t cnt, uint32_t R,
                                              uint8_t* st) {
    const uint32_t bytes = cnt * R, nvec = bytes >> 4;
    const uint4* src = reinterpret_cast<const uint4*>(recs + sub * R);
    for (uint32_t v = threadIdx.x; v < nvec; v += BLOCK) reinterpret_cast<uint4*>(st)[v] = src[v];
    for (uint32_t x = (nvec << 4) + threadIdx.x; x < bytes; x += BLOCK) st[x] = recs[sub * R + x];
}

// Record sub + threadIdx.x (< cnt) -> key + ext: two aligned 16-B loads and a register parse for
// records of <= 16 bytes, else through the LDS stage (whole block).
__device__ __forceinline__ void load_parse_record(const KParams& p, const uint8_t* __restrict__ recs, uint64_t sub,
                                                  uint32_t cnt, uint8_t* st, Key& k, uint32_t& ext) {
    if (p.R <= 16) {  // uniform
        if (threadIdx.x < cnt) {
            uint64_t x0, x1;
            load_record_regs(recs, sub + threadIdx.x, (uint32_t)p.R, x0, x1);
            parse_record_regs(x0, x1, p, k, ext);
        }
    } else {
        __syncthreads();
        stage_records(recs, sub, cnt, (uint32_t)p.R, st);
        __syncthreads();
        if (threadIdx.x < cnt) parse_record(st + threadIdx.x * p.R, p, k, ext);
    }
}

// owner rank of a k-mer whose minimizer scan is mn
__device__ __forceinline__ uint32_t owner_mn(Key k, uint32_t mn, const KParams& p, uint32_t P) {
    if (P == 1) return 0;
    return p.owner_mode == 1 ? owner_key(k, p, P) : owner_of_mini(mini_window(k, mn, p), P);
}

template <int KT>
__global__ __launch_bounds__(BLOCK) void k_route_own(KParams p_in, const uint8_t* __restrict__ recs, uint64_t n,
                                                     uint32_t P, uint32_t* own, uint64_t* hist,
                                                     uint64_t* start_mask, unsigned long long* spl) {
    const KParams p = specialize<KT>(p_in);
    __shared__ uint32_t h[MAX_RANKS], hs[MAX_RANKS];  // records / splitter k-mers per owner
    __shared__ __attribute__((aligned(16))) uint8_t st[BLOCK * 17 + 16];
    for (uint32_t q = threadIdx.x; q < P; q += BLOCK) h[q] = hs[q] = 0;
    __syncthreads();  // counters zeroed before any wave counts (records of <= 16 B take no barrier below)
    const uint64_t b0 = (uint64_t)blockIdx.x * ROUTE_TILE;
    for (uint32_t j = 0; j < ROUTE_TILE / BLOCK; ++j) {
        const uint64_t sub = b0 + (uint64_t)j * BLOCK;
        if (sub >= n) break;  // uniform
        const uint32_t cnt = n - sub < (uint64_t)BLOCK ? (uint32_t)(n - sub) : (uint32_t)BLOCK;
        Key k{0, 0};
        uint32_t ext = 0;
        load_parse_record(p, recs, sub, cnt, st, k, ext);
        if (threadIdx.x < cnt) {
            const uint32_t mn = mini_scan(k, p);
            own[sub + threadIdx.x] = mn;
            const uint32_t q = owner_mn(k, mn, p, P);
            atomicAdd(&h[q], 1u);
            if (spl && ext_bwd(ext) != EXT_F && is_splitter(k, p)) atomicAdd(&hs[q], 1u);
        }
        if (start_mask) {  // kmer_hash.cpp:27-31 start bits, same pass (ROUTE_TILE is 64-aligned)
            const uint64_t bal = __ballot(threadIdx.x < cnt && ext_bwd(ext) == EXT_F);
            const uint64_t wb = sub + (threadIdx.x & ~63u);
            if ((threadIdx.x & 63) == 0 && wb < n) start_mask[wb >> 6] = bal;
        }
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < P; q += BLOCK) {
        hist[(uint64_t)blockIdx.x * P + q] = h[q];
        if (spl && hs[q]) atomicAdd(&spl[q], (unsigned long long)hs[q]);
    }
}

template <int W, int KT>
__global__ __launch_bounds__(BLOCK) void k_route_scatter(KParams p_in, const uint8_t* __restrict__ recs, uint64_t n,
                                                         uint32_t P, const uint32_t* __restrict__ own,
                                                         const uint64_t* off, uint64_t nb, uint64_t* out) {
    const KParams p = specialize<KT>(p_in);
    __shared__ uint32_t h[MAX_RANKS];
    __shared__ __attribute__((aligned(16))) uint8_t st[BLOCK * 17 + 16];
    for (uint32_t q = threadIdx.x; q < P; q += BLOCK) h[q] = 0;
    __syncthreads();  // counters zeroed before any wave counts (records of <= 16 B take no barrier below)
    const uint64_t b0 = (uint64_t)blockIdx.x * ROUTE_TILE;
    for (uint32_t j = 0; j < ROUTE_TILE / BLOCK; ++j) {
        const uint64_t sub = b0 + (uint64_t)j * BLOCK;
        if (sub >= n) break;  // uniform
        const uint32_t cnt = n - sub < (uint64_t)BLOCK ? (uint32_t)(n - sub) : (uint32_t)BLOCK;
        Key k{0, 0};
        uint32_t ext = 0;
        load_parse_record(p, recs, sub, cnt, st, k, ext);
        if (threadIdx.x < cnt) {
            const uint32_t mn = own[sub + threadIdx.x];
            const uint32_t q = owner_mn(k, mn, p, P);
            const uint64_t d = off[(uint64_t)q * nb + blockIdx.x] + atomicAdd(&h[q], 1u);
            const uint64_t w0 = part_word0(slot_w0(k, ext, p), mn, p);  // + j*, order bits
            if (W == 2)
                *reinterpret_cast<ulonglong2*>(out + d * 2) = make_ulonglong2(w0, k.lo);
            else
                out[d] = w0;
        }
    }
}

hipError_t launch_route(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t nranks,
                        uint64_t* hist, uint64_t* off, uint64_t* scratch, uint32_t* own, uint64_t* out_words,
                        uint64_t* counts, hipStream_t s, uint64_t* start_mask, unsigned long long* spl) {
    if (!p.split_bits) spl = nullptr;
    unsigned long long* total = reinterpret_cast<unsigned long long*>(scratch);
    const uint64_t nb = route_blocks(n);
    if (nb == 0) return hipMemsetAsync(counts, 0, (nranks + 1) * 8, s);
    if (p.W == 1)
        with_kt<1>(p.K, [&](auto kt) { k_route_own<decltype(kt)::value><<<(unsigned)nb, BLOCK, 0, s>>>(p, recs, n, nranks, own, hist, start_mask, spl); });
    else
        with_kt<2>(p.K, [&](auto kt) { k_route_own<decltype(kt)::value><<<(unsigned)nb, BLOCK, 0, s>>>(p, recs, n, nranks, own, hist, start_mask, spl); });
    hipError_t e = scan_exclusive(HistF{hist, nb, nranks}, nb * nranks, off, scratch + 1,
                                  (unsigned long long*)nullptr, total, s);
    if (e != hipSuccess) return e;
    k_route_counts<0><<<1, MAX_RANKS, 0, s>>>(off, nb, nranks, total, counts);
    if (p.W == 1)
        with_kt<1>(p.K, [&](auto kt) { k_route_scatter<1, decltype(kt)::value><<<(unsigned)nb, BLOCK, 0, s>>>(p, recs, n, nranks, own, off, nb, out_words); });
    else
        with_kt<2>(p.K, [&](auto kt) { k_route_scatter<2, decltype(kt)::value><<<(unsigned)nb, BLOCK, 0, s>>>(p, recs, n, nranks, own, off, nb, out_words); });
    return hipGetLastError();
}

template <int W>
__global__ __launch_bounds__(BLOCK) void k_insert_words(KParams p, const uint64_t* __restrict__ words,
                                                        uint64_t m, uint64_t* slots, uint64_t cap,
                                                        unsigned long long* stats) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m;
         i += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t w0 = words[i * W];
        const uint64_t w1 = (W == 2) ? words[i * W + 1] : 0;
        const uint32_t ext = slot_ext(w0);
        if (ext_bwd(ext) == EXT_BAD || ext_fwd(ext) == EXT_BAD) atomicAdd(&stats[ST_BAD_EXT], 1ull);
        const Key k = slot_key(w0, w1, p);  // routed words carry no j*: full placement hash
        insert_one<W>(k, slot_w0(k, ext, p), home_of(place(k, p), cap, p), p, slots, cap, stats);
    }
}

hipError_t launch_insert_words(const KParams& p, const uint64_t* words, uint64_t m, TableView t,
                               unsigned long long* stats, hipStream_t s) {
    if (m == 0) return hipSuccess;
    const unsigned grid = (unsigned)hmin((m + BLOCK - 1) / BLOCK, 256ull * 32);
    if (p.W == 1)
        k_insert_words<1><<<grid, BLOCK, 0, s>>>(p, words, m, t.slots, t.cap, stats);
    else
        k_insert_words<2><<<grid, BLOCK, 0, s>>>(p, words, m, t.slots, t.cap, stats);
    return hipGetLastError();
}

}  // namespace kh

