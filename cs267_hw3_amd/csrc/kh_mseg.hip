// kh_mseg.hip — splitter segments for the sharded (migrating-walker) contig walk.
//
// A migrating walker hops to another rank at every owner change (~19 k-mers at k=51), so one
// contig of L k-mers costs ~L/19 rounds: a C5 chain of 10^6 k-mers would take ~50K rounds. As on
// one GPU (kh_kernels.hip, splitter segments), k-mers whose hash has split_bits low zero bits
// (and that are not contig starts) head segments of their own: every owner seeds a walker at each
// of its splitters, and every walker stops before a splitter k-mer, reporting the splitter's key
// (a link). Afterwards, per rank:
//   link    each segment that stopped before a splitter sends {splitter key, its global id, its
//           length} to the splitter's owner, which records the predecessor of that splitter's
//           segment (one all-to-all);
//   jump    pointer jumping over the predecessor links (Wyllie list ranking): every splitter
//           segment learns its contig (the start segment at the head of its chain) and its base
//           offset in it, in log2(segments per chain) query/reply rounds;
//   retag   text records of splitter segments (32-base words, already on the segment's owner)
//           become {contig origin, contig, base position, count, word} and go to the contig's
//           origin, with one {contig, end} record per segment for the contig length.
// Contigs whose walk never met a splitter (all of them at C3 sizes but a few %) need none of it.
#include "kh_device.hpp"

namespace kh {

static constexpr uint64_t GID_NONE = ~0ull;
// segment ids: rank << 40 | index; a splitter segment's index is its splitter number with
// GID_SPLIT set (start segments: the start's index), so every rank can place any rank's splitter
// segment in the all-gathered predecessor table without knowing that rank's start count
static constexpr uint64_t GID_SPLIT = 1ull << 39;

__device__ __forceinline__ uint64_t gid_make(uint32_t rank, uint64_t idx) { return ((uint64_t)rank << 40) | idx; }
__device__ __forceinline__ uint32_t gid_rank(uint64_t g) { return (uint32_t)(g >> 40); }
__device__ __forceinline__ uint64_t gid_idx(uint64_t g) { return g & ((1ull << 40) - 1); }
// local segment c (starts [0, ns), splitter segments ns + j) -> its id
__device__ __forceinline__ uint64_t gid_seg(uint32_t rank, uint64_t c, uint64_t ns) {
    return c < ns ? gid_make(rank, c) : gid_make(rank, GID_SPLIT | (c - ns));
}

// ---- splitter collection on the owner (routed words) ------------------------------------------
// One chunk of SPLIT_CHUNK words per block; splitters are gathered in LDS and reserved in the
// output list with ONE atomicAdd per block (a per-wave atomic on the single list counter cost
// ~8 ms at C3: same-address device atomics serialise at the memory side).
static constexpr uint32_t SPLIT_CHUNK = 65536;
static constexpr uint32_t SPLIT_LCAP = 2048;  // expected per chunk at 1 per 256: 256

template <int W>
__global__ __launch_bounds__(BLOCK) void k_split_collect(KParams p, const uint64_t* __restrict__ words, uint64_t m,
                                                         uint64_t* out, uint64_t cap, unsigned long long* ctr) {
    __shared__ uint64_t lbuf[SPLIT_LCAP * W];
    __shared__ uint32_t lcount;
    __shared__ unsigned long long lbase;
    for (uint64_t c0 = (uint64_t)blockIdx.x * SPLIT_CHUNK; c0 < m; c0 += (uint64_t)gridDim.x * SPLIT_CHUNK) {
        if (threadIdx.x == 0) lcount = 0;
        __syncthreads();
        const uint64_t c1 = min(c0 + SPLIT_CHUNK, m);
        for (uint64_t i = c0 + threadIdx.x; i < c1; i += BLOCK) {
            const uint64_t w0 = words[i * W], w1 = (W == 2) ? words[i * W + 1] : 0;
            if (ext_bwd(slot_ext(w0)) == EXT_F || !is_splitter(slot_key(w0, w1, p), p)) continue;
            const uint32_t pos = atomicAdd(&lcount, 1u);
            if (pos < SPLIT_LCAP) {
                lbuf[pos * W] = w0;
                if (W == 2) lbuf[pos * W + 1] = w1;
            } else {  // LDS buffer full (dense splitter bits): straight to the list
                const unsigned long long o = atomicAdd(&ctr[CT_N_SPLIT], 1ull);
                if (o < cap) {
                    out[o * W] = w0;
                    if (W == 2) out[o * W + 1] = w1;
                }
            }
        }
        __syncthreads();
        const uint32_t k = min(lcount, SPLIT_LCAP);
        if (threadIdx.x == 0) lbase = k ? atomicAdd(&ctr[CT_N_SPLIT], (unsigned long long)k) : 0ull;
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < k; x += BLOCK) {
            const uint64_t o = lbase + x;
            if (o < cap) {
                out[o * W] = lbuf[x * W];
                if (W == 2) out[o * W + 1] = lbuf[x * W + 1];
            }
        }
        __syncthreads();
    }
}

hipError_t launch_split_collect(const KParams& p, const uint64_t* words, uint64_t m, uint64_t* out, uint64_t cap,
                                unsigned long long* ctr, hipStream_t s) {
    if (m == 0 || !p.split_bits) return hipSuccess;
    const unsigned g = (unsigned)hmin((m + SPLIT_CHUNK - 1) / SPLIT_CHUNK, 8192);
    if (p.W == 1)
        k_split_collect<1><<<g, BLOCK, 0, s>>>(p, words, m, out, cap, ctr);
    else
        k_split_collect<2><<<g, BLOCK, 0, s>>>(p, words, m, out, cap, ctr);
    return hipGetLastError();
}

// ---- splitter key -> local segment index --------------------------------------------------------
__device__ __forceinline__ uint64_t stab_home(Key k, uint64_t cap2) { return mulhi64(fmix64(key_hash(k)), cap2); }

template <int W>
__global__ __launch_bounds__(BLOCK) void k_mseg_stab(KParams p, const uint64_t* splits, uint64_t nsp, uint64_t* stab,
                                                     uint32_t* id, uint64_t cap2) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nsp; i += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t w0 = splits[i * W], w1 = (W == 2) ? splits[i * W + 1] : 0;
        const Key k = slot_key(w0, w1, p);
        uint64_t s = stab_home(k, cap2);
        while (true) {  // lo < 2^62 is never EMPTY; splitters are unique
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

hipError_t launch_mseg_stab(const KParams& p, const uint64_t* splits, uint64_t nsp, uint64_t* stab, uint32_t* id,
                            uint64_t cap2, hipStream_t s) {
    hipError_t e = hipMemsetAsync(stab, 0xff, cap2 * 16, s);
    if (e != hipSuccess || nsp == 0) return e;
    const unsigned g = (unsigned)hmin((nsp + BLOCK - 1) / BLOCK, 4096);
    if (p.W == 1)
        k_mseg_stab<1><<<g, BLOCK, 0, s>>>(p, splits, nsp, stab, id, cap2);
    else
        k_mseg_stab<2><<<g, BLOCK, 0, s>>>(p, splits, nsp, stab, id, cap2);
    return hipGetLastError();
}

// ---- segment records (this rank's text records after they came home) ---------------------------
// finish records: word_no field = 0 length (bases appended), 1 / 2 = link key hi / lo. With
// chunk_data (the origin's line writer, K >= 16) the same pass scatters the first CHUNK_WORDS words
// of every start segment into the word-major first chunks (chunk c = contig c < ns) and counts the
// start segments' later words into *late (their character writer runs only when there are any).
__global__ __launch_bounds__(BLOCK) void k_mseg_scan(const uint64_t* recs, uint64_t n, uint64_t nseg, MSegState st,
                                                     unsigned long long* fin, uint64_t* chunk_data, uint64_t ns,
                                                     unsigned long long* late) {
    uint64_t f = 0, lw = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        const ulonglong2 r = reinterpret_cast<const ulonglong2*>(recs)[i];
        const uint64_t t = r.x;
        if (!((t >> 55) & 1)) {
            const uint64_t c = t & 0x7FFFFFFFull, wn = (t >> 31) & 0xFFFFFFull;
            if (chunk_data && c < ns) {
                if (wn < CHUNK_WORDS)
                    chunk_data[wn * ns + c] = r.y;
                else
                    ++lw;
            }
            continue;
        }
        const uint64_t c = t & 0x7FFFFFFFull;
        if (c >= nseg) continue;
        const uint32_t sub = (uint32_t)((t >> 31) & 0xFFFFFFull);
        const uint64_t v = r.y;
        if (sub == 0) {
            st.len[c] = (uint32_t)v;
            ++f;
        } else if (sub == 1) {
            st.link_hi[c] = v;
        } else {
            st.link_lo[c] = v;
            st.has_link[c] = 1;
        }
    }
    uint64_t tot;
    block_excl_scan(f, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(fin, (unsigned long long)tot);
    if (late) {
        block_excl_scan(lw, tot);
        if (threadIdx.x == 0 && tot) atomicAdd(late, (unsigned long long)tot);
    }
}

// link message: [key.hi, key.lo, predecessor gid, predecessor length]
struct LinkOp {
    KParams p;
    MSegState st;
    uint32_t P, rank;
    uint64_t ns;
    uint64_t* out;
    __device__ int owner(uint64_t i) const {
        if (!st.has_link[i]) return -1;
        return (int)owner_key(Key{st.link_hi[i], st.link_lo[i]}, p, P);
    }
    __device__ void emit(uint64_t i, int q, uint64_t d) const {
        if (q < 0) return;
        uint64_t* o = out + d * 4;
        o[0] = st.link_hi[i];
        o[1] = st.link_lo[i];
        o[2] = gid_seg(rank, i, ns);
        o[3] = st.len[i];
    }
};

hipError_t launch_mseg_link(const KParams& p, const MSegState& st, uint64_t ns, uint64_t nseg, uint32_t P, uint32_t rank,
                            uint64_t* hist, uint64_t* off, uint64_t* scratch, uint64_t* out, uint64_t* counts,
                            hipStream_t s) {
    unsigned long long* total = reinterpret_cast<unsigned long long*>(scratch);
    return group_by_owner(LinkOp{p, st, P, rank, ns, out}, nseg, P, hist, off, scratch + 1, counts, total, s);
}

// Owner of each linked splitter: its segment's predecessor; then the jump state of every segment.
__global__ __launch_bounds__(BLOCK) void k_mseg_pred(const uint64_t* msgs, uint64_t m, const uint64_t* stab,
                                                     const uint32_t* id, uint64_t cap2, uint64_t ns, MSegState st,
                                                     unsigned long long* stats) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += (uint64_t)gridDim.x * BLOCK) {
        const Key k{msgs[4 * i], msgs[4 * i + 1]};
        uint64_t s = stab_home(k, cap2);
        bool found = false;
        for (uint64_t probes = 0; probes < cap2; ++probes) {
            const uint64_t lo = stab[2 * s];
            if (lo == EMPTY) break;
            if (lo == k.lo && stab[2 * s + 1] == k.hi) {
                found = true;
                break;
            }
            s = (s + 1 == cap2) ? 0 : s + 1;
        }
        if (!found) {  // not a collected splitter: a start reached by another walk (overlapping walks,
                       // malformed input) or a missing k-mer; the host redoes the walk unsegmented,
                       // which walks through a start and reports a k-mer that is really missing
            atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
            continue;
        }
        const uint64_t g = ns + id[s];
        // a second predecessor: two walks run into one segment (malformed input, walks overlap)
        if (atomicExch((unsigned long long*)&st.jump[g], (unsigned long long)msgs[4 * i + 2]) != GID_NONE)
            atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
        st.acc[g] = msgs[4 * i + 3];
    }
}

// start segments: done, head = themselves; splitter segments: pending until their head is known
__global__ __launch_bounds__(BLOCK) void k_mseg_init(uint64_t ns, uint64_t nseg, uint32_t rank, MSegState st) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nseg; i += (uint64_t)gridDim.x * BLOCK) {
        st.has_link[i] = 0;
        st.len[i] = 0;
        st.done[i] = i < ns ? 1 : 0;
        st.jump[i] = i < ns ? gid_make(rank, i) : GID_NONE;
        st.acc[i] = 0;
    }
}

// ---- pointer jumping (Wyllie list ranking) over every rank's splitter segments --------------------
// After the links, each rank knows the predecessor {id, length} of its own splitter segments. Those
// tables are all-gathered (rank q's at q * stride, stride = the largest per-rank count), and every
// rank ranks the whole set on its device: log2(segments per chain) passes over the gathered table
// with no exchange per pass (the exchanged query/reply rounds of the earlier protocol needed a
// host round trip each). A pass whose predecessor found nothing pending returns at once, so the
// host launches enough passes for any chain without reading when they are done.
__global__ __launch_bounds__(BLOCK) void k_mseg_preds_out(MSegState st, uint64_t ns, const unsigned long long* nsp,
                                                          uint64_t nsp_max, uint64_t stride, uint64_t* out) {
    const uint64_t n = min((uint64_t)*nsp, nsp_max);
    for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < stride; j += (uint64_t)gridDim.x * BLOCK) {
        const bool live = j < n;
        out[2 * j] = live ? st.jump[ns + j] : GID_NONE;
        out[2 * j + 1] = live ? st.acc[ns + j] : 0;
    }
}

struct ResBuf {
    uint64_t* J;   // pointer: predecessor id, then the id it jumped to; when done: the head (a start)
    uint64_t* A;   // bases from the start of J's segment to this segment's start
    uint8_t* D;    // J is the contig's start segment
};

__global__ __launch_bounds__(BLOCK) void k_res_init(const uint64_t* all, uint64_t N, ResBuf b) {
    for (uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; g < N; g += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t j = all[2 * g];
        b.J[g] = j;
        b.A[g] = all[2 * g + 1];
        b.D[g] = (j != GID_NONE && !(gid_idx(j) & GID_SPLIT)) ? 1 : 0;
    }
}

// pass k: in -> out; pend[k] = entries still pending after it (pass k returns at once when pass
// k - 1 left none: the last written buffer is final). An entry follows up to RES_HOPS pointers of
// the previous pass (read-only here, so no races): a pointer spanning S segments becomes one
// spanning (RES_HOPS + 1) S, so log_{RES_HOPS+1} N passes rank any chain instead of log_2 N (each
// launch costs ~4.6 us even when it returns at once: 22 of them at C3's 780K splitter segments).
static constexpr uint32_t RES_HOPS = 7;
__global__ __launch_bounds__(BLOCK) void k_res_pass(uint32_t k, ResBuf in, ResBuf out, uint64_t N, uint64_t stride,
                                                    unsigned long long* pend) {
    if (k > 0 && pend[k - 1] == 0) return;
    uint64_t left = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; g < N; g += (uint64_t)gridDim.x * BLOCK) {
        uint64_t j = in.J[g], a = in.A[g];
        uint8_t d = in.D[g];
        if (!d && j != GID_NONE) {
            for (uint32_t h = 0; h < RES_HOPS && !d && j != GID_NONE; ++h) {
                const uint64_t t = (uint64_t)gid_rank(j) * stride + (gid_idx(j) & ~GID_SPLIT);
                if (t < N) {
                    const uint64_t jt = in.J[t];
                    a += in.A[t];
                    d = in.D[t];
                    j = jt;  // a broken predecessor (GID_NONE, not done) breaks this chain too
                } else {
                    j = GID_NONE;
                }
            }
            left += (!d && j != GID_NONE) ? 1 : 0;
        }
        out.J[g] = j;
        out.A[g] = a;
        out.D[g] = d;
    }
    uint64_t tot;
    block_excl_scan(left, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(&pend[k], (unsigned long long)tot);
}

// this rank's splitter segments <- the final buffer (the output of the first pass that left
// nothing pending)
__global__ __launch_bounds__(BLOCK) void k_res_apply(ResBuf b0, ResBuf b1, const unsigned long long* pend, uint32_t npass,
                                                     uint32_t rank, uint64_t stride, uint64_t ns,
                                                     const unsigned long long* nsp, uint64_t nsp_max, MSegState st) {
    uint32_t k = 0;
    while (k + 1 < npass && pend[k] != 0) ++k;
    const ResBuf& f = (k & 1) ? b0 : b1;  // pass k writes buffer (k + 1) % 2
    const uint64_t n = min((uint64_t)*nsp, nsp_max);
    for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < n; j += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t g = (uint64_t)rank * stride + j;
        st.done[ns + j] = f.D[g];
        st.jump[ns + j] = f.J[g];
        st.acc[ns + j] = f.A[g];
    }
}

// splitter segments whose head was never found (a broken chain: a missing k-mer upstream)
__global__ __launch_bounds__(BLOCK) void k_mseg_check(uint64_t ns, uint64_t nseg_max, MSegState st,
                                                      const unsigned long long* nsp, unsigned long long* stats) {
    uint64_t bad = 0;
    const uint64_t nseg = nsp ? min(ns + (uint64_t)*nsp, nseg_max) : nseg_max;
    for (uint64_t i = ns + (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nseg; i += (uint64_t)gridDim.x * BLOCK)
        bad += st.done[i] ? 0 : 1;
    uint64_t tot;
    block_excl_scan(bad, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(&stats[ST_MISSING], (unsigned long long)tot);
}

hipError_t launch_mseg_check(uint64_t ns, uint64_t nseg, const MSegState& st, const unsigned long long* nsp,
                             unsigned long long* stats, hipStream_t s) {
    if (nseg <= ns) return hipSuccess;
    k_mseg_check<<<(unsigned)hmin((nseg - ns + BLOCK - 1) / BLOCK, 1024), BLOCK, 0, s>>>(ns, nseg, st, nsp, stats);
    return hipGetLastError();
}

// ---- text of splitter segments -> contig origin --------------------------------------------------
// 3-word record: [origin << 56 | type << 48 | contig, type 0: pos | count << 48, type 1: end; word]
struct RetagOp {
    const uint64_t* recs;
    uint64_t n, ns, nsp;
    MSegState st;
    uint64_t* out;
    __device__ bool seg_rec(uint64_t i, uint64_t& c) const {
        if (i >= n) return false;
        const uint64_t t = recs[2 * i];
        if ((t >> 55) & 1) return false;
        c = t & 0x7FFFFFFFull;
        return c >= ns && c < ns + nsp && st.done[c];  // (a walker id past the segments: not ours)
    }
    __device__ int owner(uint64_t i) const {
        uint64_t c;
        if (i < n) return seg_rec(i, c) ? (int)gid_rank(st.jump[c]) : -1;
        const uint64_t g = ns + (i - n);  // one end record per splitter segment
        return st.done[g] ? (int)gid_rank(st.jump[g]) : -1;
    }
    __device__ void emit(uint64_t i, int q, uint64_t d) const {
        if (q < 0) return;
        uint64_t* o = out + 3 * d;
        if (i < n) {
            uint64_t c;
            seg_rec(i, c);
            const uint64_t t = recs[2 * i];
            const uint64_t wn = (t >> 31) & 0xFFFFFFull;
            const uint64_t len = st.len[c], j0 = wn * 32;
            const uint64_t cnt = j0 < len ? (len - j0 < 32 ? len - j0 : 32) : 0;
            o[0] = ((uint64_t)q << 56) | gid_idx(st.jump[c]);
            o[1] = (st.acc[c] + j0) | (cnt << 48);
            o[2] = recs[2 * i + 1];
        } else {
            const uint64_t g = ns + (i - n);
            o[0] = ((uint64_t)q << 56) | (1ull << 48) | gid_idx(st.jump[g]);
            o[1] = st.acc[g] + st.len[g];
            o[2] = 0;
        }
    }
};

hipError_t launch_mseg_retag(const uint64_t* recs, uint64_t n, uint64_t ns, uint64_t nsp, const MSegState& st,
                             uint32_t P, uint64_t* hist, uint64_t* off, uint64_t* scratch, uint64_t* out,
                             uint64_t* counts, hipStream_t s) {
    unsigned long long* total = reinterpret_cast<unsigned long long*>(scratch);
    return group_by_owner(RetagOp{recs, n, ns, nsp, st, out}, n + nsp, P, hist, off, scratch + 1, counts, total, s);
}

// ---- origin: lengths and characters ----------------------------------------------------------------
// contig length (k-mers) = 1 + bases appended over all its segments = 1 + max(start segment
// length, every splitter segment's end)
__global__ __launch_bounds__(BLOCK) void k_mseg_lens(const uint64_t* in3, uint64_t m, uint64_t ns, MSegState st,
                                                     uint32_t* contig_len) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < ns; i += (uint64_t)gridDim.x * BLOCK)
        contig_len[i] = st.len[i] + 1;
    (void)in3;
    (void)m;
}

__global__ __launch_bounds__(BLOCK) void k_mseg_lens_remote(const uint64_t* in3, uint64_t m, uint64_t ns,
                                                            uint32_t* contig_len) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t t = in3[3 * i];
        if (((t >> 48) & 0xFF) != 1) continue;
        const uint64_t c = t & ((1ull << 48) - 1);
        if (c < ns) atomicMax(&contig_len[c], (uint32_t)(in3[3 * i + 1] + 1));
    }
}

// start segments' own words numbered >= wmin (bounded by the start segment's length, not the
// contig's); the line writer covers the first CHUNK_WORDS when it runs (wmin = CHUNK_WORDS)
__global__ __launch_bounds__(BLOCK) void k_mseg_words_local(int K, const uint64_t* recs, uint64_t n, uint64_t ns,
                                                            MSegState st, const uint64_t* off, char* out,
                                                            uint64_t cap, uint32_t wmin,
                                                            const unsigned long long* late) {
    if (late && *late == 0) return;  // no start segment has words past the line writer's
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t t = recs[2 * i];
        if ((t >> 55) & 1) continue;
        const uint64_t c = t & 0x7FFFFFFFull;
        if (c >= ns) continue;
        const uint64_t wn = (t >> 31) & 0xFFFFFFull;
        if (wn < wmin) continue;
        const uint64_t app = st.len[c], j0 = wn * 32;
        if (j0 >= app) continue;
        const uint32_t cnt = (uint32_t)(app - j0 < 32 ? app - j0 : 32);
        if (off[c] + K + j0 + cnt > cap) continue;  // a bad length: kh_sync reports it, never overrun
        const uint64_t word = recs[2 * i + 1];
        store_chars(out + off[c] + K + j0, cnt,
                    [&](uint32_t x) { return codes4_chars((uint32_t)(word >> (8 * x)) & 0xFFu); });
    }
}

__global__ __launch_bounds__(BLOCK) void k_mseg_words_remote(int K, const uint64_t* in3, uint64_t m, uint64_t ns,
                                                             const uint64_t* off, char* out, uint64_t cap) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < m; i += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t t = in3[3 * i];
        if (((t >> 48) & 0xFF) != 0) continue;
        const uint64_t c = t & ((1ull << 48) - 1);
        if (c >= ns) continue;
        const uint64_t pc = in3[3 * i + 1];
        const uint64_t pos = pc & ((1ull << 48) - 1);
        const uint32_t cnt = (uint32_t)(pc >> 48);
        if (!cnt || off[c] + K + pos + cnt > cap) continue;  // bad position: never overrun
        const uint64_t word = in3[3 * i + 2];
        store_chars(out + off[c] + K + pos, cnt,
                    [&](uint32_t x) { return codes4_chars((uint32_t)(word >> (8 * x)) & 0xFFu); });
    }
}

static unsigned grid_n(uint64_t n, uint64_t cap) {
    const uint64_t g = (n + BLOCK - 1) / BLOCK;
    return (unsigned)(g == 0 ? 1 : (g < cap ? g : cap));
}

hipError_t launch_mseg_scan(const uint64_t* recs, uint64_t n, uint64_t nseg, const MSegState& st,
                            unsigned long long* fin, hipStream_t s, uint64_t* chunk_data, uint64_t ns,
                            unsigned long long* late) {
    if (n == 0) return hipSuccess;
    k_mseg_scan<<<grid_n(n, 2048), BLOCK, 0, s>>>(recs, n, nseg, st, fin, chunk_data, ns, late);
    return hipGetLastError();
}

hipError_t launch_mseg_pred(const uint64_t* msgs, uint64_t m, const uint64_t* stab, const uint32_t* id, uint64_t cap2,
                            uint64_t ns, const MSegState& st, unsigned long long* stats, hipStream_t s) {
    if (m == 0) return hipSuccess;
    k_mseg_pred<<<grid_n(m, 4096), BLOCK, 0, s>>>(msgs, m, stab, id, cap2, ns, st, stats);
    return hipGetLastError();
}

hipError_t launch_mseg_init(uint64_t ns, uint64_t nseg, uint32_t rank, const MSegState& st, hipStream_t s) {
    if (nseg == 0) return hipSuccess;
    k_mseg_init<<<grid_n(nseg, 8192), BLOCK, 0, s>>>(ns, nseg, rank, st);
    return hipGetLastError();
}

hipError_t launch_mseg_preds_out(const MSegState& st, uint64_t ns, const unsigned long long* nsp, uint64_t nsp_max,
                                 uint64_t stride, uint64_t* out, hipStream_t s) {
    if (stride == 0) return hipSuccess;
    k_mseg_preds_out<<<grid_n(stride, 4096), BLOCK, 0, s>>>(st, ns, nsp, nsp_max, stride, out);
    return hipGetLastError();
}

// passes for any chain of <= N segments: each pass multiplies a pointer's span by RES_HOPS + 1
uint32_t mseg_resolve_passes(uint64_t N) {
    uint32_t k = 1;
    unsigned __int128 span = 1;
    while (k < 62 && span < (unsigned __int128)N + 1) {
        span *= RES_HOPS + 1;
        ++k;
    }
    return k + 1;
}

hipError_t launch_mseg_resolve(const uint64_t* all, uint64_t N, uint64_t stride, uint32_t rank, uint64_t ns,
                               const unsigned long long* nsp, uint64_t nsp_max, const MSegState& st, uint64_t* J0,
                               uint64_t* A0, uint8_t* D0, uint64_t* J1, uint64_t* A1, uint8_t* D1,
                               unsigned long long* pend, hipStream_t s) {
    const uint32_t np = mseg_resolve_passes(N);
    hipError_t e = hipMemsetAsync(pend, 0, np * 8, s);
    if (e != hipSuccess) return e;
    const ResBuf b0{J0, A0, D0}, b1{J1, A1, D1};
    if (N) {
        k_res_init<<<grid_n(N, 4096), BLOCK, 0, s>>>(all, N, b0);
        for (uint32_t k = 0; k < np; ++k)
            k_res_pass<<<grid_n(N, 4096), BLOCK, 0, s>>>(k, (k & 1) ? b1 : b0, (k & 1) ? b0 : b1, N, stride, pend);
        k_res_apply<<<grid_n(nsp_max, 4096), BLOCK, 0, s>>>(b0, b1, pend, np, rank, stride, ns, nsp, nsp_max, st);
    }
    return hipGetLastError();
}

hipError_t launch_mseg_lens(const uint64_t* in3, uint64_t m, uint64_t ns, const MSegState& st, uint32_t* contig_len,
                            hipStream_t s) {
    if (ns) k_mseg_lens<<<grid_n(ns, 8192), BLOCK, 0, s>>>(in3, m, ns, st, contig_len);
    if (m) k_mseg_lens_remote<<<grid_n(m, 8192), BLOCK, 0, s>>>(in3, m, ns, contig_len);
    return hipGetLastError();
}

hipError_t launch_mseg_words(int K, const uint64_t* recs, uint64_t n, const uint64_t* in3, uint64_t m, uint64_t ns,
                             const MSegState& st, const uint64_t* off, char* out, uint64_t cap, hipStream_t s,
                             uint32_t wmin, const unsigned long long* late) {
    if (n) k_mseg_words_local<<<grid_n(n, 8192), BLOCK, 0, s>>>(K, recs, n, ns, st, off, out, cap, wmin, late);
    if (m) k_mseg_words_remote<<<grid_n(m, 8192), BLOCK, 0, s>>>(K, in3, m, ns, off, out, cap);
    return hipGetLastError();
}

}  // namespace kh
