// kh_mwalk.hip — sharded contig walk with migrating walkers (the multi-GPU walk path).
//
// Reference: assemble_contigs (kmer_hash.cpp:38-55) walks every start k-mer of its rank with one
// DistributedHashMap::find per step, a blocking RPC to the owner for (P-1)/P of the steps
// (hash_map.hpp:83-107). Here the table is sharded by owner_key, a hash of the k-mer's minimizer,
// so consecutive k-mers of a contig mostly live on the same rank. A walker therefore moves to the
// data instead of querying it: on the rank that owns its current k-mer it keeps walking through
// the local shard until the next k-mer belongs to another rank, then it is sent there (one
// all-to-all per round, done by the caller between kernels). Rounds ~ longest contig / minimizer
// run length instead of longest contig.
//
// Bases appended by a walker are flushed as 32-base words tagged (origin rank, walker, word
// number) into a rank-local text store; after the last round the store is routed to the origin
// ranks, which materialise their test_<rank>.dat bytes (extract_contig, read_kmers.hpp:81-92).
#include "kh_device.hpp"

namespace kh {

static constexpr uint32_t MW_LOOKUP = 0xFF;   // message state: key must be looked up by its owner
static constexpr uint32_t MW_READREC = 0xFE;  // message state: read head record (m[4] >> 32) - 1 of this
                                              // rank (its run starts at the key; only sent to self)
static constexpr uint32_t MW_ENTRY = 0xFD;    // a new walker (first round): look up its own start k-mer
                                              // for the record covering its run; its forward
                                              // extension is the start record's own
static constexpr uint8_t MW_NONE = 0xFF;      // destination: walker finished this round

__device__ __forceinline__ uint64_t rec_tag(uint32_t origin, bool fin, uint64_t word_no, uint32_t idx) {
    return ((uint64_t)origin << 56) | ((uint64_t)fin << 55) | (word_no << 31) | idx;
}

// One lane per input message (static stride, no work-queue atomics), one load per lane per loop
// iteration, like k_walk_q. A lane's run ends when the walker finishes, migrates, or has flushed
// MW_RUN_WORDS words this round (it then re-sends itself, bounding the per-input text region).
// Chains (kh_build.hip): a probed k-mer whose slot names a head record is crossed in one step —
// the record's tail key carries the run's bases. A chain shares one minimizer, hence one owner,
// so it never crosses ranks. As on one GPU (k_walk_q), a walker starts from its own record when
// k_mw_init found one, and after a run follows the record's successor (k_rec_succ) without probing
// the next run's head k-mer: one dependent request per run.
template <int W, int KT>
__global__ __launch_bounds__(BLOCK) void k_mw_run(KParams p_in, const uint64_t* __restrict__ slots, uint64_t cap,
                                                  MWalkRound mw, unsigned long long* stats) {
    KParams p = specialize<KT>(p_in);
    if (mw.hot_on && *mw.hot_on == 0) p.hot = nullptr;  // no remapped region: skip the bitmap loads
    const bool chains = p.chain && mw.hcap != 0;
    const uint64_t n_live = mw.n_dev ? min((uint64_t)*mw.n_dev, mw.n_in) : mw.n_in;
    const uint32_t q4 = lane_id() & 3u, ql4 = lane_id() & ~3u;  // quad member, quad's first lane
    uint32_t reg = 0;  // region of the k-mer being probed (its head records live there)
    // append n bases (base i at bits 2i of piece, n <= room in the current word) to the walker's
    // buffer, flushing a finished 32-base word as a text record
    auto put = [&](uint64_t piece, uint32_t n, uint64_t& buf, uint32_t& steps, uint32_t& nrec, uint32_t& nwords,
                   uint64_t* rec, uint32_t origin, uint32_t idx) {
        buf |= piece << (2 * (steps & 31));
        steps += n;
        if ((steps & 31) == 0) {
            rec[2 * nrec] = rec_tag(origin, false, (steps >> 5) - 1, idx);
            rec[2 * nrec + 1] = buf;
            ++nrec;
            ++nwords;
            buf = 0;
        }
    };
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    bool active = false, probing = false, entry = false;
    Key k{0, 0};
    uint64_t s = 0, buf = 0, pb = 0;          // pb: 4-slot blocks probed for the current k-mer
    const uint64_t pb_max = (cap >> 2) + 1;   // every block once: the k-mer is absent (a full table)
    uint32_t steps = 0, idx = 0, origin = 0, st = 0, nrec = 0, nwords = 0, efwd = 0;
    uint32_t nsucc = 0;  // the last record's successor run (head-record index + 1 in its region)
    uint64_t* rec = nullptr;
    auto finish = [&](uint64_t jj) {
        if (steps & 31) {
            rec[2 * nrec] = rec_tag(origin, false, steps >> 5, idx);
            rec[2 * nrec + 1] = buf;
            ++nrec;
        }
        rec[2 * nrec] = rec_tag(origin, true, 0, idx);
        rec[2 * nrec + 1] = steps;
        ++nrec;
        mw.dst[jj] = MW_NONE;
    };
    while (true) {
        // one minimizer scan site per iteration, for a new message's lookup and for a stepped
        // walker's next k-mer (owner + region): lanes on either path share one scan, not one each
        bool scan = false, fresh = false;
        if (!active && j < n_live) {
            uint64_t m4;
            if (mw.in) {
                const uint64_t* m = mw.in + j * MSG_WORDS;
                k.hi = m[0];
                k.lo = m[1];
                buf = m[2];
                steps = (uint32_t)m[3];
                idx = (uint32_t)(m[3] >> 32);
                m4 = m[4];
            } else {
                // first round: walker j is start k-mer j, then splitter j - ns (segment ids in that
                // order, kh_mseg.hip); with chains it looks up its own k-mer first (MW_ENTRY), as the
                // single-GPU walker does, else it steps from its own extension
                const uint64_t* x = j < mw.ns ? mw.starts + j * W : mw.splits + (j - mw.ns) * W;
                const uint64_t x0 = x[0], x1 = (W == 2) ? x[1] : 0;
                k = slot_key(x0, x1, p);
                const uint32_t f = ext_fwd(slot_ext(x0));
                efwd = f > 4 ? EXT_BAD : f;
                buf = 0;
                steps = 0;
                idx = (uint32_t)j;
                m4 = mw.rank | ((uint64_t)(chains && efwd <= 3u ? MW_ENTRY : efwd) << 8);
            }
            origin = (uint32_t)m4 & 0xFFu;
            st = (uint32_t)(m4 >> 8) & 0xFFu;
            rec = mw.stage + j * (MW_REC_SLOTS * 2);
            nrec = 0;
            nwords = 0;
            nsucc = 0;
            active = true;
            entry = st == MW_ENTRY;
            probing = st == MW_LOOKUP || st == MW_READREC || entry;
            if (st == MW_READREC) {
                s = WQ_REC | ((m4 >> 32) - 1);
            } else if (probing) {
                scan = fresh = true;  // s: its home slot, below
            }
        }
        if (!__any(active)) break;
        bool fin = false, ovf = false;
        const bool stepped = active && !probing;
        if (stepped) {
            if (st > 3) {
                if (st != EXT_F) atomicAdd(&stats[ST_BAD_EXT], 1ull);
                fin = true;
            } else if (mw.soft_steps && steps > mw.soft_steps) {  // a long contig: walk again segmented
                atomicAdd(mw.long_ctr, 1ull);
                fin = true;
            } else if (steps > mw.max_steps) {
                atomicAdd(&stats[ST_CYCLE], 1ull);
                fin = true;
            } else {
                put(st, 1, buf, steps, nrec, nwords, rec, origin, idx);
                k = key_next(k, st, p);
                if (split_test(k, (int)mw.split_bits)) {
                    // the next k-mer heads a segment of its own: report it as this segment's link
                    rec[2 * nrec] = rec_tag(origin, true, 1, idx);
                    rec[2 * nrec + 1] = k.hi;
                    ++nrec;
                    rec[2 * nrec] = rec_tag(origin, true, 2, idx);
                    rec[2 * nrec + 1] = k.lo;
                    ++nrec;
                    fin = true;
                }
                scan = !fin;
            }
        }
        // one minimizer scan gives both the owner rank and the placement region
        uint32_t mv = 0;
        Place pl{0u, 0u};
        if (scan) {
            const uint32_t mn = mini_scan(k, p);
            mv = mini_window(k, mn, p);
            pl = place_w(mv, k, p, (int)(mn & 63u));
        }
        if (fresh) {
            reg = pl.r;
            s = home_of(pl, cap, p);
            pb = 0;
        }
        if (stepped) {
            if (scan) {
                const uint32_t q = mw.P == 1 ? 0u
                                             : (p.owner_mode == 1 ? owner_key(k, p, mw.P) : owner_of_mini(mv, mw.P));
                if (q != mw.rank || nwords >= MW_RUN_WORDS) {
                    // to the owner (or to itself, bounding this round's text): a successor record
                    // is only meaningful on this rank
                    uint64_t* o = mw.tmp + j * MSG_WORDS;
                    o[0] = k.hi;
                    o[1] = k.lo;
                    o[2] = buf;
                    o[3] = ((uint64_t)idx << 32) | steps;
                    o[4] = (nsucc && q == mw.rank)
                               ? origin | ((uint64_t)MW_READREC << 8) |
                                     (((uint64_t)pl.r * mw.hcap + nsucc) << 32)
                               : origin | ((uint64_t)MW_LOOKUP << 8);
                    mw.dst[j] = (uint8_t)q;
                    ovf = true;
                } else {
                    probing = true;
                    reg = pl.r;
                    // the record names the run that starts at k (k_rec_succ): read it, no probe
                    s = (nsucc && nwords + 3 <= MW_RUN_WORDS) ? WQ_REC | ((uint64_t)reg * mw.hcap + nsucc - 1)
                                                              : home_of(pl, cap, p);
                    pb = 0;
                }
            }
            nsucc = 0;
            if (fin) finish(j);
            if (fin || ovf) {
                mw.nrec[j] = (uint8_t)nrec;
                active = false;
                j += stride;
            }
        }
        // quad-transposed block probe (as k_walk_q): lane q of a quad loads slot q of each member's
        // 64-B block (one request per block), the members learn their first hit / EMPTY by ballot;
        // a record read loads the same 16 B in all 4 lanes (one request)
        const uint64_t sp = (active && probing) ? s : WQ_IDLE;
        uint64_t sj[4], w0[4], w1[4];
        sj[0] = qbcast64<0>(sp);
        sj[1] = qbcast64<1>(sp);
        sj[2] = qbcast64<2>(sp);
        sj[3] = qbcast64<3>(sp);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            w0[jj] = EMPTY;
            w1[jj] = 0;
            if (sj[jj] == WQ_IDLE) continue;
            if (sj[jj] & WQ_REC) {
                const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(mw.headrec + (sj[jj] & ~WQ_REC) * 2);
                w0[jj] = v.x;
                w1[jj] = v.y;
            } else {
                const uint64_t my = (sj[jj] & ~3ull) + q4;
                if (my < cap) load_slot_nt<W>(slots, my, w0[jj], w1[jj]);
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
        for (int jj = 0; jj < 4; ++jj) {
            const uint64_t my = (sj[jj] & ~3ull) + q4;
            const bool probe_j = sj[jj] != WQ_IDLE && !(sj[jj] & WQ_REC);
            const bool valid = probe_j && my >= sj[jj] && my < cap;
            const bool empty = w0[jj] == EMPTY;
            const bool hit = !empty & (slot_keybits(w0[jj], p) == ((W == 1) ? kl_[jj] : kh_[jj])) &
                             ((W == 1) | (w1[jj] == kl_[jj]));
            const uint32_t bh = (uint32_t)(__ballot(valid && hit) >> ql4) & 0xFu;
            const uint32_t be = (uint32_t)(__ballot(valid && empty) >> ql4) & 0xFu;
            const uint32_t fh = bh ? (uint32_t)__builtin_ctz(bh) : 4u;
            const uint32_t fe = be ? (uint32_t)__builtin_ctz(be) : 4u;
            // hit slot: ext | found flag | head-record index << 7
            const uint32_t ext =
                qor32(q4 == fh ? (slot_ext(w0[jj]) | 0x40u | ((chains ? slot_hidx(w0[jj], p) : 0u) << 7)) : 0u);
            if (q4 == (uint32_t)jj) {
                myfh = fh;
                myfe = fe;
                myext = ext;
                r0 = w0[jj];
                r1 = w1[jj];
            }
        }
        if (active && probing) {
            if (s & WQ_REC) {
                // head record: jump to the run's tail, appending the bases of its links
                k = slot_key(r0, r1, p);
                st = ext_fwd(slot_ext(r0));
                nsucc = rec_succ(r0, p);
                uint32_t n = rec_links(r0, p);  // links: the last n bases of the tail key
                while (n) {
                    const uint32_t room = 32u - (steps & 31u), m = n < room ? n : room;
                    const int sh = 2 * (int)(n - m);  // bits [sh, sh + 2m) of V, oldest base first
                    const uint64_t x = sh < 62 ? (k.lo >> sh) | (k.hi << (62 - sh)) : k.hi >> (sh - 62);
                    const uint64_t v = m >= 32 ? x : x & ((1ull << (2 * m)) - 1);
                    const uint64_t r = ((uint64_t)__builtin_bitreverse32((uint32_t)v) << 32) |
                                       __builtin_bitreverse32((uint32_t)(v >> 32));
                    const uint64_t rev = ((r >> 1) & 0x5555555555555555ull) | ((r & 0x5555555555555555ull) << 1);
                    put(rev >> (64 - 2 * m), m, buf, steps, nrec, nwords, rec, origin, idx);
                    n -= m;
                }
                probing = false;
            } else if (myfh < myfe) {
                const uint32_t hidx = myext >> 7, tf = ext_fwd(myext & 63u);
                // a start walks from its own record (kmer_hash.cpp:42-44): a record whose run
                // begins with another extension (a duplicate key) is not used for it
                if (hidx && !(entry && tf != efwd) && nwords + 3 <= MW_RUN_WORDS) {  // the run's <= 2 words fit
                    s = WQ_REC | ((uint64_t)reg * mw.hcap + hidx - 1);
                } else {
                    st = entry ? efwd : tf;
                    probing = false;
                }
                entry = false;
            } else if (myfe < 4u || ++pb > pb_max) {
                if (entry) {  // a start k-mer need not be in this shard (kh_set_starts): step from its own
                    st = efwd;
                    probing = false;
                    entry = false;
                } else {  // find() miss: kmer_hash.cpp:47-49 throws; finish the contig here
                    atomicAdd(&stats[ST_MISSING], 1ull);
                    finish(j);
                    mw.nrec[j] = (uint8_t)nrec;
                    active = false;
                    j += stride;
                }
            } else {
                const uint64_t nx = (s & ~3ull) + 4;
                s = nx >= cap ? 0 : nx;
            }
        }
    }
}

struct NrecF {
    const uint8_t* n;
    const unsigned long long* n_dev;  // inputs past the live count wrote nothing
    __device__ uint64_t operator()(uint64_t i) const { return (!n_dev || i < *n_dev) ? n[i] : 0u; }
};

// The records of a wave's 64 inputs are contiguous in the store (off is their exclusive scan), so
// the wave copies them as one run: lane t takes record t of the run (its input by a binary search
// over the 64 offsets), one coalesced 16-B store per lane (a lane copying its own input's records
// stored 64 inputs' records 192 B apart per instruction: 0.25 ms at C3).
__global__ __launch_bounds__(BLOCK) void k_mw_compact(const uint64_t* stage, const uint8_t* nrec,
                                                      const uint64_t* off, uint64_t nb, uint64_t* store,
                                                      const unsigned long long* n_dev, uint64_t store_cap,
                                                      unsigned long long* stats) {
    const uint64_t n = n_dev ? min((uint64_t)*n_dev, nb) : nb;
    const uint32_t lane = lane_id();
    const uint64_t waves = (uint64_t)gridDim.x * (BLOCK / 64);
    for (uint64_t j0 = ((uint64_t)blockIdx.x * BLOCK + threadIdx.x) / 64 * 64; j0 < n; j0 += waves * 64) {
        const uint64_t j = j0 + lane;
        const uint32_t c = j < n ? nrec[j] : 0u;
        const uint64_t o = j < n ? off[j] : 0;
        const uint64_t base = __shfl(o, 0, 64);
        const uint32_t rel = (uint32_t)(o - base);  // < 64 * MW_REC_SLOTS
        // inclusive end of each lane's records; the run's total from the last lane
        const uint32_t last = (uint32_t)min<uint64_t>(n - j0, 64) - 1;
        const uint32_t tot = __shfl(rel + c, (int)last, 64);
        // past the store's bound (malformed input: overlapping walks): the records that fit are
        // written, so every record below the bound is real (the text grouping reads up to it), and
        // the overflow is reported (the walk is redone with a larger store)
        if (base + tot > store_cap && lane == 0) atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
        if (base >= store_cap) continue;
        for (uint32_t t0 = 0; t0 < tot; t0 += 64) {
            const uint32_t t = t0 + lane;
            // the input holding record t: the last lane whose run starts at or before t (lanes
            // with no records share their start with the next one: take the last such lane)
            uint32_t lo = 0;
#pragma unroll
            for (uint32_t st = 32; st > 0; st >>= 1) {
                const uint32_t v = __shfl(rel, (int)(lo + st), 64);
                if (lo + st <= last && v <= t) lo += st;
            }
            const uint32_t r0 = __shfl(rel, (int)lo, 64);
            if (t < tot && base + t < store_cap) {
                const ulonglong2* src =
                    reinterpret_cast<const ulonglong2*>(stage + (j0 + lo) * (MW_REC_SLOTS * 2)) + (t - r0);
                reinterpret_cast<ulonglong2*>(store)[base + t] = *src;
            }
        }
    }
}

struct MsgOp {
    const uint8_t* dst;
    const uint64_t* tmp;
    uint64_t* out;
    __device__ int owner(uint64_t i) const { return dst[i] == MW_NONE ? -1 : (int)dst[i]; }
    __device__ void emit(uint64_t i, int q, uint64_t d) const {
        if (q < 0) return;
        const uint64_t* a = tmp + i * MSG_WORDS;
        uint64_t* b = out + d * MSG_WORDS;
#pragma unroll
        for (int w = 0; w < MSG_WORDS; ++w) b[w] = a[w];
    }
};

struct RecOp {
    const uint64_t* recs;
    uint64_t* out;
    const unsigned long long* n_dev;  // records past the live count do not exist (null: all)
    uint32_t P;
    __device__ int owner(uint64_t i) const {
        if (n_dev && i >= *n_dev) return -1;
        const uint32_t q = (uint32_t)(recs[2 * i] >> 56);
        return q < P ? (int)q : -1;  // (a record's origin is a rank: anything else is not sent)
    }
    __device__ void emit(uint64_t i, int q, uint64_t d) const {
        if (q < 0) return;  // past the live count
        reinterpret_cast<ulonglong2*>(out)[d] = reinterpret_cast<const ulonglong2*>(recs)[i];
    }
};

// Origin side: finish records -> contig lengths (k-mers = bases appended + 1); *fin counts them
// (one atomic per block) so the host can check that every walker came home. With chunk_data (the
// line writer, K >= 16) the first CHUNK_WORDS words of each contig go into its word-major first
// chunk (chunk c = contig c) in the same pass.
__global__ __launch_bounds__(BLOCK) void k_mw_lens(const uint64_t* recs, uint64_t n, uint64_t nc, uint32_t* len,
                                                   unsigned long long* fin, uint64_t* chunk_data) {
    uint64_t f = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        const ulonglong2 r = reinterpret_cast<const ulonglong2*>(recs)[i];
        const uint64_t t = r.x;
        const uint64_t c = t & 0x7FFFFFFFull;
        if (!((t >> 55) & 1)) {
            const uint64_t wn = (t >> 31) & 0xFFFFFFull;
            if (chunk_data && c < nc && wn < CHUNK_WORDS) chunk_data[wn * nc + c] = r.y;
            continue;
        }
        if (c < nc) {
            len[c] = (uint32_t)r.y + 1;
            ++f;
        }
    }
    uint64_t tot;
    block_excl_scan(f, tot);
    if (threadIdx.x == 0 && tot) atomicAdd(fin, (unsigned long long)tot);
}

// Origin side: word records (number >= wmin) -> characters.
__global__ __launch_bounds__(BLOCK) void k_mw_words(int K, const uint64_t* recs, uint64_t n, uint64_t nc,
                                                    const uint32_t* len, const uint64_t* off, char* out,
                                                    uint64_t cap, uint32_t wmin) {
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK) {
        const uint64_t t = recs[2 * i];
        if ((t >> 55) & 1) continue;
        const uint32_t c = (uint32_t)(t & 0x7FFFFFFFull);
        if (c >= nc) continue;
        const uint64_t wn = (t >> 31) & 0xFFFFFFull;
        if (wn < wmin) continue;
        const uint64_t app = (uint64_t)len[c] - 1;
        const uint64_t j0 = wn * 32;
        if (j0 >= app) continue;
        const uint32_t cnt = (uint32_t)(app - j0 < 32 ? app - j0 : 32);
        if (off[c] + K + j0 + cnt > cap) continue;  // a bad length: kh_sync reports it, never overrun
        const uint64_t word = recs[2 * i + 1];
        char* o = out + off[c] + K + j0;
        store_chars(o, cnt, [&](uint32_t x) { return codes4_chars((uint32_t)(word >> (8 * x)) & 0xFFu); });
    }
}

static unsigned grid_for(uint64_t n, uint64_t cap_blocks) {
    const uint64_t g = (n + BLOCK - 1) / BLOCK;
    return (unsigned)(g == 0 ? 1 : (g < cap_blocks ? g : cap_blocks));
}

hipError_t launch_mw_run(const KParams& p, TableView t, const MWalkRound& mw, unsigned long long* stats,
                         hipStream_t s) {
    if (mw.n_in == 0) return hipSuccess;
    // ~4 inputs per lane keeps lanes busy through the run-length tail without a work queue
    constexpr uint64_t ipl = 4;
    const unsigned g = grid_for((mw.n_in + ipl - 1) / ipl, 4096);
    if (p.W == 1)
        with_kt<1>(p.K, [&](auto kt) { k_mw_run<1, decltype(kt)::value><<<g, BLOCK, 0, s>>>(p, t.slots, t.cap, mw, stats); });
    else
        with_kt<2>(p.K, [&](auto kt) { k_mw_run<2, decltype(kt)::value><<<g, BLOCK, 0, s>>>(p, t.slots, t.cap, mw, stats); });
    return hipGetLastError();
}

hipError_t launch_mw_text_offsets(const MWalkRound& mw, uint64_t* off, uint64_t* scratch,
                                  unsigned long long* store_n, hipStream_t s) {
    if (mw.n_in == 0) return hipSuccess;
    // offsets continue the store's running count (store_n, on the device: no host round trip)
    return scan_exclusive(NrecF{mw.nrec, mw.n_dev}, mw.n_in, off, scratch, store_n, (unsigned long long*)nullptr, s);
}

hipError_t launch_mw_compact(const MWalkRound& mw, const uint64_t* off, uint64_t* store, uint64_t store_cap,
                             unsigned long long* stats, hipStream_t s) {
    if (mw.n_in == 0) return hipSuccess;
    k_mw_compact<<<grid_for(mw.n_in, 4096), BLOCK, 0, s>>>(mw.stage, mw.nrec, off, mw.n_in, store, mw.n_dev, store_cap,
                                                           stats);
    return hipGetLastError();
}

hipError_t launch_mw_group(const MWalkRound& mw, uint64_t* hist, uint64_t* off, uint64_t* scratch,
                           uint64_t* out, uint64_t* counts, hipStream_t s) {
    unsigned long long* total = reinterpret_cast<unsigned long long*>(scratch);
    return group_by_owner(MsgOp{mw.dst, mw.tmp, out}, mw.n_in, mw.P, hist, off, scratch + 1, counts, total, s);
}

// one rank: every record's origin is this rank, so grouping is a copy of the n_dev records
__global__ __launch_bounds__(BLOCK) void k_mw_text_copy(const uint64_t* recs, uint64_t n_max,
                                                        const unsigned long long* n_dev, uint64_t* out,
                                                        uint64_t* counts) {
    const uint64_t n = min((uint64_t)*n_dev, n_max);
    if (blockIdx.x == 0 && threadIdx.x < 2) counts[threadIdx.x] = n;
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BLOCK)
        reinterpret_cast<ulonglong2*>(out)[i] = reinterpret_cast<const ulonglong2*>(recs)[i];
}

hipError_t launch_mw_group_text(const uint64_t* recs, uint64_t n, uint32_t P, uint64_t* hist, uint64_t* off,
                                uint64_t* scratch, uint64_t* out, uint64_t* counts, hipStream_t s,
                                const unsigned long long* n_dev) {
    if (P == 1 && n_dev) {  // (the histogram + scan + scatter: 0.15 ms at C3; the copy ~0.05)
        k_mw_text_copy<<<grid_for(n, 4096), BLOCK, 0, s>>>(recs, n, n_dev, out, counts);
        return hipGetLastError();
    }
    unsigned long long* total = reinterpret_cast<unsigned long long*>(scratch);
    return group_by_owner(RecOp{recs, out, n_dev, P}, n, P, hist, off, scratch + 1, counts, total, s);
}

// ---- fixed-size exchange slots ---------------------------------------------------------------------
// prefix of the P slot counts (clamped to cap) in LDS; returns the total
__device__ __forceinline__ uint64_t slot_prefix(const uint64_t* slots, uint32_t P, uint64_t cap, uint64_t* pre) {
    __shared__ uint64_t tot;
    if (threadIdx.x == 0) {
        uint64_t a = 0;
        for (uint32_t q = 0; q < P; ++q) {
            pre[q] = a;
            const uint64_t c = slots[q * slot_words(cap)];
            a += c < cap ? c : cap;
        }
        pre[P] = a;
        tot = a;
    }
    __syncthreads();
    return tot;
}

__global__ __launch_bounds__(BLOCK) void k_slot_gather(const uint64_t* slots, uint32_t P, uint64_t cap, uint64_t* list,
                                                       unsigned long long* n, uint64_t n_max,
                                                       unsigned long long* stats) {
    __shared__ uint64_t pre[MAX_RANKS + 1];
    // the list holds n_max messages (walkers never multiply; more is a sender's bug: reported at
    // kh_sync as an overflow in the round it happens, the messages past n_max are not walked)
    const uint64_t all = slot_prefix(slots, P, cap, pre), tot = min(all, n_max);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        *n = tot;
        if (all > n_max) atomicAdd(&stats[ST_CHUNK_OVF], 1ull);
    }
    for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < tot; i += (uint64_t)gridDim.x * BLOCK) {
        uint32_t q = 0;
        while (q + 1 < P && pre[q + 1] <= i) ++q;
        const uint64_t* src = slots + q * slot_words(cap) + 2 + (i - pre[q]) * MSG_WORDS;
        uint64_t* d = list + i * MSG_WORDS;
#pragma unroll
        for (int w = 0; w < MSG_WORDS; ++w) d[w] = src[w];
    }
}

hipError_t launch_slot_gather(const uint64_t* slots, uint32_t P, uint64_t cap, uint64_t* list,
                              unsigned long long* n, uint64_t n_max, hipStream_t s, unsigned long long* stats) {
    k_slot_gather<<<grid_for((uint64_t)P * cap, 4096), BLOCK, 0, s>>>(slots, P, cap, list, n, n_max, stats);
    return hipGetLastError();
}

// outgoing messages of a round: last round's held-back ones first (they go out before newer
// ones to the same destination), then the walk outputs with a destination; each lands straight in
// its destination's slot, or past the slot's capacity in the held-back list
struct SlotMsgOp {
    SlotRound r;
    const uint64_t* off;   // owner-major exclusive scan of the per-block counts (start of q's run)
    uint64_t nbk;          // blocks of the grouping
    const uint64_t* cbase; // held-back list position of each destination's overflow
    __device__ int owner(uint64_t i) const {
        if (i < r.cb) return i < *r.carry_n ? (int)r.carry_dst[i] : -1;
        const uint64_t j = i - r.cb;
        return (j < *r.n_dev && j < r.nb && r.dst[j] != MW_NONE) ? (int)r.dst[j] : -1;
    }
    __device__ void emit(uint64_t i, int q, uint64_t d) const {
        if (q < 0) return;
        const uint64_t* a = i < r.cb ? r.carry + i * MSG_WORDS : r.tmp + (i - r.cb) * MSG_WORDS;
        const uint64_t k = d - off[(uint64_t)q * nbk];  // rank among the messages to q
        uint64_t* b;
        if (k < r.cap) {
            b = r.out + (uint64_t)q * slot_words(r.cap) + 2 + k * MSG_WORDS;
        } else {  // slot full: held back for a later round (rare)
            const uint64_t c = cbase[q] + (k - r.cap);
            b = r.carry_out + c * MSG_WORDS;
            r.carry_dst_out[c] = (uint8_t)q;
        }
#pragma unroll
        for (int w = 0; w < MSG_WORDS; ++w) b[w] = a[w];
    }
};

// slot headers, the held-back list's per-destination bases and its length, live = [messages in
// flight, largest per-destination count]
__global__ void k_slot_heads(SlotRound r, uint64_t* cbase) {
    if (threadIdx.x == 0) {
        uint64_t tot = 0, mx = 0, over = 0;
        for (uint32_t q = 0; q < r.P; ++q) {
            const uint64_t c = r.cnt[q];
            r.out[q * slot_words(r.cap)] = c < r.cap ? c : r.cap;
            r.out[q * slot_words(r.cap) + 1] = 0;
            cbase[q] = over;
            over += c > r.cap ? c - r.cap : 0;
            tot += c;
            mx = c > mx ? c : mx;
        }
        *r.carry_n_out = over;
        r.live[0] = tot;
        r.live[1] = mx;
    }
}

hipError_t launch_slot_round(const SlotRound& r, uint64_t* hist, uint64_t* off, uint64_t* scratch, hipStream_t s) {
    const uint64_t n = r.nb + r.cb;
    const uint64_t nbk = route_blocks(n);
    unsigned long long* total = reinterpret_cast<unsigned long long*>(scratch);
    uint64_t* cbase = r.cnt + r.P + 1;  // cnt holds 2P + 1 words
    SlotMsgOp op{r, off, nbk, cbase};
    if (nbk == 0) {  // nothing in flight: empty slots
        hipError_t e = hipMemsetAsync(r.cnt, 0, (r.P + 1) * 8, s);
        if (e != hipSuccess) return e;
        k_slot_heads<<<1, 64, 0, s>>>(r, cbase);
        return hipGetLastError();
    }
    k_group_hist<SlotMsgOp><<<(unsigned)nbk, BLOCK, 0, s>>>(op, n, r.P, hist);
    hipError_t e = scan_exclusive(HistF{hist, nbk, r.P}, nbk * r.P, off, scratch + 1, (unsigned long long*)nullptr,
                                  total, s);
    if (e != hipSuccess) return e;
    k_route_counts<0><<<1, MAX_RANKS, 0, s>>>(off, nbk, r.P, total, r.cnt);
    k_slot_heads<<<1, 64, 0, s>>>(r, cbase);
    k_group_scatter<SlotMsgOp><<<(unsigned)nbk, BLOCK, 0, s>>>(op, n, r.P, off, nbk);
    return hipGetLastError();
}

// [walks' overflow / overlap reports (ST_CHUNK_OVF), text records the store needed]
// out[0]: overlap / overflow reports, + 2^40 when a short walk met a long contig
__global__ void k_mw_flags(const unsigned long long* ovf, const unsigned long long* store_n, uint64_t* out,
                           const unsigned long long* long_ctr) {
    out[0] = *ovf + ((long_ctr && *long_ctr) ? (1ull << 40) : 0ull);
    out[1] = *store_n;
}

hipError_t launch_mw_flags(const unsigned long long* ovf, const unsigned long long* store_n, uint64_t* out,
                           hipStream_t s, const unsigned long long* long_ctr) {
    k_mw_flags<<<1, 1, 0, s>>>(ovf, store_n, out, long_ctr);
    return hipGetLastError();
}

__global__ void k_add_count(unsigned long long* out, uint64_t a, const unsigned long long* b, uint64_t bmax) {
    const uint64_t v = b ? (uint64_t)*b : 0;
    *out = a + (v < bmax ? v : bmax);
}

hipError_t launch_add_count(unsigned long long* out, uint64_t a, const unsigned long long* b, uint64_t bmax,
                            hipStream_t s) {
    k_add_count<<<1, 1, 0, s>>>(out, a, b, bmax);
    return hipGetLastError();
}

__global__ void k_fin_check(const unsigned long long* fin, uint64_t want, const unsigned long long* want_dev,
                            uint64_t want_max, unsigned long long* stats) {
    uint64_t w = want;
    if (want_dev) w += (uint64_t)*want_dev < want_max ? (uint64_t)*want_dev : want_max;
    if ((uint64_t)*fin != w) atomicAdd(&stats[ST_MISSING], 1ull);
}

hipError_t launch_fin_check(const unsigned long long* fin, uint64_t want, const unsigned long long* want_dev,
                            uint64_t want_max, unsigned long long* stats, hipStream_t s) {
    k_fin_check<<<1, 1, 0, s>>>(fin, want, want_dev, want_max, stats);
    return hipGetLastError();
}

hipError_t launch_mw_lens(const uint64_t* recs, uint64_t n, uint64_t nc, uint32_t* len, unsigned long long* fin,
                          hipStream_t s, uint64_t* chunk_data) {
    if (n == 0) return hipSuccess;
    k_mw_lens<<<grid_for(n, 2048), BLOCK, 0, s>>>(recs, n, nc, len, fin, chunk_data);
    return hipGetLastError();
}

hipError_t launch_mw_words(int K, const uint64_t* recs, uint64_t n, uint64_t nc, const uint32_t* len,
                           const uint64_t* off, char* out, uint64_t cap, hipStream_t s, uint32_t wmin) {
    if (n == 0) return hipSuccess;
    k_mw_words<<<grid_for(n, 8192), BLOCK, 0, s>>>(K, recs, n, nc, len, off, out, cap, wmin);
    return hipGetLastError();
}


}  // namespace kh
