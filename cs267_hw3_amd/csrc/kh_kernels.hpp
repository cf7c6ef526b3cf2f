// kh_kernels.hpp — launch wrappers for the gfx950 k-mer table / contig walker kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kh_codec.hpp"

namespace kh {

// KH_DEBUG = comma-separated test switches (e.g. "plain_build"); not for production runs.
bool debug_flag(const char* name);

// Device-side error / event counters (one 64-bit word each).
enum StatIdx : int {
    ST_DUP = 0,        // duplicate key on insert (input contract: keys unique, README.md:35)
    ST_FULL = 1,       // probe wrapped the whole table
    ST_BAD_EXT = 2,    // extension byte not in {A,C,G,T,F}
    ST_MISSING = 3,    // walk: next k-mer absent (kmer_hash.cpp:47-49 throws)
    ST_CYCLE = 4,      // walk: more steps than k-mers in the table (no 'F' terminator)
    ST_SPIN = 5,       // insert: gave up waiting for a half-published 16 B slot
    ST_CHUNK_OVF = 6,  // walk: contig chunk pool exhausted (sized as an upper bound; never expected)
    ST_BAD_BASE = 7,   // text parse: k-mer character outside {A,C,G,T}
    ST_NUM = 8
};

// Device counters used by the host-side orchestration.
enum CtrIdx : int {
    CT_N_STARTS = 0,   // start k-mers collected so far (all insert calls)
    CT_WALK_NEXT = 1,  // walker work-queue head
    CT_CHUNK_NEXT = 2, // chunk allocator head
    CT_OUT_BYTES = 3,  // total contig bytes (incl. '\n')
    CT_OVF = 4,        // partitioned build: keys whose probe run left their region
    CT_MW_FIN = 5,     // migrating walk: finish records received by the origin
    CT_N_SPLIT = 6,    // splitter k-mers collected (walk segments beyond the contig starts)
    CT_N_SPLIT_W = 7,  // splitters of the walk subset (denser collection filtered at assemble)
    CT_OVF2 = 8,       // partitioned build: keys left for the global CAS insert (full windows, probe
                       // runs that left their slice) after the hot-region fixup
    CT_HOT = 9,        // remapped ("hot") placement regions of the table (kh_build.hip k_hot_mark)
    CT_HOTNEW = 10,    // regions the last exact mark remapped (their window words move: k_hot_gather)
    CT_HOT2 = 11,      // level-2 marks: target regions whose remapped keys spread by key hash
    CT_NUM = 12
};

// Several fills in one launch (each hipMemsetAsync is a ~5 us dispatch of its own): up to
// FILL_MAX buffers of whole 4-byte words, each set to a byte value. Null / empty entries are skipped.
static constexpr int FILL_MAX = 6;
struct FillSet {
    void* p[FILL_MAX] = {};
    uint64_t bytes[FILL_MAX] = {};
    uint32_t byte[FILL_MAX] = {};
    int n = 0;
    void add(void* ptr, uint64_t nbytes, uint32_t value) {
        p[n] = ptr;
        bytes[n] = nbytes;
        byte[n] = value & 0xFFu;
        ++n;
    }
};
hipError_t launch_fill(const FillSet& f, hipStream_t s);

// Chunk of appended bases: 8 words x 32 bases (2 bits each) = 256 bases.
static constexpr int CHUNK_WORDS = 8;
static constexpr uint32_t WMIN_ERR = 0xFFFFFFFFu;  // origin_lines (kh_capi.cpp): no memory
static constexpr int CHUNK_BASES = 256;

struct TableView {
    uint64_t* slots;   // W words per slot, cap slots
    uint64_t cap;
};

// Insert records (reference kmer_pair layout, R bytes each, 16-B aligned base) into the table.
// Writes one start bit per record (bwd == 'F') into start_mask[i/64].
hipError_t launch_insert(const KParams& p, const uint8_t* recs, uint64_t n, TableView t,
                         uint64_t* start_mask, uint64_t* split_mask, unsigned long long* stats, hipStream_t s);

// Append start k-mers of a batch, in record order, to starts (W words each) at
// ctr[CT_N_STARTS]. scratch must hold >= scan_scratch_words(ceil(n/64)) words.
hipError_t launch_collect_starts(const KParams& p, const uint8_t* recs, uint64_t n,
                                 const uint64_t* start_mask, uint64_t* mask_offsets,
                                 uint64_t* scratch, uint64_t* starts, unsigned long long* ctr,
                                 hipStream_t s, int ctr_idx = CT_N_STARTS);

// Explicit start list (caller's start_nodes): R-byte records -> start words, sets CT_N_STARTS.
hipError_t launch_load_starts(const KParams& p, const uint8_t* recs, uint64_t n, uint64_t* starts,
                              unsigned long long* ctr, hipStream_t s);

// Batched find: keys are PACKED bytes each; out gets R-byte records, found 0/1.
hipError_t launch_find(const KParams& p, const uint8_t* keys, uint64_t n, TableView t, uint8_t* out,
                       uint8_t* found, hipStream_t s);

struct WalkBuffers {
    const uint64_t* starts;
    uint64_t n_starts;
    // splitter walkers (segments n_starts .. n_starts + n_splits - 1); contig_len/chunks are then
    // per segment and seg_next/seg_key record where a segment stopped (see k_walk)
    const uint64_t* splits;
    uint64_t n_splits;                         // host bound (sizes, grids)
    const unsigned long long* n_splits_dev;    // exact count on the device when set
    uint32_t* seg_next;       // next segment, SEG_NONE, or SEG_AT_SPLIT (resolved by k_seg_link)
    uint64_t* seg_key;        // 2 words per segment: the splitter k-mer it stopped before
    uint32_t* contig_len;     // k-mers per contig (>= 1); per segment when n_splits > 0
    uint64_t* chunk_data;     // chunk_cap * CHUNK_WORDS
    uint32_t* chunk_owner;    // contig id of each chunk
    uint32_t* chunk_seq;      // chunk index within its contig
    uint64_t chunk_cap;
    uint64_t max_steps;
    // chain head records of the last region build (kh_build.hip region_chains); hcap 0 = none
    const uint64_t* headrec = nullptr;
    uint32_t hcap = 0;
    // bytes of the text buffer the materialisation writes into (0: sized from the scanned total);
    // a contig that would pass it is not written (the caller compares the total with it)
    uint64_t text_cap = 0;
    // work-queue batches a wave reserves per atomic (0: WALK_BATCHES); kh_assemble_dev takes 32
    // for short contigs (C5: 21M contigs of ~9 k-mers), where the queue's one counter is the limit
    uint32_t batches = 0;
    // Deferred splitter segments (split_min > 0): a contig's walker stops before a splitter only
    // once it has appended split_min bases, and then sets seg_long[0]; splitter walkers reached in
    // the queue before that are deferred (seg_long[1]) to a second launch (phase 1), which walks
    // them only if some contig did stop at a splitter (k_walk_q). Contigs shorter than split_min
    // (C3: all) then need no splitter segment at all. The splitter segments' contig_len must be 0
    // before phase 0 (phase 1 walks those still 0).
    uint32_t split_min = 0;
    uint32_t* seg_long = nullptr;  // 4 words (k_walk_q, k_stab_gate)
    uint32_t phase = 0;
};

// Persistent per-lane walker (single GPU): every lane walks whole contigs, pulling start k-mers
// from a wave-batched work queue.
// head records' successor runs (before a walk; KH_REC_SUCC=0 skips it: the walker then probes)
bool rec_succ_fits(const KParams& p, uint32_t hcap);
bool rec_succ_side(const KParams& p);
hipError_t launch_rec_succ(const KParams& p, TableView t, uint64_t* headrec, uint32_t hcap, hipStream_t s,
                           unsigned blocks = 0);
// grid_blocks > 0: that many blocks; <= 0: -grid_blocks blocks per CU (0: two)
hipError_t launch_walk(const KParams& p, TableView t, const WalkBuffers& wb, unsigned long long* ctr,
                       unsigned long long* stats, int grid_blocks, hipStream_t s);

static constexpr uint32_t SEG_NONE = 0xFFFFFFFFu, SEG_AT_SPLIT = 0xFFFFFFFEu;

// Splitter segments -> contigs: a small open-addressing table of the splitter k-mers (key -> id),
// segment links, then per contig the chain of its segments (contig_len = final k-mers per contig,
// seg_contig/seg_off = where each segment's bases go).
struct SegBuffers {
    uint64_t* stab;        // cap2 * 2 words (key lo, key hi)
    uint32_t* stab_id;     // cap2
    uint64_t cap2;
    uint32_t* seg_contig;  // nseg
    uint32_t* seg_off;     // nseg: bases of the contig before this segment
    uint32_t* clen;        // n_starts: final contig k-mers
    uint32_t* jump;        // nseg: the segment SEG_JUMP links ahead (k_seg_chain)
    uint32_t* jsum;        // nseg: bases of the SEG_JUMP segments from this one
    uint8_t* anchor;       // nseg: a contig's walk over jump pointers visited this segment
    uint32_t* pend;        // n_starts: segment where a contig's serial walk stopped (SEG_NONE: done)
    uint32_t* long_flag;   // one word: some contig has more than `serial` segments
    uint32_t serial = 0;   // segments a contig's thread follows before the jump passes (launch_segments)
};
// splits with (hash & (2^bits - 1)) == 0 -> out (count to *count)
hipError_t launch_filter_splits(const KParams& p, const uint64_t* splits, uint64_t n, int bits, uint64_t* off,
                                uint64_t* scratch, uint64_t* out, unsigned long long* count, hipStream_t s);
// after: the second launch of deferred splitter segments (builds the table only if the first,
// beside the walk, did not and some contig stopped at a splitter)
hipError_t launch_seg_table(const KParams& p, const WalkBuffers& wb, const SegBuffers& sb, hipStream_t s,
                            bool after = false);
hipError_t launch_segments(const KParams& p, const WalkBuffers& wb, const SegBuffers& sb,
                           unsigned long long* stats, hipStream_t s);
// phases: MAT_SCAN = offsets + ctr[CT_OUT_BYTES]; MAT_WRITE = the text (out must hold the
// scanned total: callers size it from CT_OUT_BYTES between the two phases)
enum MatPhase : int { MAT_SCAN = 1, MAT_WRITE = 2, MAT_ALL = 3 };
hipError_t launch_materialize_seg(const KParams& p, const WalkBuffers& wb, const SegBuffers& sb,
                                  uint64_t* offsets, uint64_t* scratch, char* out, unsigned long long* ctr,
                                  hipStream_t s, int phases = MAT_ALL, uint32_t* line_first = nullptr,
                                  uint64_t out_bytes = 0);

// Contig bytes: offsets = exclusive scan of (K + len) (K + len-1 bases + '\n'), then write chars.
hipError_t launch_materialize(const KParams& p, const WalkBuffers& wb, uint64_t* offsets,
                              uint64_t* scratch, char* out, unsigned long long* ctr, hipStream_t s,
                              int phases = MAT_ALL, uint32_t* line_first = nullptr, uint64_t out_bytes = 0);
// line_first: LINE_WORDS(out_bytes) uint32 entries for the line writer (K >= 16), or nullptr
inline uint64_t line_first_words(uint64_t out_bytes) { return out_bytes / 1024 + 2; }
// The line writer alone (K >= 16; false otherwise, nothing launched): heads, the first
// CHUNK_BASES bases of each contig's first segment from wb.chunk_data (word-major chunk c =
// contig c, chunk_cap = wb.chunk_cap), newlines; wb.contig_len[c] + slen_add = that segment's
// k-mers. Bytes past the first chunk are left to a writer that runs after it.
bool launch_text_lines(const KParams& p, const WalkBuffers& wb, const uint32_t* clen, int slen_add,
                       const uint64_t* offsets, char* out, const unsigned long long* ctr, hipStream_t s, uint64_t cap,
                       uint32_t* line_first, uint64_t out_bytes);

// ---- migrating-walker rounds (kh_mwalk.hip) -------------------------------------------------
// message: MSG_WORDS words [key.hi, key.lo, partial word, idx << 32 | bases appended,
// origin | state << 8]; text record: 2 words [origin << 56 | fin << 55 | word_no << 31 | idx,
// word (or bases appended, fin)].
static constexpr int MSG_WORDS = 5;
static constexpr int MW_RUN_WORDS = 8;                  // words a walker may flush per round
static constexpr int MW_REC_SLOTS = MW_RUN_WORDS + 4;   // + final partial word + finish + 2 link records
struct MWalkRound {
    uint32_t P, rank;
    uint32_t split_bits = 0;  // > 0: walkers stop before splitter k-mers (kh_mseg.hip)
    uint64_t max_steps;
    const uint64_t* in;   // n_in messages; null in the first round: the walkers are the start
                          // k-mers (starts[0, ns)) and then the splitters (splits), read directly
    const uint64_t* starts = nullptr;
    const uint64_t* splits = nullptr;
    uint64_t ns = 0;
    uint64_t n_in;        // bound (grids, buffers)
    const unsigned long long* n_dev = nullptr;  // live inputs on the device (null: n_in)
    const unsigned long long* hot_on = nullptr;  // ctr[CT_HOT]: remapped regions exist (null: use p.hot)
    uint64_t* tmp;        // n_in * MSG_WORDS: outgoing message of input j
    uint8_t* dst;         // n_in: its destination rank (0xFF = finished)
    uint64_t* stage;      // n_in * MW_REC_SLOTS * 2: text records of input j
    uint8_t* nrec;        // n_in
    const uint64_t* headrec = nullptr;  // chain head records of this shard's build (hcap 0 = none)
    uint32_t hcap = 0;
    // short walk (kh_mwalk_short): a walker past soft_steps bases ends, counted in *long_ctr (the
    // hosts then walk again with splitter segments)
    uint64_t soft_steps = 0;
    unsigned long long* long_ctr = nullptr;
};

// ---- splitter segments of the migrating walk (kh_mseg.hip) ----------------------------------
struct MSegState {       // per local segment: starts [0, ns), splitter segments [ns, ns + nsp)
    uint32_t* len;       // bases appended by the segment's walker
    uint64_t* link_hi;   // key of the splitter it stopped before
    uint64_t* link_lo;
    uint8_t* has_link;
    uint8_t* done;       // head known
    uint64_t* jump;      // pointer-jumping target (gid = rank << 40 | index); when done: head
    uint64_t* acc;       // bases from the start of `jump` to this segment; when done: offset
};
hipError_t launch_split_collect(const KParams& p, const uint64_t* words, uint64_t m, uint64_t* out, uint64_t cap,
                                unsigned long long* ctr, hipStream_t s);
hipError_t launch_mseg_stab(const KParams& p, const uint64_t* splits, uint64_t nsp, uint64_t* stab, uint32_t* id,
                            uint64_t cap2, hipStream_t s);
hipError_t launch_mseg_init(uint64_t ns, uint64_t nseg, uint32_t rank, const MSegState& st, hipStream_t s);
// chunk_data (K >= 16, else null): start segments' first CHUNK_WORDS words into word-major first
// chunks (chunk c = contig c < ns); *late counts their later words
hipError_t launch_mseg_scan(const uint64_t* recs, uint64_t n, uint64_t nseg, const MSegState& st,
                            unsigned long long* fin, hipStream_t s, uint64_t* chunk_data = nullptr, uint64_t ns = 0,
                            unsigned long long* late = nullptr);
hipError_t launch_mseg_link(const KParams& p, const MSegState& st, uint64_t ns, uint64_t nseg, uint32_t P, uint32_t rank,
                            uint64_t* hist, uint64_t* off, uint64_t* scratch, uint64_t* out, uint64_t* counts,
                            hipStream_t s);
hipError_t launch_mseg_pred(const uint64_t* msgs, uint64_t m, const uint64_t* stab, const uint32_t* id, uint64_t cap2,
                            uint64_t ns, const MSegState& st, unsigned long long* stats, hipStream_t s);
// this rank's splitter segments' {predecessor id, predecessor length} (stride entries, the tail
// past *nsp = none), for the all-gather of every rank's table
hipError_t launch_mseg_preds_out(const MSegState& st, uint64_t ns, const unsigned long long* nsp, uint64_t nsp_max,
                                 uint64_t stride, uint64_t* out, hipStream_t s);
uint32_t mseg_resolve_passes(uint64_t N);
// pointer jumping over the gathered tables (N = P * stride entries, buffers of N each, pend:
// mseg_resolve_passes(N) words) -> head and offset of this rank's splitter segments
hipError_t launch_mseg_resolve(const uint64_t* all, uint64_t N, uint64_t stride, uint32_t rank, uint64_t ns,
                               const unsigned long long* nsp, uint64_t nsp_max, const MSegState& st, uint64_t* J0,
                               uint64_t* A0, uint8_t* D0, uint64_t* J1, uint64_t* A1, uint8_t* D1,
                               unsigned long long* pend, hipStream_t s);
hipError_t launch_mseg_check(uint64_t ns, uint64_t nseg, const MSegState& st, const unsigned long long* nsp,
                             unsigned long long* stats, hipStream_t s);
hipError_t launch_mseg_retag(const uint64_t* recs, uint64_t n, uint64_t ns, uint64_t nsp, const MSegState& st,
                             uint32_t P, uint64_t* hist, uint64_t* off, uint64_t* scratch, uint64_t* out,
                             uint64_t* counts, hipStream_t s);
hipError_t launch_mseg_lens(const uint64_t* in3, uint64_t m, uint64_t ns, const MSegState& st, uint32_t* contig_len,
                            hipStream_t s);
hipError_t launch_mseg_words(int K, const uint64_t* recs, uint64_t n, const uint64_t* in3, uint64_t m, uint64_t ns,
                             const MSegState& st, const uint64_t* off, char* out, uint64_t cap, hipStream_t s,
                             uint32_t wmin, const unsigned long long* late = nullptr);
hipError_t launch_mw_run(const KParams& p, TableView t, const MWalkRound& mw, unsigned long long* stats,
                         hipStream_t s);
// ---- fixed-size exchange slots (no host read per round) ----------------------------------------
// A round's exchange buffer is P slots of slot_words(cap) words: [count, 0, cap messages].
__host__ __device__ inline uint64_t slot_words(uint64_t cap) { return 2 + cap * MSG_WORDS; }
// messages of P slots -> list (contiguous, n_max at most), *n = their number
hipError_t launch_slot_gather(const uint64_t* slots, uint32_t P, uint64_t cap, uint64_t* list,
                              unsigned long long* n, uint64_t n_max, hipStream_t s, unsigned long long* stats);
// this round's outgoing messages (walk outputs j < *n_dev with a destination, then the messages
// held back last round) -> P slots of cap (overflow held back in carry_out / carry_dst_out,
// *carry_n_out); live = [messages in flight, largest per-destination count].
struct SlotRound {
    uint32_t P;
    uint64_t nb;                     // walk outputs (bound)
    const unsigned long long* n_dev; // walk outputs live
    const uint8_t* dst;              // their destination (MW_NONE: finished)
    const uint64_t* tmp;             // their messages
    uint64_t cb;                     // held-back messages (bound)
    const unsigned long long* carry_n;
    const uint8_t* carry_dst;
    const uint64_t* carry;
    uint64_t cap;
    uint64_t* out;                   // P slots
    uint64_t* carry_out;
    uint8_t* carry_dst_out;
    unsigned long long* carry_n_out;
    unsigned long long* live;        // 2 words
    uint64_t* cnt;                   // 2P + 1 words of scratch
};
hipError_t launch_slot_round(const SlotRound& r, uint64_t* hist, uint64_t* off, uint64_t* scratch, hipStream_t s);
// *out = a + min(*b, bmax) (the first round's live walkers: starts + collected splitters)
hipError_t launch_add_count(unsigned long long* out, uint64_t a, const unsigned long long* b, uint64_t bmax,
                            hipStream_t s);
// text records of this round: absolute store offsets continuing *store_n (device counter, updated)
hipError_t launch_mw_text_offsets(const MWalkRound& mw, uint64_t* off, uint64_t* scratch,
                                  unsigned long long* store_n, hipStream_t s);
// store_cap: the store's records; a round that would pass it fails the walk (ST_CHUNK_OVF)
hipError_t launch_mw_compact(const MWalkRound& mw, const uint64_t* off, uint64_t* store, uint64_t store_cap,
                             unsigned long long* stats, hipStream_t s);
hipError_t launch_mw_group(const MWalkRound& mw, uint64_t* hist, uint64_t* off, uint64_t* scratch,
                           uint64_t* out, uint64_t* counts, hipStream_t s);
hipError_t launch_mw_group_text(const uint64_t* recs, uint64_t n, uint32_t P, uint64_t* hist, uint64_t* off,
                                uint64_t* scratch, uint64_t* out, uint64_t* counts, hipStream_t s,
                                const unsigned long long* n_dev = nullptr);
// *fin != want (+ *want_dev) -> stats[ST_MISSING] (walkers that never came home)
hipError_t launch_mw_flags(const unsigned long long* ovf, const unsigned long long* store_n, uint64_t* out,
                           hipStream_t s, const unsigned long long* long_ctr = nullptr);
hipError_t launch_fin_check(const unsigned long long* fin, uint64_t want, const unsigned long long* want_dev,
                            uint64_t want_max, unsigned long long* stats, hipStream_t s);
hipError_t launch_mw_lens(const uint64_t* recs, uint64_t n, uint64_t nc, uint32_t* len,
                          unsigned long long* fin, hipStream_t s, uint64_t* chunk_data = nullptr);
// cap: bytes of `out` (words past it are skipped: a bad length fails at kh_sync, never overruns)
hipError_t launch_mw_words(int K, const uint64_t* recs, uint64_t n, uint64_t nc, const uint32_t* len,
                           const uint64_t* off, char* out, uint64_t cap, hipStream_t s, uint32_t wmin);

// read_kmers.hpp:62-76 on the device: n fixed-width "KMER BF\n" lines (K+4 bytes) -> kmer_pair
// records; lines with a non-ACGT k-mer character count in stats[ST_BAD_BASE].
hipError_t launch_pack_text(const KParams& p, const char* text, uint64_t n, uint8_t* recs,
                            unsigned long long* stats, hipStream_t s);

// Pieces of the materialisation for other walkers: offsets (+ total bytes) and start k-mer heads
// (with the trailing '\n' at off + K + len - 1).
hipError_t launch_contig_offsets(int K, const uint32_t* len, uint64_t nc, uint64_t* offsets,
                                 uint64_t* scratch, unsigned long long* total, hipStream_t s);
// cap: bytes of `out` (contigs past it are skipped; default: unbounded)
hipError_t launch_write_heads(const KParams& p, const uint64_t* starts, uint64_t nc, const uint32_t* len,
                              const uint64_t* offsets, char* out, hipStream_t s, uint64_t cap = ~0ull);

// Scratch words needed by the scans for m elements.
uint64_t scan_scratch_words(uint64_t m);

}  // namespace kh

// ---- sharded multi-GPU path (one table per rank; the exchange itself is the caller's) -------
namespace kh {

// Items per block of the owner-routing kernels (histogram / scatter).
static constexpr int ROUTE_TILE = 2048;
static constexpr int MAX_RANKS = 64;
inline uint64_t route_blocks(uint64_t n) { return (n + ROUTE_TILE - 1) / ROUTE_TILE; }

// Start bits only (no insert): bwd == 'F' per record, wave ballot -> start_mask[i/64].
hipError_t launch_start_mask(const KParams& p, const uint8_t* recs, uint64_t n, uint64_t* start_mask,
                             hipStream_t s);

// Records -> internal words (W per record) grouped by owner rank (owner_key).
// hist/off: route_blocks(n) * nranks words each; counts: nranks + 1 words (last = n).
hipError_t launch_route(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t nranks,
                        uint64_t* hist, uint64_t* off, uint64_t* scratch, uint32_t* own, uint64_t* out_words,
                        uint64_t* counts, hipStream_t s, uint64_t* start_mask = nullptr,
                        unsigned long long* spl = nullptr);

// Insert routed internal words.
hipError_t launch_insert_words(const KParams& p, const uint64_t* words, uint64_t m, TableView t,
                               unsigned long long* stats, hipStream_t s);

}  // namespace kh

// ---- partitioned (atomic-free) bulk build ------------------------------------------------------
namespace kh {

// The key space is cut into 2^rbits regions (kh_codec.hpp place: a hash of the minimizer); because the home slot
// mulhi(h, cap) is monotonic in h, region r owns the slot range
// [floor(r*cap/2^17), floor((r+1)*cap/2^17)). Two windowed LDS-sort passes (512 buckets, then 256
// bins per bucket) group the batch by region, then one workgroup per region builds its slot range
// in LDS (kh_build.hip).
static constexpr int PART_TILE = 4096;  // records per block-tile of k_part1_convert

static constexpr uint32_t PART_W1_COUNTERS = 512 * 8;  // pass-1 windows: 512 buckets x 8
uint64_t part_count_words();                      // words of the pass-1 + pass-2 window counters
uint64_t part_overflow_cap(uint64_t n);           // overflow entries
uint32_t part_region_cap(const KParams& p, uint64_t n);  // words per region window of pass 2
uint64_t part_buf2_words(const KParams& p, uint64_t n);  // buf2 size (region windows or n * W)
uint32_t part_win1_cap(uint64_t n);               // words per pass-1 window
uint64_t part_buf1_words(const KParams& p, uint64_t n);  // buf1 size (pass-1 windows or n * W)
// True when the region slices fit LDS and the batch is large enough to be worth it.
bool part_usable(const KParams& p, uint64_t cap, uint64_t n);
// True when every region slice fits LDS (forced partitioned mode for tests of small batches).
bool region_slots_fit(const KParams& p, uint64_t cap);

struct PartBuffers {
    uint64_t* buf1;      // part_buf1_words(p, n) words: pass-1 windows; after pass 2 the list of
                         // keys left for the global CAS insert (counter CT_OVF2)
    uint64_t* buf2;      // part_buf2_words(p, n) words: region windows
    uint32_t* wcnt;      // pass-1 window fill counters
    uint32_t* rcnt;      // region window fill counters
    uint32_t* hot_list;  // remapped regions of this build (NREG_MAX; wcnt + rcnt + hot_list = part_count_words())
    uint64_t* overflow;  // part_overflow_cap(n) * W words: words that missed their pass-1/2 window (CT_OVF)
    uint32_t* hot;       // the table's remapped-region bitmap (KParams::hot, writable)
    const uint64_t* rbt; // region slot ranges (equal or balanced: KParams::rb), read by the build
    uint64_t* headrec = nullptr;  // 2^rbits * hcap chain head records of 2 words (null: no chains)
    uint32_t hcap = 0;
};
// Bitmap words of the remapped-region set (one bit per region, 2^17 regions at most).
static constexpr uint32_t HOT_WORDS = HOT_LEVEL_WORDS;  // one level of the hot bitmap (two levels)

// Balanced region bounds (KParams::rb) from region counts (nullptr: equal ranges).
// rb: the table's bounds (2^rbits + 1 words); counts nullptr: equal ranges (the build kernels read
// every region's slot range from rb, balanced or not)
void launch_bounds(const KParams& p, uint64_t cap, const uint32_t* counts, uint32_t RC, uint64_t* rb, hipStream_t s);

// CAS-path inserts into an empty table (batches too small for the partitioned build): count the
// batch's keys per minimizer region and remap the regions that cannot hold theirs (records or
// routed words), so a repeat family does not pile up one linear-probing run.
// total: the whole build when this batch is the first of several staged ones (its counts are then
// scaled up to it); 0 = this batch is the build
hipError_t launch_hot_prepass(const KParams& p, const uint8_t* recs, const uint64_t* words, uint64_t n,
                              uint64_t cap, uint32_t* rcnt, uint32_t* hot, uint32_t* hot_list,
                              unsigned long long* ctr, hipStream_t s, uint64_t total = 0);
// chain head records per region for a table of cap slots (0: K or LDS leave no room for chains)
uint32_t part_head_cap(const KParams& p, uint64_t cap);

// Build: input is either reference records (recs, R bytes each; start bits -> start_mask) or
// internal words (words, W each). table_empty: skip loading the current region contents.
hipError_t launch_part_insert(const KParams& p, const uint8_t* recs, const uint64_t* words,
                              uint64_t n, TableView t, bool table_empty, const PartBuffers& b,
                              uint64_t* start_mask, uint64_t* split_mask, unsigned long long* ctr,
                              unsigned long long* stats, hipStream_t s, hipEvent_t after_records = nullptr,
                              uint64_t* word_splits = nullptr, uint64_t word_splits_cap = 0,
                              hipEvent_t before_build = nullptr, hipEvent_t after_hot = nullptr);

// Staged build of routed words (sharded insert): launch_part_stage per received chunk (first = the
// first chunk of a build sized for `total` words), then launch_part_finish once. Requires
// region_slots_fit and buffers from ensure_part(total).
hipError_t launch_part_stage(const KParams& p, const uint64_t* words, uint64_t m, uint64_t total, bool first,
                             const PartBuffers& b, unsigned long long* ctr, unsigned long long* stats,
                             hipStream_t s, uint64_t* word_splits = nullptr, uint64_t word_splits_cap = 0,
                             bool sample = false, uint64_t cap = 0);
// The same from reference records (converted into words_tmp, chunk records' start / splitter
// bits into start_mask / split_mask): kh_insert's chunked upload.
hipError_t launch_part_stage_recs(const KParams& p, const uint8_t* recs, uint64_t m, uint64_t total, bool first,
                                  const PartBuffers& b, uint64_t* words_tmp, uint64_t* start_mask,
                                  uint64_t* split_mask, unsigned long long* ctr, unsigned long long* stats,
                                  hipStream_t s, bool sample, uint64_t cap);
// One-pass route of the sharded insert: owner q's words at words + q * win * W (win >= n, < 2^32),
// counts[q] = their number, counts[P] = n; start bits into start_mask (kh_build.hip).
// spl: splitter k-mers routed to each owner are added to spl[owner] (null: not counted)
hipError_t launch_route_win(const KParams& p, const uint8_t* recs, uint64_t n, uint32_t P, uint64_t* words,
                            uint64_t win, uint32_t* cnt, uint64_t* counts, uint64_t* start_mask,
                            unsigned long long* ctr, unsigned long long* stats, hipStream_t s,
                            unsigned long long* spl = nullptr);
hipError_t launch_part_finish(const KParams& p, uint64_t total, TableView t, bool table_empty,
                              const PartBuffers& b, unsigned long long* ctr, unsigned long long* stats,
                              hipStream_t s);

}  // namespace kh
