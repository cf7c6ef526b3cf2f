// kh_capi.cpp — C ABI implementation (include/kmer_hash_amd.h): table lifetime, device buffers,
// HIP streams/events, and the host-side orchestration of the kernels in kh_kernels.hip.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/kmer_hash_amd.h"
#include "kh_codec.hpp"
#include "kh_internal.hpp"
#include "kh_kernels.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define KH_HIP(call)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(KH_ERR_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),     \
                        __FILE__, __LINE__);                                                  \
    } while (0)

// A blocking host wait on the table's stream (a device -> host round trip); counted per table so
// that hosts can report the syncs of a sharded step (kh_host_syncs).
#define KH_SYNC(t)                                          \
    do {                                                    \
        ++(t)->host_syncs;                                  \
        KH_HIP(hipStreamSynchronize((t)->stream));          \
    } while (0)

// Grow-only device buffer.
// device bytes held by every table's buffers in this process, and their high-water mark
// (kh_device_bytes: checks tools/mem_model.py against what the sharded path really allocates)
std::atomic<uint64_t> g_dev_bytes{0}, g_dev_peak{0};

void dev_account(int64_t delta) {
    const uint64_t now = g_dev_bytes.fetch_add((uint64_t)delta) + (uint64_t)delta;
    uint64_t pk = g_dev_peak.load();
    while (now > pk && !g_dev_peak.compare_exchange_weak(pk, now)) {
    }
}

struct DevBuf {
    void* p = nullptr;
    uint64_t bytes = 0;
    int ensure(uint64_t want) {
        if (want <= bytes && p) return KH_OK;
        release();
        if (want == 0) want = 16;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            p = nullptr;
            return fail(KH_ERR_NOMEM, "hipMalloc(%llu) failed: %s", (unsigned long long)want,
                        hipGetErrorString(e));
        }
        bytes = want;
        dev_account((int64_t)want);
        return KH_OK;
    }
    void release() {
        if (p) {
            (void)hipFree(p);
            dev_account(-(int64_t)bytes);
        }
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
};

}  // namespace

void kh_set_error_internal(const char* msg) { g_err = msg ? msg : ""; }

bool kh::debug_flag(const char* name) {
    const char* e = getenv("KH_DEBUG");
    if (!e || !*e) return false;
    const size_t n = strlen(name);
    for (const char* p = e; (p = strstr(p, name)) != nullptr; p += n)
        if ((p == e || p[-1] == ',') && (p[n] == 0 || p[n] == ',')) return true;
    return false;
}

struct kh_table {
    int device = 0;
    kh::KParams kp{};
    uint64_t cap = 0;       // slots
    uint64_t n_kmers = 0;   // k-mers the table was created (or last reserved) for
    double load = 0.5;      // load factor
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;

    DevBuf slots, starts, ctr, stats;
    DevBuf splits, splits_w;                 // splitter k-mers (walk segments) / walk subset
    DevBuf seg_next, seg_key, seg_contig, seg_off, clen, stab, stab_id;  // splitter segments
    DevBuf seg_jump, seg_jsum, seg_anchor, seg_pend;
    DevBuf mask, mask_off, scratch;          // per insert batch
    DevBuf stage;                            // host-API staging of records / keys
    DevBuf stage2, stage3;
    DevBuf contig_len, contig_off, chunk_data, chunk_owner, chunk_seq, text, line_first;
    DevBuf route_hist, route_off, route_scratch, route_own;                       // sharded path
    DevBuf pb_buf1, pb_buf2, pb_cnt, pb_ovf;  // partitioned build
    DevBuf headrec;                           // chain head records (region build -> walker)
    DevBuf hot;                               // remapped-region bitmap (KParams::hot), 2 levels of HOT_WORDS
    DevBuf rbounds;                           // balanced region bounds (KParams::rb), 2^17 + 1 words
    uint32_t hcap = 0;                        // head records per region (0 = no chains)
    bool last_insert_part = false;
    bool staging = false, stage_part = false, stage_fresh = false;  // kh_insert_words_stage_dev build
    uint64_t stage_total = 0, stage_n = 0;
    uint64_t collected_n = 0;  // records passed to kh_route_starts_dev since the last clear
    bool slots_stale = true;   // cleared lazily: a partitioned build of an empty table writes every slot
    DevBuf mw_tmp, mw_dst, mw_stage, mw_nrec, mw_off, mw_misc, mw_store;  // migrating walk
    // splitter segments of the migrating walk (kh_mseg.hip)
    DevBuf ms_len, ms_hi, ms_lo, ms_has, ms_done, ms_jump, ms_acc, ms_stab, ms_stab_id, ms_qsrc, ms_misc;
    bool ms_chunks = false;  // the record scan filled the origin's first chunks (line writer)
    DevBuf mw_cnt, mw_list, mw_carry[2], mw_carry_dst[2];  // fixed-slot rounds
    DevBuf ms_res[6], ms_pend;               // pointer jumping over the gathered predecessor tables
    DevBuf route_spl;                        // splitter k-mers routed to each owner (MAX_RANKS words)
    int mw_cur = 0;                          // carry buffer written by the last round
    bool words_split = true;   // every routed word since the last clear went through splitter collection
    bool ms_on = false;        // the current migrating walk uses splitter segments
    uint64_t ms_ns = 0, ms_nsp = 0, ms_cap2 = 0, ms_nq = 0;
    bool walk_bounded = false; // the last walk's text was sized before it ran (kh_assemble_dev)
    bool split_forced = false; // KH_SPLIT_BITS set: the walk uses every collected splitter
    uint64_t mw_wg = 0;        // walkers of every rank (bound of a round's input / held-back messages)
    uint64_t mw_store_n = 0;   // text records in mw_store (valid when mw_store_known)
    uint64_t mw_store_bound = 0;  // upper bound of the store's records (its device count: mw_misc[2])
    bool mw_seg_off = false;      // kh_mwalk_redo: the next walk runs without splitter segments
    uint64_t mw_soft_next = 0;    // kh_mwalk_short: the next walk's soft step limit (0: none)
    uint64_t mw_soft = 0;         // this walk's
    uint64_t mw_store_min = 0;    // ... with a text store of at least this many records
    bool mw_store_known = true;
    uint32_t mw_P = 0, mw_rank = 0;
    bool mw_live = false, mw_stepped = false;
    bool mw_hot = true;        // the shard has remapped regions (the walk reads the bitmap)
    bool succ_pending = false; // k_rec_succ of the migrating walk still queued on the side stream
    uint64_t rw_n = 0, rw_total = 0;  // migrating walk: local walkers, bound on contig length
    uint64_t starts_cap = 0;                 // start entries the starts buffer holds
    uint64_t splits_cap = 0, splits_w_cap = 0;
    bool split_ok = true;                    // every inserted k-mer was checked for splitters
    bool starts_explicit = false;            // kh_set_starts: walks may overlap (text not bounded)
    bool text_sync = false;                  // the next assemble sizes the text from the scanned total
    uint64_t chunk_cap = 0;

    uint64_t n_inserted = 0;                 // host-side count (what was submitted)
    uint64_t host_syncs = 0;                 // blocking stream waits of this table (KH_SYNC)
    uint64_t last_contigs = 0;               // n_starts seen by the last assemble
    bool assembled = false;

    hipEvent_t ev_ins0 = nullptr, ev_ins1 = nullptr, ev_ins2 = nullptr;
    hipEvent_t ev_walk0 = nullptr, ev_walk1 = nullptr, ev_mat1 = nullptr;
    hipEvent_t ev_b0 = nullptr, ev_b1 = nullptr, ev_wk1 = nullptr;  // build / walk-kernel brackets
    bool build_timed = false;
    // side stream: start / splitter compaction overlapped with the partition passes
    hipStream_t side = nullptr;
    hipEvent_t ev_conv = nullptr, ev_side = nullptr;
    bool ins_timed = false, walk_timed = false, wk_timed = false;  // wk: ev_wk1 recorded by this walk
    // counters copied to pinned host memory on the side stream once the last device insert's start
    // compaction and hot-region mark are final (ev_hot / ev_ctr), so assemble reads them without
    // waiting for the build: ctr_early says the copy belongs to the current table state
    unsigned long long* hctr = nullptr;
    hipEvent_t ev_hot = nullptr, ev_ctr = nullptr;
    bool ctr_early = false;
};

namespace {

int set_device(const kh_table* t) {
    KH_HIP(hipSetDevice(t->device));
    return KH_OK;
}

kh::TableView view(const kh_table* t) { return kh::TableView{t->slots.as<uint64_t>(), t->cap}; }

int ensure_list(kh_table* t, DevBuf& buf, uint64_t& cap, uint64_t need) {
    if (need <= cap) return KH_OK;
    const uint64_t W = (uint64_t)t->kp.W;
    uint64_t newcap = need < 1024 ? 1024 : need;
    if (newcap < 2 * cap) newcap = 2 * cap;  // geometric: many small batches stay O(n) copies
    DevBuf nb;
    int rc = nb.ensure(newcap * W * 8);
    if (rc) return rc;
    if (buf.p && cap)
        KH_HIP(hipMemcpyAsync(nb.p, buf.p, cap * W * 8, hipMemcpyDeviceToDevice, t->stream));
    KH_SYNC(t);
    buf.release();
    buf = nb;
    nb.p = nullptr;
    cap = newcap;
    return KH_OK;
}

int ensure_starts(kh_table* t, uint64_t need) { return ensure_list(t, t->starts, t->starts_cap, need); }

int read_ctr(kh_table* t, int idx, uint64_t* v) {
    unsigned long long x = 0;
    KH_HIP(hipMemcpyAsync(&x, t->ctr.as<unsigned long long>() + idx, sizeof x,
                          hipMemcpyDeviceToHost, t->stream));
    KH_SYNC(t);
    *v = x;
    return KH_OK;
}

// First device-side error of a copy of the stats, as a status code.
static int stats_status(const unsigned long long* st) {
    if (st[kh::ST_FULL]) return fail(KH_ERR_FULL, "table full: %llu probes wrapped", st[kh::ST_FULL]);
    if (st[kh::ST_DUP]) return fail(KH_ERR_DUPLICATE, "%llu duplicate k-mers inserted", st[kh::ST_DUP]);
    if (st[kh::ST_BAD_EXT])
        return fail(KH_ERR_BAD_BASE, "%llu extension bytes outside {A,C,G,T,F}", st[kh::ST_BAD_EXT]);
    if (st[kh::ST_MISSING])
        return fail(KH_ERR_NOT_FOUND, "Error: k-mer not found in hash map (%llu walks)",
                    st[kh::ST_MISSING]);
    if (st[kh::ST_CYCLE]) return fail(KH_ERR_CYCLE, "%llu walks exceeded the table size", st[kh::ST_CYCLE]);
    if (st[kh::ST_SPIN]) return fail(KH_ERR_HIP, "%llu inserts timed out on a slot", st[kh::ST_SPIN]);
    if (st[kh::ST_CHUNK_OVF])
        return fail(KH_ERR_NOMEM, "walker output overflow or overlapping walks (malformed input; kh_assemble redoes "
                                  "such a walk unsegmented)");
    if (st[kh::ST_BAD_BASE])
        return fail(KH_ERR_BAD_BASE, "%llu k-mer lines with a base outside {A,C,G,T}", st[kh::ST_BAD_BASE]);
    return KH_OK;
}

// First device-side error, as a status code.
int check_stats(kh_table* t) {
    unsigned long long st[kh::ST_NUM];
    KH_HIP(hipMemcpyAsync(st, t->stats.p, sizeof st, hipMemcpyDeviceToHost, t->stream));
    KH_SYNC(t);
    return stats_status(st);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Empty the slot array (all-ones) unless that already happened since the last clear.
int clean_slots(kh_table* t) {
    if (!t->slots_stale) return KH_OK;
    KH_HIP(hipMemsetAsync(t->slots.p, 0xff, t->cap * (uint64_t)t->kp.W * 8, t->stream));
    t->slots_stale = false;
    return KH_OK;
}

// The migrating walk resolves record successors on the side stream beside its rounds: the
// table's stream waits for it before anything rewrites the records (end of the walk, clear).
int join_succ(kh_table* t) {
    if (!t->succ_pending) return KH_OK;
    KH_HIP(hipStreamWaitEvent(t->stream, t->ev_conv, 0));
    t->succ_pending = false;
    return KH_OK;
}

// Insert strategy: KH_INSERT=cas (global CAS per key), part (partitioned LDS build), auto
// (default: partitioned when the batch is large and the region slices fit LDS).
bool use_part_build(const kh_table* t, uint64_t n) {
    const char* m = getenv("KH_INSERT");
    const bool usable = kh::part_usable(t->kp, t->cap, n);
    if (m && !strcmp(m, "cas")) return false;
    if (m && !strcmp(m, "part"))
        return kh::region_slots_fit(t->kp, t->cap) && n > 0;
    return usable;
}

int ensure_part(kh_table* t, uint64_t n, kh::PartBuffers& b) {
    const uint64_t W = (uint64_t)t->kp.W;
    int rc;
    if ((rc = t->pb_buf1.ensure(kh::part_buf1_words(t->kp, n) * 8)) || (rc = t->pb_buf2.ensure(kh::part_buf2_words(t->kp, n) * 8)) ||
        (rc = t->pb_cnt.ensure(kh::part_count_words() * 8)) ||
        (rc = t->pb_ovf.ensure(kh::part_overflow_cap(n) * W * 8)))
        return rc;
    b.buf1 = t->pb_buf1.as<uint64_t>();
    b.buf2 = t->pb_buf2.as<uint64_t>();
    b.wcnt = t->pb_cnt.as<uint32_t>();
    b.rcnt = b.wcnt + kh::PART_W1_COUNTERS;
    b.hot_list = b.rcnt + kh::HOT_WORDS * 32;
    b.overflow = t->pb_ovf.as<uint64_t>();
    b.hot = t->hot.as<uint32_t>();
    b.rbt = t->rbounds.as<uint64_t>();
    // chain head records: sized by the table (regions x records per region), kept across builds
    const uint32_t hcap = kh::part_head_cap(t->kp, t->cap);
    if (hcap) {
        // + the per-region record counts the build writes after the records (k_rec_succ reads them)
        const uint64_t recb = (uint64_t)hcap * (1ull << t->kp.rbits) * 16, cntb = (1ull << t->kp.rbits) * 4;
        const void* before = t->headrec.p;
        if ((rc = t->headrec.ensure(recb + cntb))) return rc;
        if (t->headrec.p != before) KH_HIP(hipMemsetAsync((char*)t->headrec.p + recb, 0, cntb, t->stream));
    }
    t->hcap = hcap;
    b.headrec = hcap ? t->headrec.as<uint64_t>() : nullptr;
    b.hcap = hcap;
    return KH_OK;
}

// Balanced region bounds (kh_build.hip k_bounds) above load 0.6, where equal slices overflow
// (at load 0.5 they measured slower: C3 8.84 -> 17.5 ms).
bool balanced_bounds(const kh_table* t) { return t->load > 0.6; }

// CAS-path insert into an empty table: remap the minimizer regions the batch would overfill
// (kh_build.hip launch_hot_prepass); later batches place keys with the same bitmap.
int cas_hot_prepass(kh_table* t, const void* recs, const void* words, uint64_t n, uint64_t total = 0) {
    if (t->n_inserted != 0) return KH_OK;
    if (int rc = t->pb_cnt.ensure(kh::part_count_words() * 8)) return rc;
    uint32_t* rcnt = t->pb_cnt.as<uint32_t>() + kh::PART_W1_COUNTERS;
    KH_HIP(hipMemsetAsync(t->hot.p, 0, 2 * kh::HOT_WORDS * 4, t->stream));
    KH_HIP(kh::launch_hot_prepass(t->kp, (const uint8_t*)recs, (const uint64_t*)words, n, t->cap, rcnt,
                                  t->hot.as<uint32_t>(), rcnt + kh::HOT_WORDS * 32, t->ctr.as<unsigned long long>(),
                                  t->stream, total));
    return KH_OK;
}

// Capacity and splitter density for n_kmers (kh_create, kh_reserve).
void size_table(kh_table* t, uint64_t n_kmers) {
    t->n_kmers = n_kmers;
    // splitter density: ~1 per 2^bits k-mers; enough extra walkers for long-chain inputs (C2, C5)
    // at a few % more walkers on short-contig inputs. KH_SPLIT_BITS overrides (0 = off).
    // Collected at insert: 1 per 2^bits k-mers, bits = clamp(log2(n / 2^20) + 1, 4, 12); the walk
    // then uses a subset sized from the start count (kh_assemble_dev).
    int bits = 1;
    while (bits < 12 && (n_kmers >> (20 + bits)) != 0) ++bits;
    bits = bits < 4 ? 4 : bits;
    t->split_forced = false;
    if (const char* e = getenv("KH_SPLIT_BITS")) {  // tests: dense, sparse or no splitters
        bits = atoi(e);
        t->split_forced = true;
    }
    t->kp.split_bits = bits < 0 ? 0 : (bits > 30 ? 30 : bits);
    const double c = (double)(n_kmers ? n_kmers : 1) / t->load;
    t->cap = (uint64_t)c;
    if ((double)t->cap < c) t->cap++;
    if (t->cap < 2) t->cap = 2;
    kh::set_region_bits(t->kp, t->cap);
}

}  // namespace

static_assert(KH_MSG_WORDS == kh::MSG_WORDS, "message layout");

extern "C" {

int kh_abi_version(void) { return KH_ABI_VERSION; }

int kh_device_bytes(uint64_t* now, uint64_t* peak, int reset_peak) {
    if (now) *now = g_dev_bytes.load();
    if (peak) *peak = g_dev_peak.load();
    if (reset_peak) g_dev_peak.store(g_dev_bytes.load());
    return KH_OK;
}
int kh_packed_size(int k) { return (k >= 1 && k <= KH_K_MAX) ? (k + 3) / 4 : KH_ERR_ARG; }
int kh_record_size(int k) { return (k >= 1 && k <= KH_K_MAX) ? (k + 3) / 4 + 2 : KH_ERR_ARG; }
const char* kh_last_error(void) { return g_err.c_str(); }

int kh_device_count(int* n) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *n = 0;
        return fail(KH_ERR_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *n = c;
    return KH_OK;
}

int kh_create(kh_table** out, int k, uint64_t n_kmers, double load_factor, int device) {
    if (!out) return fail(KH_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (k < 1 || k > KH_K_MAX) return fail(KH_ERR_ARG, "k=%d outside [1,%d]", k, KH_K_MAX);
    if (!(load_factor > 0.0 && load_factor < 1.0))
        return fail(KH_ERR_ARG, "load factor %g outside (0,1)", load_factor);
    kh_table* t = new (std::nothrow) kh_table();
    if (!t) return fail(KH_ERR_NOMEM, "host allocation failed");
    t->device = device;
    t->kp = kh::make_params(k);
    t->load = load_factor;
    if (const char* e = getenv("KH_OWNER")) t->kp.owner_mode = strcmp(e, "hash") == 0 ? 1 : 0;
    size_table(t, n_kmers);
    int rc = KH_OK;
    auto bail = [&](int r) {
        kh_destroy(t);
        return r;
    };
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return bail(fail(KH_ERR_HIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e)));
    if (hipStreamCreateWithFlags(&t->own_stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(KH_ERR_HIP, "hipStreamCreate failed"));
    t->stream = t->own_stream;
    if (hipStreamCreateWithFlags(&t->side, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(KH_ERR_HIP, "hipStreamCreate failed"));
    hipEvent_t* evs[] = {&t->ev_ins0, &t->ev_ins1, &t->ev_ins2, &t->ev_walk0, &t->ev_walk1, &t->ev_mat1,
                         &t->ev_b0, &t->ev_b1, &t->ev_wk1};
    for (auto* ev : evs)
        if (hipEventCreate(ev) != hipSuccess) return bail(fail(KH_ERR_HIP, "hipEventCreate failed"));
    for (auto* ev : {&t->ev_conv, &t->ev_side, &t->ev_hot, &t->ev_ctr})
        if (hipEventCreateWithFlags(ev, hipEventDisableTiming) != hipSuccess)
            return bail(fail(KH_ERR_HIP, "hipEventCreate failed"));
    if (hipHostMalloc((void**)&t->hctr, kh::CT_NUM * 8, hipHostMallocDefault) != hipSuccess)
        return bail(fail(KH_ERR_NOMEM, "pinned host counters"));
    if ((rc = t->slots.ensure(t->cap * (uint64_t)t->kp.W * 8))) return bail(rc);
    if ((rc = t->hot.ensure(2 * kh::HOT_WORDS * 4))) return bail(rc);
    if (hipMemset(t->hot.p, 0, 2 * kh::HOT_WORDS * 4) != hipSuccess) return bail(fail(KH_ERR_HIP, "hipMemset failed"));
    t->kp.hot = t->hot.as<uint32_t>();
    // region slot ranges: equal until a balanced table's first build (lookups read them only when
    // balanced; the build always does)
    if ((rc = t->rbounds.ensure((kh::HOT_WORDS * 32 + 1) * 8))) return bail(rc);
    if (balanced_bounds(t)) t->kp.rb = t->rbounds.as<uint64_t>();
    kh::launch_bounds(t->kp, t->cap, nullptr, 0, t->rbounds.as<uint64_t>(), t->stream);
    if ((rc = t->ctr.ensure(kh::CT_NUM * 8))) return bail(rc);
    if ((rc = t->route_spl.ensure(kh::MAX_RANKS * 8))) return bail(rc);
    if ((rc = t->stats.ensure(kh::ST_NUM * 8))) return bail(rc);
    if ((rc = kh_clear(t))) return bail(rc);
    if (hipStreamSynchronize(t->stream) != hipSuccess) return bail(fail(KH_ERR_HIP, "sync failed"));
    *out = t;
    return KH_OK;
}

int kh_destroy(kh_table* t) {
    if (!t) return KH_OK;
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    DevBuf* bufs[] = {&t->slots, &t->starts, &t->ctr, &t->stats, &t->mask, &t->mask_off,
                      &t->scratch, &t->stage, &t->stage2, &t->stage3, &t->contig_len,
                      &t->contig_off, &t->chunk_data, &t->chunk_owner, &t->chunk_seq, &t->text, &t->line_first,
                      &t->route_hist, &t->route_off, &t->route_scratch, &t->route_own, &t->splits, &t->splits_w, &t->seg_next,
                      &t->seg_key, &t->seg_contig, &t->seg_off, &t->clen, &t->stab, &t->stab_id,
                      &t->seg_jump, &t->seg_jsum, &t->seg_anchor, &t->seg_pend,
                      &t->mw_tmp, &t->mw_dst, &t->mw_stage, &t->mw_nrec, &t->mw_off,
                      &t->mw_misc, &t->mw_store, &t->ms_len, &t->ms_hi, &t->ms_lo, &t->ms_has, &t->ms_done,
                      &t->ms_jump, &t->ms_acc, &t->ms_stab, &t->ms_stab_id, &t->ms_qsrc, &t->ms_misc,
                      &t->mw_cnt, &t->mw_list, &t->mw_carry[0], &t->mw_carry[1], &t->mw_carry_dst[0],
                      &t->mw_carry_dst[1], &t->ms_res[0], &t->ms_res[1], &t->ms_res[2], &t->ms_res[3], &t->ms_res[4],
                      &t->ms_res[5], &t->ms_pend, &t->route_spl,
                      &t->pb_buf1, &t->pb_buf2, &t->pb_cnt, &t->pb_ovf, &t->headrec, &t->hot, &t->rbounds};
    if (t->side) (void)hipStreamSynchronize(t->side);  // k_rec_succ may still read the table
    for (auto* b : bufs) b->release();
    hipEvent_t evs[] = {t->ev_ins0, t->ev_ins1, t->ev_ins2, t->ev_walk0, t->ev_walk1, t->ev_mat1, t->ev_b0,
                        t->ev_b1, t->ev_wk1, t->ev_conv,
                        t->ev_side, t->ev_hot, t->ev_ctr};
    for (auto ev : evs)
        if (ev) (void)hipEventDestroy(ev);
    if (t->hctr) (void)hipHostFree(t->hctr);
    if (t->side) (void)hipStreamDestroy(t->side);
    if (t->own_stream) (void)hipStreamDestroy(t->own_stream);
    delete t;
    // teardown errors are not the caller's: leave the thread's HIP last-error clear, or the
    // caller's next launch check (torch's, say) reports it as its own
    (void)hipGetLastError();
    return KH_OK;
}

int kh_reserve(kh_table* t, uint64_t n_kmers) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (n_kmers <= t->n_kmers) return KH_OK;
    if (t->n_inserted || t->staging)
        return fail(KH_ERR_STATE, "kh_reserve on a table holding %llu k-mers (clear it first)",
                    (unsigned long long)t->n_inserted);
    if (int rc = set_device(t)) return rc;
    KH_SYNC(t);
    const uint64_t old_n = t->n_kmers;
    const int old_bits = t->kp.split_bits;
    size_table(t, n_kmers);
    // the splitter density stays the one the table was created with: every shard of a sharded
    // table must use the same (a walker stops before splitters that their owner seeds walkers at)
    t->kp.split_bits = old_bits;
    // the new slot array first: when it cannot be had, the table keeps its old one and old size
    DevBuf ns;
    if (int rc = ns.ensure(t->cap * (uint64_t)t->kp.W * 8)) {
        size_table(t, old_n);
        t->kp.split_bits = old_bits;
        return rc;
    }
    t->slots.release();
    t->slots = ns;
    ns.p = nullptr;
    t->slots_stale = true;
    kh::launch_bounds(t->kp, t->cap, nullptr, 0, t->rbounds.as<uint64_t>(), t->stream);
    KH_HIP(hipGetLastError());
    return KH_OK;
}

int kh_clear(kh_table* t) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (int rc = set_device(t)) return rc;
    if (int rc = join_succ(t)) return rc;
    t->slots_stale = true;
    kh::FillSet f;
    f.add(t->ctr.p, kh::CT_NUM * 8, 0);
    f.add(t->stats.p, kh::ST_NUM * 8, 0);
    f.add(t->hot.p, 2 * kh::HOT_WORDS * 4, 0);  // placement by minimizer again
    f.add(t->route_spl.p, kh::MAX_RANKS * 8, 0);
    KH_HIP(kh::launch_fill(f, t->stream));
    t->n_inserted = 0;
    t->assembled = false;
    t->split_ok = true;
    t->starts_explicit = false;
    t->staging = false;
    t->stage_n = 0;
    t->collected_n = 0;
    t->words_split = true;
    return KH_OK;
}

int kh_set_stream(kh_table* t, void* s) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->stream = s ? (hipStream_t)s : t->own_stream;
    return KH_OK;
}

int kh_sync(kh_table* t) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    if (int rc = set_device(t)) return rc;
    return check_stats(t);  // one wait: the stats read is ordered after the queued work
}

uint64_t kh_capacity(const kh_table* t) { return t ? t->cap : 0; }

int kh_host_syncs(const kh_table* t, uint64_t* n) {
    if (!t || !n) return fail(KH_ERR_ARG, "null argument");
    *n = t->host_syncs;
    return KH_OK;
}

int kh_insert_dev(kh_table* t, const void* dev_recs, uint64_t n) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    if (n == 0) return KH_OK;
    if (!dev_recs) return fail(KH_ERR_ARG, "null records");
    if (!aligned16(dev_recs)) return fail(KH_ERR_ARG, "device records must be 16-byte aligned");
    if (t->n_inserted + n > t->n_kmers)
        return fail(KH_ERR_FULL, "inserting %llu k-mers into a table created for %llu (%llu in)",
                    (unsigned long long)n, (unsigned long long)t->n_kmers,
                    (unsigned long long)t->n_inserted);
    if (int rc = set_device(t)) return rc;
    if (int rc = join_succ(t)) return rc;
    int rc;
    const uint64_t nw = (n + 63) / 64;
    const bool split = t->kp.split_bits > 0;
    if ((rc = t->mask.ensure(nw * 8 * (split ? 2 : 1)))) return rc;
    if ((rc = t->mask_off.ensure(nw * 8))) return rc;
    if ((rc = t->scratch.ensure(kh::scan_scratch_words(nw > n ? nw : n) * 8 + 64))) return rc;
    if ((rc = ensure_starts(t, t->n_inserted + n))) return rc;
    if (split && (rc = ensure_list(t, t->splits, t->splits_cap, t->n_inserted + n))) return rc;
    uint64_t* split_mask = split ? t->mask.as<uint64_t>() + nw : nullptr;
    const bool part = use_part_build(t, n);
    kh::PartBuffers pb{};
    if (part && (rc = ensure_part(t, n, pb))) return rc;
    // a partitioned build into a fresh table rewrites every slot: no clear needed
    const bool fresh = part && t->n_inserted == 0;  // empty (stale or clean): the build writes every slot
    if (!fresh && (rc = clean_slots(t))) return rc;
    t->slots_stale = false;
    KH_HIP(hipEventRecord(t->ev_ins0, t->stream));
    // partitioned build: the start / splitter bits exist once the record pass has run, so their
    // compaction runs on the side stream, overlapped with the partition passes and the build
    const bool overlap = part;
    hipStream_t cs = overlap ? t->side : t->stream;
    t->build_timed = part;
    if (part) {
        KH_HIP(kh::launch_part_insert(t->kp, (const uint8_t*)dev_recs, nullptr, n, view(t),
                                      fresh, pb, t->mask.as<uint64_t>(), split_mask,
                                      t->ctr.as<unsigned long long>(),
                                      t->stats.as<unsigned long long>(), t->stream,
                                      overlap ? t->ev_conv : nullptr, nullptr, 0, t->ev_b0,
                                      overlap ? t->ev_hot : nullptr));
        KH_HIP(hipEventRecord(t->ev_b1, t->stream));
    } else {
        if ((rc = cas_hot_prepass(t, dev_recs, nullptr, n))) return rc;
        KH_HIP(kh::launch_insert(t->kp, (const uint8_t*)dev_recs, n, view(t), t->mask.as<uint64_t>(),
                                 split_mask, t->stats.as<unsigned long long>(), t->stream));
    }
    t->last_insert_part = part;
    if (overlap) KH_HIP(hipStreamWaitEvent(t->side, t->ev_conv, 0));
    KH_HIP(kh::launch_collect_starts(t->kp, (const uint8_t*)dev_recs, n, t->mask.as<uint64_t>(),
                                     t->mask_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                     t->starts.as<uint64_t>(), t->ctr.as<unsigned long long>(), cs));
    if (split)
        KH_HIP(kh::launch_collect_starts(t->kp, (const uint8_t*)dev_recs, n, split_mask,
                                         t->mask_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                         t->splits.as<uint64_t>(), t->ctr.as<unsigned long long>(), cs,
                                         kh::CT_N_SPLIT));
    KH_HIP(hipEventRecord(t->ev_ins1, t->stream));
    t->ctr_early = false;
    if (overlap) {
        KH_HIP(hipEventRecord(t->ev_side, t->side));
        KH_HIP(hipStreamWaitEvent(t->stream, t->ev_side, 0));
        // start / splitter counts (final after the compaction above) and the remapped-region count
        // (final after the hot mark, ev_hot) to pinned memory beside the build
        KH_HIP(hipStreamWaitEvent(t->side, t->ev_hot, 0));
        KH_HIP(hipMemcpyAsync(t->hctr, t->ctr.p, kh::CT_NUM * 8, hipMemcpyDeviceToHost, t->side));
        KH_HIP(hipEventRecord(t->ev_ctr, t->side));
        t->ctr_early = true;
    }
    KH_HIP(hipEventRecord(t->ev_ins2, t->stream));
    t->ins_timed = true;
    t->n_inserted += n;
    t->assembled = false;
    return KH_OK;
}

// kh_insert of a large batch into an empty table (the reference's boundary: records in host
// memory, kmer_hash.cpp:129): the records go up in chunks on the side stream while the table's
// stream converts and partitions each chunk that has landed (passes 1-2 into the region windows);
// one build after the last chunk. The upload is the bound (~55 GB/s over PCIe for 3 GB at C3);
// all device work but the last chunk's passes, the build and the walk hides behind it.
static int insert_chunked_upload(kh_table* t, const uint8_t* host_recs, uint64_t n) {
    const uint64_t R = (uint64_t)t->kp.R, W = (uint64_t)t->kp.W;
    // chunks of a multiple of 8192 records (the convert pass's tiles; start-mask words stay whole)
    uint64_t nch = 16;
    uint64_t chunk = ((n + nch - 1) / nch + 8191) & ~8191ull;
    nch = (n + chunk - 1) / chunk;
    int rc;
    if ((rc = t->stage.ensure(n * R + 16))) return rc;
    if ((rc = t->stage2.ensure(chunk * W * 8 + 16))) return rc;
    const uint64_t nw = (n + 63) / 64;
    const bool split = t->kp.split_bits > 0;
    if ((rc = t->mask.ensure(nw * 8 * (split ? 2 : 1)))) return rc;
    if ((rc = t->mask_off.ensure(nw * 8))) return rc;
    if ((rc = t->scratch.ensure(kh::scan_scratch_words(nw > n ? nw : n) * 8 + 64))) return rc;
    if ((rc = ensure_starts(t, n))) return rc;
    if (split && (rc = ensure_list(t, t->splits, t->splits_cap, n))) return rc;
    uint64_t* start_mask = t->mask.as<uint64_t>();
    uint64_t* split_mask = split ? start_mask + nw : nullptr;
    kh::PartBuffers pb{};
    if ((rc = ensure_part(t, n, pb))) return rc;
    struct Events {  // one per chunk: its upload landed
        std::vector<hipEvent_t> e;
        ~Events() {
            for (auto x : e)
                if (x) (void)hipEventDestroy(x);
        }
    } ev;
    ev.e.assign(nch, nullptr);
    for (auto& e : ev.e) KH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    uint8_t* d = t->stage.as<uint8_t>();
    unsigned long long* ctr = t->ctr.as<unsigned long long>();
    unsigned long long* stats = t->stats.as<unsigned long long>();
    auto upload = [&](uint64_t c) -> hipError_t {
        const uint64_t b = c * chunk, m = (b + chunk < n ? chunk : n - b);
        hipError_t e = hipMemcpyAsync(d + b * R, host_recs + b * R, m * R, hipMemcpyHostToDevice, t->side);
        return e != hipSuccess ? e : hipEventRecord(ev.e[c], t->side);
    };
    // the side stream starts after everything already queued on the table's stream; chunk c + 1's
    // upload is queued after chunk c's passes, so a pageable (host-synchronous) copy overlaps too
    KH_HIP(hipEventRecord(t->ev_side, t->stream));
    KH_HIP(hipStreamWaitEvent(t->side, t->ev_side, 0));
    KH_HIP(upload(0));
    KH_HIP(hipEventRecord(t->ev_ins0, t->stream));
    t->slots_stale = false;  // the build of an empty table writes every slot
    for (uint64_t c = 0; c < nch; ++c) {
        const uint64_t b = c * chunk, m = (b + chunk < n ? chunk : n - b);
        KH_HIP(hipStreamWaitEvent(t->stream, ev.e[c], 0));
        KH_HIP(kh::launch_part_stage_recs(t->kp, d + b * R, m, n, c == 0, pb, t->stage2.as<uint64_t>(),
                                          start_mask + b / 64, split ? split_mask + b / 64 : nullptr, ctr, stats,
                                          t->stream, c == 0, t->cap));
        KH_HIP(kh::launch_collect_starts(t->kp, d + b * R, m, start_mask + b / 64, t->mask_off.as<uint64_t>(),
                                         t->scratch.as<uint64_t>(), t->starts.as<uint64_t>(), ctr, t->stream));
        if (split)
            KH_HIP(kh::launch_collect_starts(t->kp, d + b * R, m, split_mask + b / 64, t->mask_off.as<uint64_t>(),
                                             t->scratch.as<uint64_t>(), t->splits.as<uint64_t>(), ctr, t->stream,
                                             kh::CT_N_SPLIT));
        if (c + 1 < nch) KH_HIP(upload(c + 1));
    }
    KH_HIP(hipEventRecord(t->ev_b0, t->stream));
    KH_HIP(kh::launch_part_finish(t->kp, n, view(t), true, pb, ctr, stats, t->stream));
    KH_HIP(hipEventRecord(t->ev_b1, t->stream));
    KH_HIP(hipEventRecord(t->ev_ins1, t->stream));
    KH_HIP(hipEventRecord(t->ev_ins2, t->stream));
    t->build_timed = t->ins_timed = true;
    t->last_insert_part = true;
    t->n_inserted += n;
    t->assembled = false;
    return check_stats(t);  // one wait: the stats read is ordered after the queued work
}

int kh_insert(kh_table* t, const uint8_t* host_recs, uint64_t n) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (n == 0) return KH_OK;
    if (!host_recs) return fail(KH_ERR_ARG, "null records");
    if (int rc = set_device(t)) return rc;
    if (t->n_inserted + n > t->n_kmers)
        return fail(KH_ERR_FULL, "inserting %llu k-mers into a table created for %llu (%llu in)",
                    (unsigned long long)n, (unsigned long long)t->n_kmers, (unsigned long long)t->n_inserted);
    if (t->n_inserted == 0 && n >= (1ull << 24) && use_part_build(t, n))
        return insert_chunked_upload(t, host_recs, n);
    const uint64_t bytes = n * (uint64_t)t->kp.R;
    if (int rc = t->stage.ensure(bytes)) return rc;
    KH_HIP(hipMemcpyAsync(t->stage.p, host_recs, bytes, hipMemcpyHostToDevice, t->stream));
    if (int rc = kh_insert_dev(t, t->stage.p, n)) return rc;
    return check_stats(t);  // one wait: the stats read is ordered after the queued work
}

int kh_find_dev(kh_table* t, const void* dev_keys, uint64_t n, void* dev_out, void* dev_found) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    if (n == 0) return KH_OK;
    if (!dev_keys || !dev_out || !dev_found) return fail(KH_ERR_ARG, "null buffer");
    if (int rc = set_device(t)) return rc;
    if (int rc = clean_slots(t)) return rc;
    KH_HIP(kh::launch_find(t->kp, (const uint8_t*)dev_keys, n, view(t), (uint8_t*)dev_out,
                           (uint8_t*)dev_found, t->stream));
    return KH_OK;
}

int kh_find(kh_table* t, const uint8_t* keys, uint64_t n, uint8_t* out, uint8_t* found) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    if (n == 0) return KH_OK;
    if (!keys || !out || !found) return fail(KH_ERR_ARG, "null buffer");
    if (int rc = set_device(t)) return rc;
    const uint64_t kb = n * (uint64_t)t->kp.P, rb = n * (uint64_t)t->kp.R;
    int rc;
    if ((rc = t->stage.ensure(kb))) return rc;
    if ((rc = t->stage2.ensure(rb))) return rc;
    if ((rc = t->stage3.ensure(n))) return rc;
    KH_HIP(hipMemcpyAsync(t->stage.p, keys, kb, hipMemcpyHostToDevice, t->stream));
    if ((rc = kh_find_dev(t, t->stage.p, n, t->stage2.p, t->stage3.p))) return rc;
    KH_HIP(hipMemcpyAsync(out, t->stage2.p, rb, hipMemcpyDeviceToHost, t->stream));
    KH_HIP(hipMemcpyAsync(found, t->stage3.p, n, hipMemcpyDeviceToHost, t->stream));
    KH_SYNC(t);
    return KH_OK;
}

int kh_set_starts(kh_table* t, const uint8_t* recs, uint64_t n) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (n && !recs) return fail(KH_ERR_ARG, "null records");
    if (int rc = set_device(t)) return rc;
    int rc;
    if ((rc = ensure_starts(t, n))) return rc;
    const uint64_t bytes = n * (uint64_t)t->kp.R;
    if ((rc = t->stage.ensure(bytes))) return rc;
    if (n) KH_HIP(hipMemcpyAsync(t->stage.p, recs, bytes, hipMemcpyHostToDevice, t->stream));
    KH_HIP(kh::launch_load_starts(t->kp, t->stage.as<uint8_t>(), n, t->starts.as<uint64_t>(),
                                  t->ctr.as<unsigned long long>(), t->stream));
    KH_SYNC(t);
    t->assembled = false;
    t->split_ok = false;  // caller's starts may share segments (e.g. two starts on one contig)
    t->starts_explicit = true;
    return KH_OK;
}

int kh_assemble_dev(kh_table* t) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    if (int rc = set_device(t)) return rc;
    if (int rc = join_succ(t)) return rc;
    if (int rc = clean_slots(t)) return rc;
    int rc;
    // The start count decides buffer sizes and the grid (the reference also knows
    // start_nodes.size() on the host before walking, kmer_hash.cpp:41).
    unsigned long long cv[kh::CT_NUM];
    if (t->ctr_early) {  // copied beside the build (kh_insert_dev): wait for the copy, not the build
        ++t->host_syncs;
        KH_HIP(hipEventSynchronize(t->ev_ctr));
        memcpy(cv, t->hctr, sizeof cv);
        t->ctr_early = false;
    } else {
        KH_HIP(hipMemcpyAsync(cv, t->ctr.p, sizeof cv, hipMemcpyDeviceToHost, t->stream));
        KH_SYNC(t);
    }
    const uint64_t ns = cv[kh::CT_N_STARTS];
    uint64_t nsp = 0;
    const unsigned long long* nsp_dev = nullptr;
    kh::KParams kp = t->kp;
    if (!cv[kh::CT_HOT]) kp.hot = nullptr;  // no remapped region: the walker skips the bitmap load
    // splitter segments only where walks are known disjoint (table-collected starts): a segment
    // is written once, so walks that overlap (explicit starts, malformed input) walk unsegmented
    const bool disjoint = !t->starts_explicit && !t->text_sync;
    if (kp.split_bits && t->split_ok && disjoint)
        nsp = cv[kh::CT_N_SPLIT];
    else
        kp.split_bits = 0;
    // Walk density: enough segments for ~1M walkers in all (few, long contigs: C2, C5) but at
    // least 1 splitter per 256 k-mers, so that no single chain dominates the critical path (the
    // longest segment bounds the walk: C5 with 10^6-k-mer chains took 64 ms at 1 per 4096, with
    // geometric segment lengths up to ~10x their mean; C3 pays +0.2 ms for the extra segments).
    const uint64_t* splits = t->splits.as<uint64_t>();
    if (kp.split_bits && !t->split_forced) {
        // (round 5, C2: a 2^18-walker target 1.25 -> 1.39 ms/step, 2^19 and 2^21 unchanged)
        const uint64_t want = ns < (1ull << 20) ? (1ull << 20) - ns : 0;
        const uint64_t floor_cnt = t->n_inserted >> 8;
        const uint64_t d = want > floor_cnt ? want : floor_cnt;
        int bw = kp.split_bits;
        while (bw < 12 && d && (t->n_inserted >> (bw + 1)) >= d) ++bw;
        if (bw > kp.split_bits && nsp) {
            if ((rc = ensure_list(t, t->splits_w, t->splits_w_cap, nsp))) return rc;
            if ((rc = t->scratch.ensure(kh::scan_scratch_words(nsp) * 8 + 64)) ||
                (rc = t->mask_off.ensure((nsp + 1) * 8)))
                return rc;
            KH_HIP(kh::launch_filter_splits(kp, splits, nsp, bw, t->mask_off.as<uint64_t>(),
                                            t->scratch.as<uint64_t>(), t->splits_w.as<uint64_t>(),
                                            t->ctr.as<unsigned long long>() + kh::CT_N_SPLIT_W, t->stream));
            // nsp stays the bound for sizes; kernels read the exact count (no host round trip)
            nsp_dev = t->ctr.as<unsigned long long>() + kh::CT_N_SPLIT_W;
            splits = t->splits_w.as<uint64_t>();
        }
        kp.split_bits = bw;
    }
    const uint64_t nseg = ns + nsp;
    const uint64_t n = t->n_inserted > ns ? t->n_inserted : ns;
    const uint64_t chunk_cap = n / kh::CHUNK_BASES + nseg + 64;
    if ((rc = t->contig_len.ensure((nseg + 1) * 4))) return rc;
    if ((rc = t->contig_off.ensure((ns + 1) * 8))) return rc;
    if ((rc = t->chunk_data.ensure(chunk_cap * kh::CHUNK_WORDS * 8))) return rc;
    if ((rc = t->chunk_owner.ensure(chunk_cap * 4))) return rc;
    if ((rc = t->chunk_seq.ensure(chunk_cap * 4))) return rc;
    if ((rc = t->scratch.ensure(kh::scan_scratch_words(ns) * 8 + 64))) return rc;
    t->chunk_cap = chunk_cap;
    kh::WalkBuffers wb{};
    wb.starts = t->starts.as<uint64_t>();
    wb.n_starts = ns;
    wb.contig_len = t->contig_len.as<uint32_t>();
    wb.chunk_data = t->chunk_data.as<uint64_t>();
    wb.chunk_owner = t->chunk_owner.as<uint32_t>();
    wb.chunk_seq = t->chunk_seq.as<uint32_t>();
    wb.chunk_cap = chunk_cap;
    wb.max_steps = n;
    // (32 queue batches per atomic for short contigs measured slower at C5 in round 6: walk kernel
    // 2.745 -> 2.87 ms; round 5's 3.27 -> 2.99 predates the single place() site)
    wb.batches = 0;
    wb.headrec = t->headrec.as<uint64_t>();
    wb.hcap = t->headrec.p ? t->hcap : 0u;
    kh::SegBuffers sb{};
    if (kp.split_bits) {
        // walkers may stop before a splitter k-mer even when none was collected (then the link
        // step reports it missing), so the segment arrays exist whenever splitting is on
        const uint64_t cap2 = 2 * nsp + 64;
        if ((rc = t->seg_next.ensure((nseg + 4) * 4)) || (rc = t->seg_key.ensure((nseg + 1) * 16)) ||
            (rc = t->seg_contig.ensure((nseg + 1) * 4)) || (rc = t->seg_off.ensure((nseg + 1) * 4)) ||
            (rc = t->clen.ensure((ns + 1) * 4)) || (rc = t->stab.ensure(cap2 * 16)) ||
            (rc = t->stab_id.ensure(cap2 * 4)) || (rc = t->seg_jump.ensure((nseg + 1) * 4)) ||
            (rc = t->seg_jsum.ensure((nseg + 1) * 4)) || (rc = t->seg_anchor.ensure(nseg + 1)) ||
            (rc = t->seg_pend.ensure((ns + 6) * 4)))
            return rc;
        wb.splits = splits;
        wb.n_splits = nsp;
        wb.n_splits_dev = nsp_dev;
        wb.seg_next = t->seg_next.as<uint32_t>();
        wb.seg_key = t->seg_key.as<uint64_t>();
        sb.stab = t->stab.as<uint64_t>();
        sb.stab_id = t->stab_id.as<uint32_t>();
        sb.cap2 = cap2;
        sb.seg_contig = t->seg_contig.as<uint32_t>();
        sb.seg_off = t->seg_off.as<uint32_t>();
        sb.clen = t->clen.as<uint32_t>();
        sb.jump = t->seg_jump.as<uint32_t>();
        sb.jsum = t->seg_jsum.as<uint32_t>();
        sb.anchor = t->seg_anchor.as<uint8_t>();
        sb.pend = t->seg_pend.as<uint32_t>();
        sb.long_flag = sb.pend + ns + 1;
        // deferred splitter segments (k_walk_q): a contig's walker stops at a splitter only past
        // the walk density's spacing, so contigs shorter than it (C3: all) need no splitter segment
        // and the splitter walkers are skipped; KH_DEBUG=seg_eager stops at every splitter
        // (not where the mean contig is longer than the splitter spacing, C2: most walkers stop
        // anyway and phase 1 would only run after the start walkers instead of beside them)
        wb.seg_long = sb.pend + ns + 2;  // [0] a contig's walker stopped at a splitter, [1] splitter walkers deferred
        const bool short_mean = ns && n / ns <= (1ull << kp.split_bits);
        wb.split_min = (kh::debug_flag("seg_eager") || !short_mean) ? 0u : (1u << kp.split_bits);
    }
    unsigned long long* ctr = t->ctr.as<unsigned long long>();
    unsigned long long* stats = t->stats.as<unsigned long long>();
    // Walks from the table's own start k-mers are disjoint: the text is at most K + 1 bytes per
    // contig plus one per k-mer, and the chunk pool holds them, so the text is sized before the
    // walk and nothing is read back between walk and text (one host round trip less per assemble;
    // a total past the bound, only possible on malformed input, is not written and kh_assemble
    // redoes the walk the slow way). Otherwise (explicit starts: walks that overlap, e.g. two
    // starts on one contig, make the text longer than the k-mer count) the text is sized from the
    // scanned total, and if overlapping walks exhaust the chunk pool the walk is redone once with
    // the pool the first attempt asked for.
    const bool bounded = !t->starts_explicit && !t->text_sync;
    t->text_sync = false;
    t->walk_bounded = bounded;
    if (bounded) {
        if ((rc = t->text.ensure(ns * (uint64_t)(t->kp.K + 1) + n + 64))) return rc;
        wb.text_cap = t->text.bytes;
    }
    for (int attempt = 0;; ++attempt) {
        {
            kh::FillSet f;
            f.add(ctr + kh::CT_WALK_NEXT, 8 * 3, 0);  // WALK, CHUNK, OUT
            if (kp.split_bits) f.add(wb.seg_next, nseg * 4, 0xff);
            if (wb.split_min) {
                f.add(wb.seg_long, 16, 0);
                f.add(wb.contig_len + ns, nsp * 4, 0);  // phase 1: not walked yet
            }
            KH_HIP(kh::launch_fill(f, t->stream));
        }
        KH_HIP(hipEventRecord(t->ev_walk0, t->stream));
        // Successor runs of the head records (k_rec_succ). A record read before its successor is
        // resolved still says 0 (the walker probes, as without), so the resolve runs on the side
        // stream beside the walk (request-bound beside a latency-bound walker); the table stream
        // waits for it after the walk (the next build rewrites the records).
        bool succ_side = false;
        if (attempt == 0 && wb.hcap && kh::rec_succ_fits(kp, wb.hcap)) {
            // beside the walk where a torn read is harmless (rec_succ_side: k > 40 at 16-B slots),
            // else before it on the table stream; beside the walk 1024 blocks (C3 walk + resolve
            // 1.28 ms; the full 8192-block grid 1.32-1.34, 256 blocks 1.85: the resolve then lags
            // the walkers; no resolve 1.46)
            const bool conc = kh::rec_succ_side(kp);
            const unsigned blocks = conc ? 1024u : 0u;
            hipStream_t rs = t->stream;
            if (conc && t->side) {
                KH_HIP(hipEventRecord(t->ev_side, t->stream));
                KH_HIP(hipStreamWaitEvent(t->side, t->ev_side, 0));
                rs = t->side;
                succ_side = true;
            }
            KH_HIP(kh::launch_rec_succ(kp, view(t), t->headrec.as<uint64_t>(), wb.hcap, rs, blocks));
        }
        // the splitter table reads only the splitter list: behind the resolve, beside the walk
        // (walk bracket C3 1.35 -> 1.33, C2 0.61 -> 0.59, C5 3.46 -> 3.43 ms;
        // profiles/r05/ab/ab_seg_table_beside_walk.txt)
        if (kp.split_bits) KH_HIP(kh::launch_seg_table(kp, wb, sb, succ_side ? t->side : t->stream));
        if (succ_side) KH_HIP(hipEventRecord(t->ev_conv, t->side));
        // three walker blocks per CU for 16-B slots at load <= 0.6, else two (kh_kernels.hip)
        // (round 5, after the single place() site: 4 / 5 blocks per CU C3 walk 1.40 / 1.43 ms vs 1.16)
        const int wgrid = (kp.W == 2 && t->load <= 0.6) ? -3 : -2;
        KH_HIP(kh::launch_walk(kp, view(t), wb, ctr, stats, wgrid, t->stream));
        if (wb.split_min && wb.n_splits) {  // the splitter walkers, if some contig was long
            kh::WalkBuffers wb1 = wb;
            wb1.phase = 1;
            KH_HIP(hipMemsetAsync(ctr + kh::CT_WALK_NEXT, 0, 8, t->stream));
            KH_HIP(kh::launch_walk(kp, view(t), wb1, ctr, stats, wgrid, t->stream));
        }
        if (succ_side) KH_HIP(hipStreamWaitEvent(t->stream, t->ev_conv, 0));
        // the splitter table, if the walk found it needed and it was not built beside the walk
        if (kp.split_bits && wb.split_min) KH_HIP(kh::launch_seg_table(kp, wb, sb, t->stream, true));
        KH_HIP(hipEventRecord(t->ev_wk1, t->stream));
        t->wk_timed = true;
        if (kp.split_bits) KH_HIP(kh::launch_segments(kp, wb, sb, stats, t->stream));
        KH_HIP(hipEventRecord(t->ev_walk1, t->stream));
        if (kp.split_bits)
            KH_HIP(kh::launch_materialize_seg(kp, wb, sb, t->contig_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                              nullptr, ctr, t->stream, kh::MAT_SCAN));
        else
            KH_HIP(kh::launch_materialize(kp, wb, t->contig_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                          nullptr, ctr, t->stream, kh::MAT_SCAN));
        if (bounded) break;
        unsigned long long hv[2], ovf = 0;
        KH_HIP(hipMemcpyAsync(hv, ctr + kh::CT_CHUNK_NEXT, sizeof hv, hipMemcpyDeviceToHost, t->stream));
        KH_HIP(hipMemcpyAsync(&ovf, stats + kh::ST_CHUNK_OVF, 8, hipMemcpyDeviceToHost, t->stream));
        KH_SYNC(t);
        if (ns == 0) hv[1] = 0;
        if (ovf && attempt == 0) {
            const uint64_t need = nseg + hv[0] + 64;
            if ((rc = t->chunk_data.ensure(need * kh::CHUNK_WORDS * 8)) || (rc = t->chunk_owner.ensure(need * 4)) ||
                (rc = t->chunk_seq.ensure(need * 4)))
                return rc;
            t->chunk_cap = wb.chunk_cap = need;
            wb.chunk_data = t->chunk_data.as<uint64_t>();
            wb.chunk_owner = t->chunk_owner.as<uint32_t>();
            wb.chunk_seq = t->chunk_seq.as<uint32_t>();
            KH_HIP(hipMemsetAsync(stats + kh::ST_CHUNK_OVF, 0, 8, t->stream));
            continue;  // (seg_next is reset at the top of the attempt)
        }
        if ((rc = t->text.ensure(hv[1] + 64))) return rc;
        break;
    }
    if ((rc = t->line_first.ensure(kh::line_first_words(t->text.bytes) * 4))) return rc;
    uint32_t* lf = t->line_first.as<uint32_t>();
    if (kp.split_bits)
        KH_HIP(kh::launch_materialize_seg(kp, wb, sb, t->contig_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                          t->text.as<char>(), ctr, t->stream, kh::MAT_WRITE, lf, t->text.bytes));
    else
        KH_HIP(kh::launch_materialize(kp, wb, t->contig_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                      t->text.as<char>(), ctr, t->stream, kh::MAT_WRITE, lf, t->text.bytes));
    KH_HIP(hipEventRecord(t->ev_mat1, t->stream));
    t->walk_timed = true;
    t->last_contigs = ns;
    t->assembled = true;
    return KH_OK;
}

int kh_assemble(kh_table* t, uint64_t* n_contigs, uint64_t* out_bytes) {
    if (int rc = kh_assemble_dev(t)) return rc;
    // the stats and the text's byte count in one wait (ordered after the queued work)
    unsigned long long st[kh::ST_NUM], ob = 0;
    KH_HIP(hipMemcpyAsync(st, t->stats.p, sizeof st, hipMemcpyDeviceToHost, t->stream));
    KH_HIP(hipMemcpyAsync(&ob, t->ctr.as<unsigned long long>() + kh::CT_OUT_BYTES, 8, hipMemcpyDeviceToHost,
                          t->stream));
    KH_SYNC(t);
    // a walk sized before it ran (kh_assemble_dev's bound) that passed its text bound or ran out of
    // walker chunks (both only on malformed input, e.g. walks that overlap) is redone the slow way:
    // the text sized from the scanned total, the chunk pool from what the first attempt asked for
    if (t->walk_bounded && t->last_contigs && (st[kh::ST_CHUNK_OVF] || ob > t->text.bytes)) {
        KH_HIP(hipMemsetAsync(t->stats.as<unsigned long long>() + kh::ST_CHUNK_OVF, 0, 8, t->stream));
        t->text_sync = true;
        if (int rc = kh_assemble_dev(t)) return rc;
        if (int rc = check_stats(t)) return rc;
        uint64_t o2 = 0;
        if (int rc = read_ctr(t, kh::CT_OUT_BYTES, &o2)) return rc;
        ob = o2;
    } else if (int rc = stats_status(st)) {
        return rc;
    }
    if (n_contigs) *n_contigs = t->last_contigs;
    if (out_bytes) *out_bytes = ob;
    return KH_OK;
}

int kh_contigs_text_dev(kh_table* t, const char** dev_text, uint64_t* bytes) {
    if (!t || !dev_text || !bytes) return fail(KH_ERR_ARG, "null argument");
    if (!t->assembled) return fail(KH_ERR_STATE, "no assemble since the last insert/clear");
    uint64_t ob = 0;
    if (int rc = read_ctr(t, kh::CT_OUT_BYTES, &ob)) return rc;
    if (t->last_contigs && ob > t->text.bytes)
        return fail(KH_ERR_STATE, "contig text of %llu bytes passed its %llu-byte bound (malformed input?): "
                                  "kh_assemble redoes the walk sized", (unsigned long long)ob,
                    (unsigned long long)t->text.bytes);
    *dev_text = t->text.as<const char>();
    *bytes = t->last_contigs ? ob : 0;
    return KH_OK;
}

int kh_contigs_text(kh_table* t, char* out, uint64_t cap) {
    const char* d = nullptr;
    uint64_t b = 0;
    if (int rc = kh_contigs_text_dev(t, &d, &b)) return rc;
    if (cap < b) return fail(KH_ERR_ARG, "buffer of %llu bytes < %llu", (unsigned long long)cap,
                             (unsigned long long)b);
    if (b) KH_HIP(hipMemcpy(out, d, b, hipMemcpyDeviceToHost));
    return KH_OK;
}

int kh_contigs_offsets(kh_table* t, uint64_t* out, uint64_t n) {
    if (!t || (!out && n)) return fail(KH_ERR_ARG, "null argument");
    if (!t->assembled) return fail(KH_ERR_STATE, "no assemble since the last insert/clear");
    if (n > t->last_contigs) return fail(KH_ERR_ARG, "asked for %llu offsets of %llu contigs",
                                         (unsigned long long)n, (unsigned long long)t->last_contigs);
    if (n) {
        KH_SYNC(t);
        KH_HIP(hipMemcpy(out, t->contig_off.p, n * 8, hipMemcpyDeviceToHost));
    }
    return KH_OK;
}

int kh_get_stats(kh_table* t, kh_stats* s) {
    if (!t || !s) return fail(KH_ERR_ARG, "null argument");
    if (int rc = set_device(t)) return rc;
    KH_SYNC(t);
    unsigned long long st[kh::ST_NUM], ct[kh::CT_NUM];
    KH_HIP(hipMemcpy(st, t->stats.p, sizeof st, hipMemcpyDeviceToHost));
    KH_HIP(hipMemcpy(ct, t->ctr.p, sizeof ct, hipMemcpyDeviceToHost));
    std::memset(s, 0, sizeof *s);
    s->capacity = t->cap;
    s->n_inserted = t->n_inserted;
    s->n_starts = ct[kh::CT_N_STARTS];
    if (t->assembled) {
        s->n_contigs = t->last_contigs;
        s->out_bytes = ct[kh::CT_OUT_BYTES];
        // bytes = sum(K + len) -> lookups = sum(len - 1) = bytes - contigs * (K + 1)
        s->n_lookups = s->out_bytes - s->n_contigs * ((uint64_t)t->kp.K + 1);
        const uint64_t nch = t->last_contigs + ct[kh::CT_CHUNK_NEXT];
        s->n_chunks = nch < t->chunk_cap ? nch : t->chunk_cap;
    }
    s->n_dup = st[kh::ST_DUP];
    s->n_full = st[kh::ST_FULL];
    s->n_bad_ext = st[kh::ST_BAD_EXT];
    s->n_missing = st[kh::ST_MISSING];
    s->n_cycle = st[kh::ST_CYCLE];
    s->n_spin = st[kh::ST_SPIN];
    s->n_chunk_ovf = st[kh::ST_CHUNK_OVF];
    s->n_bad_base = st[kh::ST_BAD_BASE];
    float ms = 0.f;
    if (t->ins_timed) {
        if (hipEventElapsedTime(&ms, t->ev_ins0, t->ev_ins2) == hipSuccess) s->ms_insert = ms;
        if (hipEventElapsedTime(&ms, t->ev_ins0, t->ev_ins1) == hipSuccess) s->ms_insert_kernel = ms;
    }
    if (t->walk_timed) {
        if (hipEventElapsedTime(&ms, t->ev_walk0, t->ev_walk1) == hipSuccess) s->ms_walk = ms;
        if (hipEventElapsedTime(&ms, t->ev_walk1, t->ev_mat1) == hipSuccess) s->ms_materialize = ms;
        if (t->wk_timed && hipEventElapsedTime(&ms, t->ev_walk0, t->ev_wk1) == hipSuccess) s->ms_walk_kernel = ms;
    }
    if (t->build_timed && hipEventElapsedTime(&ms, t->ev_b0, t->ev_b1) == hipSuccess) s->ms_build = ms;
    s->n_hot_regions = ct[kh::CT_HOT];
    s->n_spread_regions = ct[kh::CT_HOT2];
    s->n_overflow = t->last_insert_part ? ct[kh::CT_OVF2] : 0;
    (void)hipGetLastError();  // a failed elapsed-time query is not the caller's error
    return KH_OK;
}

// ---- device memory helpers -------------------------------------------------------------------
int kh_dev_malloc(void** p, uint64_t bytes, int device) {
    if (!p) return fail(KH_ERR_ARG, "null out pointer");
    KH_HIP(hipSetDevice(device));
    hipError_t e = hipMalloc(p, bytes ? bytes : 16);
    if (e != hipSuccess) return fail(KH_ERR_NOMEM, "hipMalloc(%llu): %s", (unsigned long long)bytes,
                                     hipGetErrorString(e));
    return KH_OK;
}
int kh_dev_free(void* p) {
    if (p) KH_HIP(hipFree(p));
    return KH_OK;
}
int kh_memcpy_htod(void* dst, const void* src, uint64_t bytes) {
    if (bytes) KH_HIP(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return KH_OK;
}
int kh_memcpy_dtoh(void* dst, const void* src, uint64_t bytes) {
    if (bytes) KH_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return KH_OK;
}

// ---- sharded multi-GPU path -------------------------------------------------------------------
int kh_key_owner(const kh_table* t, const uint8_t* packed_key, int nranks) {
    if (!t || !packed_key) return fail(KH_ERR_ARG, "null argument");
    if (nranks < 1 || nranks > kh::MAX_RANKS) return fail(KH_ERR_ARG, "nranks %d outside [1,%d]", nranks, kh::MAX_RANKS);
    return (int)kh::owner_key(kh::key_from_packed(packed_key, t->kp), t->kp, (uint32_t)nranks);
}

int kh_word_count(int k) { return (k >= 1 && k <= KH_K_MAX) ? kh::make_params(k).W : KH_ERR_ARG; }

namespace {
int ensure_route(kh_table* t, uint64_t n, int nranks) {
    const uint64_t m = kh::route_blocks(n) * (uint64_t)nranks + 1;
    int rc;
    if ((rc = t->route_hist.ensure(m * 8))) return rc;
    if ((rc = t->route_off.ensure(m * 8))) return rc;
    if ((rc = t->route_scratch.ensure((kh::scan_scratch_words(m) + 2) * 8))) return rc;
    return KH_OK;
}

}  // namespace

int kh_collect_starts_dev(kh_table* t, const void* dev_recs, uint64_t n) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (n == 0) return KH_OK;
    if (!dev_recs) return fail(KH_ERR_ARG, "null records");
    if (int rc = set_device(t)) return rc;
    int rc;
    const uint64_t nw = (n + 63) / 64;
    if ((rc = t->mask.ensure(nw * 8))) return rc;
    if ((rc = t->mask_off.ensure(nw * 8))) return rc;
    if ((rc = t->scratch.ensure(kh::scan_scratch_words(nw) * 8 + 64))) return rc;
    uint64_t have = 0;
    if ((rc = read_ctr(t, kh::CT_N_STARTS, &have))) return rc;
    if ((rc = ensure_starts(t, have + n))) return rc;
    KH_HIP(kh::launch_start_mask(t->kp, (const uint8_t*)dev_recs, n, t->mask.as<uint64_t>(), t->stream));
    KH_HIP(kh::launch_collect_starts(t->kp, (const uint8_t*)dev_recs, n, t->mask.as<uint64_t>(),
                                     t->mask_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                     t->starts.as<uint64_t>(), t->ctr.as<unsigned long long>(),
                                     t->stream));
    t->assembled = false;
    return KH_OK;
}

int kh_pack_text_dev(kh_table* t, const void* dev_text, uint64_t len, void* dev_recs, uint64_t* n_out) {
    if (!t || !n_out) return fail(KH_ERR_ARG, "null argument");
    const uint64_t n = len / ((uint64_t)t->kp.K + 4);  // read_kmers.hpp:64 fixed line length
    *n_out = n;
    if (!dev_recs || n == 0) return KH_OK;
    if (!dev_text) return fail(KH_ERR_ARG, "null text");
    if (!aligned16(dev_recs)) return fail(KH_ERR_ARG, "device records must be 16-byte aligned");
    if (int rc = set_device(t)) return rc;
    KH_HIP(kh::launch_pack_text(t->kp, (const char*)dev_text, n, (uint8_t*)dev_recs,
                                t->stats.as<unsigned long long>(), t->stream));
    return KH_OK;
}

int kh_route_dev(kh_table* t, const void* dev_recs, uint64_t n, int nranks, void* words_out,
                 void* counts_out) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (nranks < 1 || nranks > kh::MAX_RANKS) return fail(KH_ERR_ARG, "nranks %d outside [1,%d]", nranks, kh::MAX_RANKS);
    if (!counts_out || (n && (!dev_recs || !words_out))) return fail(KH_ERR_ARG, "null buffer");
    if (!aligned16(dev_recs)) return fail(KH_ERR_ARG, "device records must be 16-byte aligned");
    if (int rc = set_device(t)) return rc;
    if (int rc = ensure_route(t, n, nranks)) return rc;
    if (int rc = t->route_own.ensure((n + 16) * 4)) return rc;
    KH_HIP(kh::launch_route(t->kp, (const uint8_t*)dev_recs, n, (uint32_t)nranks,
                            t->route_hist.as<uint64_t>(), t->route_off.as<uint64_t>(),
                            t->route_scratch.as<uint64_t>(), t->route_own.as<uint32_t>(), (uint64_t*)words_out,
                            (uint64_t*)counts_out, t->stream));
    return KH_OK;
}

// Splitter segments for the migrating walk (on with the table's splitters, KH_SPLIT_BITS=0 off).
static bool mseg_enabled(const kh_table* t) { return t->kp.split_bits > 0; }

// Splitter density of the migrating walk: the table's (1 per 256 k-mers at C3 sizes). Measured
// at one rank (C3 / C5 ms per step): segments off 15.4 / 2159, table density 17.8 / 36.5, 4x
// sparser 17.3 / 66.6 — the segment phase is mostly a fixed cost (link, jump, retag rounds),
// while sparser splitters leave longer segments (more rounds) on long chains.
static kh::KParams mseg_params(const kh_table* t) {
    kh::KParams p = t->kp;
    if (p.split_bits < 1) p.split_bits = 1;
    return p;
}

// Routed words: collect the splitter k-mers this shard owns (they head migrating-walk segments).
// in_insert: the partitioned insert that follows collects them itself (k_win1): only size the list.
static int collect_word_splits(kh_table* t, const void* words, uint64_t m, bool in_insert = false) {
    if (!mseg_enabled(t) || !t->words_split) return KH_OK;
    const kh::KParams mp = mseg_params(t);
    const uint64_t need = (t->n_kmers >> (mp.split_bits > 3 ? mp.split_bits - 3 : 0)) + 4096;
    if (int rc = ensure_list(t, t->splits, t->splits_cap, need)) return rc;
    if (in_insert) return KH_OK;
    KH_HIP(kh::launch_split_collect(mp, (const uint64_t*)words, m, t->splits.as<uint64_t>(), t->splits_cap,
                                    t->ctr.as<unsigned long long>(), t->stream));
    return KH_OK;
}

int kh_route_starts_dev(kh_table* t, const void* dev_recs, uint64_t n, int nranks, void* words_out,
                        void* counts_out) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (nranks < 1 || nranks > kh::MAX_RANKS) return fail(KH_ERR_ARG, "nranks %d outside [1,%d]", nranks, kh::MAX_RANKS);
    if (!counts_out || (n && (!dev_recs || !words_out))) return fail(KH_ERR_ARG, "null buffer");
    if (!aligned16(dev_recs)) return fail(KH_ERR_ARG, "device records must be 16-byte aligned");
    if (int rc = set_device(t)) return rc;
    if (int rc = ensure_route(t, n, nranks)) return rc;
    if (int rc = t->route_own.ensure((n + 16) * 4)) return rc;
    const uint64_t nw = (n + 63) / 64;
    int rc;
    if ((rc = t->mask.ensure(nw * 8 + 8))) return rc;
    if ((rc = t->mask_off.ensure(nw * 8 + 8))) return rc;
    if ((rc = t->scratch.ensure(kh::scan_scratch_words(nw) * 8 + 64))) return rc;
    // capacity bound from host-side counts: no device read (and no host sync) per call
    if ((rc = ensure_starts(t, t->collected_n + n))) return rc;
    KH_HIP(kh::launch_route(t->kp, (const uint8_t*)dev_recs, n, (uint32_t)nranks,
                            t->route_hist.as<uint64_t>(), t->route_off.as<uint64_t>(),
                            t->route_scratch.as<uint64_t>(), t->route_own.as<uint32_t>(), (uint64_t*)words_out,
                            (uint64_t*)counts_out, t->stream, n ? t->mask.as<uint64_t>() : nullptr,
                            mseg_enabled(t) ? t->route_spl.as<unsigned long long>() : nullptr));
    if (n)
        KH_HIP(kh::launch_collect_starts(t->kp, (const uint8_t*)dev_recs, n, t->mask.as<uint64_t>(),
                                         t->mask_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                         t->starts.as<uint64_t>(), t->ctr.as<unsigned long long>(),
                                         t->stream));
    t->collected_n += n;
    t->assembled = false;
    return KH_OK;
}

int kh_route_starts_win_dev(kh_table* t, const void* dev_recs, uint64_t n, int nranks, void* words_out,
                            uint64_t win, void* counts_out) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (nranks < 1 || nranks > kh::MAX_RANKS) return fail(KH_ERR_ARG, "nranks %d outside [1,%d]", nranks, kh::MAX_RANKS);
    if (!counts_out || (n && (!dev_recs || !words_out))) return fail(KH_ERR_ARG, "null buffer");
    if (!aligned16(dev_recs) || !aligned16(words_out)) return fail(KH_ERR_ARG, "device buffers must be 16-byte aligned");
    if (win < n || win >= (1ull << 32))
        return fail(KH_ERR_ARG, "window of %llu words for %llu records (need n <= win < 2^32)", (unsigned long long)win,
                    (unsigned long long)n);
    if (t->kp.R > 15) return fail(KH_ERR_ARG, "the one-pass route takes records of <= 15 bytes (k <= 52)");
    if (int rc = set_device(t)) return rc;
    if (int rc = ensure_route(t, n, nranks)) return rc;
    const uint64_t nw = (n + 63) / 64;
    int rc;
    if ((rc = t->mask.ensure(nw * 8 + 8))) return rc;
    if ((rc = t->mask_off.ensure(nw * 8 + 8))) return rc;
    if ((rc = t->scratch.ensure(kh::scan_scratch_words(nw) * 8 + 64))) return rc;
    if ((rc = t->route_own.ensure(kh::MAX_RANKS * 4 + 64))) return rc;
    if ((rc = ensure_starts(t, t->collected_n + n))) return rc;
    KH_HIP(kh::launch_route_win(t->kp, (const uint8_t*)dev_recs, n, (uint32_t)nranks, (uint64_t*)words_out, win,
                                t->route_own.as<uint32_t>(), (uint64_t*)counts_out, n ? t->mask.as<uint64_t>() : nullptr,
                                t->ctr.as<unsigned long long>(), t->stats.as<unsigned long long>(), t->stream,
                                mseg_enabled(t) ? t->route_spl.as<unsigned long long>() : nullptr));
    if (n)
        KH_HIP(kh::launch_collect_starts(t->kp, (const uint8_t*)dev_recs, n, t->mask.as<uint64_t>(),
                                         t->mask_off.as<uint64_t>(), t->scratch.as<uint64_t>(),
                                         t->starts.as<uint64_t>(), t->ctr.as<unsigned long long>(), t->stream));
    t->collected_n += n;
    t->assembled = false;
    return KH_OK;
}

int kh_route_splitters_dev(kh_table* t, void* dev_out, int nranks) {
    if (!t || !dev_out) return fail(KH_ERR_ARG, "null argument");
    if (nranks < 1 || nranks > kh::MAX_RANKS) return fail(KH_ERR_ARG, "nranks %d outside [1,%d]", nranks, kh::MAX_RANKS);
    if (int rc = set_device(t)) return rc;
    KH_HIP(hipMemcpyAsync(dev_out, t->route_spl.p, (size_t)nranks * 8, hipMemcpyDeviceToDevice, t->stream));
    return KH_OK;
}

int kh_counters_dev(kh_table* t, void* dev_out) {
    if (!t || !dev_out) return fail(KH_ERR_ARG, "null argument");
    if (int rc = set_device(t)) return rc;
    uint64_t* o = (uint64_t*)dev_out;
    const unsigned long long* c = t->ctr.as<unsigned long long>();
    KH_HIP(hipMemcpyAsync(o, c + kh::CT_N_STARTS, 8, hipMemcpyDeviceToDevice, t->stream));
    KH_HIP(hipMemcpyAsync(o + 1, c + kh::CT_N_SPLIT, 8, hipMemcpyDeviceToDevice, t->stream));
    return KH_OK;
}

int kh_counters(kh_table* t, uint64_t* out) {
    if (!t || !out) return fail(KH_ERR_ARG, "null argument");
    if (int rc = set_device(t)) return rc;
    unsigned long long cv[kh::CT_NUM];
    ++t->host_syncs;
    if (t->ctr_early) {  // copied beside the build (kh_insert_dev): wait for that copy, not the build
        KH_HIP(hipEventSynchronize(t->ev_ctr));
        memcpy(cv, t->hctr, sizeof cv);
    } else {
        KH_HIP(hipMemcpyAsync(cv, t->ctr.p, sizeof cv, hipMemcpyDeviceToHost, t->stream));
        KH_HIP(hipStreamSynchronize(t->stream));
    }
    out[0] = cv[kh::CT_N_STARTS];
    out[1] = cv[kh::CT_N_SPLIT];
    return KH_OK;
}

int kh_insert_words_dev(kh_table* t, const void* words, uint64_t m) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (m == 0) return KH_OK;
    if (!words) return fail(KH_ERR_ARG, "null words");
    if (t->n_inserted + m > t->n_kmers)
        return fail(KH_ERR_FULL, "inserting %llu k-mers into a shard created for %llu (%llu in)",
                    (unsigned long long)m, (unsigned long long)t->n_kmers,
                    (unsigned long long)t->n_inserted);
    if (int rc = set_device(t)) return rc;
    if (int rc = join_succ(t)) return rc;
    t->split_ok = false;  // routed words carry no splitter marks: walks on this table use none
    const bool part = use_part_build(t, m);
    const bool coll = part && mseg_enabled(t) && t->words_split;
    if (int rc = collect_word_splits(t, words, m, coll)) return rc;
    kh::PartBuffers pb{};
    if (part)
        if (int rc = ensure_part(t, m, pb)) return rc;
    const bool fresh = part && t->n_inserted == 0;  // empty (stale or clean): the build writes every slot
    if (!fresh)
        if (int rc = clean_slots(t)) return rc;
    t->slots_stale = false;
    KH_HIP(hipEventRecord(t->ev_ins0, t->stream));
    t->build_timed = part;
    if (part) {
        KH_HIP(kh::launch_part_insert(coll ? mseg_params(t) : t->kp, nullptr, (const uint64_t*)words, m, view(t),
                                      fresh, pb, nullptr, nullptr, t->ctr.as<unsigned long long>(),
                                      t->stats.as<unsigned long long>(), t->stream, nullptr,
                                      coll ? t->splits.as<uint64_t>() : nullptr, coll ? t->splits_cap : 0, t->ev_b0));
        KH_HIP(hipEventRecord(t->ev_b1, t->stream));
    } else {
        if (int rc = cas_hot_prepass(t, nullptr, words, m)) return rc;
        KH_HIP(kh::launch_insert_words(t->kp, (const uint64_t*)words, m, view(t),
                                       t->stats.as<unsigned long long>(), t->stream));
    }
    t->last_insert_part = part;
    KH_HIP(hipEventRecord(t->ev_ins1, t->stream));
    KH_HIP(hipEventRecord(t->ev_ins2, t->stream));
    t->ins_timed = true;
    t->n_inserted += m;
    t->assembled = false;
    return KH_OK;
}

int kh_insert_words_stage_dev(kh_table* t, const void* words, uint64_t m, uint64_t total_hint) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (m && !words) return fail(KH_ERR_ARG, "null words");
    if (int rc = set_device(t)) return rc;
    if (int rc = join_succ(t)) return rc;
    if (!t->staging) {
        if (total_hint < m) total_hint = m;
        if (t->n_inserted + total_hint > t->n_kmers)
            return fail(KH_ERR_FULL, "staging %llu k-mers into a shard created for %llu (%llu in)",
                        (unsigned long long)total_hint, (unsigned long long)t->n_kmers,
                        (unsigned long long)t->n_inserted);
        t->split_ok = false;  // routed words carry no splitter marks
        t->stage_total = total_hint;
        t->stage_n = 0;
        t->stage_part = use_part_build(t, total_hint);
        kh::PartBuffers pb{};
        if (t->stage_part)
            if (int rc = ensure_part(t, total_hint, pb)) return rc;
        // a partitioned build into a fresh table rewrites every slot: no clear needed
        t->stage_fresh = t->stage_part && t->n_inserted == 0;
        if (!t->stage_fresh)
            if (int rc = clean_slots(t)) return rc;
        KH_HIP(hipEventRecord(t->ev_ins0, t->stream));
        t->staging = true;
        t->last_insert_part = t->stage_part;
        if (t->stage_part) {
            kh::PartBuffers b{};
            if (int rc = ensure_part(t, total_hint, b)) return rc;
            KH_HIP(kh::launch_part_stage(t->kp, nullptr, 0, total_hint, true, b, t->ctr.as<unsigned long long>(),
                                         t->stats.as<unsigned long long>(), t->stream));
        }
    }
    if (t->stage_n + m > t->stage_total)
        return fail(KH_ERR_FULL, "staged %llu + %llu words exceed the build's %llu",
                    (unsigned long long)t->stage_n, (unsigned long long)m, (unsigned long long)t->stage_total);
    if (m == 0) return KH_OK;
    const bool coll = t->stage_part && mseg_enabled(t) && t->words_split;
    if (int rc = collect_word_splits(t, words, m, coll)) return rc;
    if (t->stage_part) {
        kh::PartBuffers b{};
        if (int rc = ensure_part(t, t->stage_total, b)) return rc;
        KH_HIP(kh::launch_part_stage(coll ? mseg_params(t) : t->kp, (const uint64_t*)words, m, t->stage_total, false, b,
                                     t->ctr.as<unsigned long long>(), t->stats.as<unsigned long long>(),
                                     t->stream, coll ? t->splits.as<uint64_t>() : nullptr,
                                     coll ? t->splits_cap : 0, t->stage_fresh && t->stage_n == 0, t->cap));
    } else {
        if (t->stage_n == 0)  // the first staged batch stands for the whole build (stage_total)
            if (int rc = cas_hot_prepass(t, nullptr, words, m, t->stage_total)) return rc;
        KH_HIP(kh::launch_insert_words(t->kp, (const uint64_t*)words, m, view(t),
                                       t->stats.as<unsigned long long>(), t->stream));
    }
    t->stage_n += m;
    return KH_OK;
}

int kh_insert_words_finish(kh_table* t) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (!t->staging) return fail(KH_ERR_STATE, "no staged insert open");
    if (int rc = set_device(t)) return rc;
    t->build_timed = t->stage_part;
    if (t->stage_part) {
        kh::PartBuffers b{};
        if (int rc = ensure_part(t, t->stage_total, b)) return rc;
        KH_HIP(hipEventRecord(t->ev_b0, t->stream));
        KH_HIP(kh::launch_part_finish(t->kp, t->stage_total, view(t), t->stage_fresh, b, t->ctr.as<unsigned long long>(),
                                      t->stats.as<unsigned long long>(), t->stream));
        KH_HIP(hipEventRecord(t->ev_b1, t->stream));
        t->slots_stale = false;
    }
    KH_HIP(hipEventRecord(t->ev_ins1, t->stream));
    KH_HIP(hipEventRecord(t->ev_ins2, t->stream));
    t->ins_timed = true;
    t->n_inserted += t->stage_n;
    t->staging = false;
    t->stage_n = 0;
    t->assembled = false;
    return KH_OK;
}

// ---- migrating-walker rounds --------------------------------------------------------------------

static kh::MSegState mseg_state(kh_table* t) {
    kh::MSegState st;
    st.len = t->ms_len.as<uint32_t>();
    st.link_hi = t->ms_hi.as<uint64_t>();
    st.link_lo = t->ms_lo.as<uint64_t>();
    st.has_link = t->ms_has.as<uint8_t>();
    st.done = t->ms_done.as<uint8_t>();
    st.jump = t->ms_jump.as<uint64_t>();
    st.acc = t->ms_acc.as<uint64_t>();
    return st;
}

// device words of mw_misc: [0] link-scan finish count, [2] text-store count, [3] first round's
// walkers, [4] carry count of buffer 0, [5] of buffer 1
static unsigned long long* mw_word(kh_table* t, int i) { return t->mw_misc.as<unsigned long long>() + i; }

int kh_mwalk_begin(kh_table* t, int nranks, int rank, uint64_t total_kmers, uint64_t n_starts, uint64_t n_splitters,
                   uint64_t total_walkers, uint64_t* n_walkers) {
    if (!t) return fail(KH_ERR_ARG, "null table");
    t->ctr_early = false;  // counters may change: assemble reads them on the stream
    if (nranks < 1 || nranks > kh::MAX_RANKS || rank < 0 || rank >= nranks)
        return fail(KH_ERR_ARG, "bad rank %d of %d", rank, nranks);
    if (int rc = set_device(t)) return rc;
    if (int rc = join_succ(t)) return rc;
    if (int rc = clean_slots(t)) return rc;
    int rc;
    // the counts come from the caller (kh_counters_dev / kh_route_splitters_dev, read together
    // with its own exchange): no device read here
    const uint64_t ns = n_starts;
    if (ns >= (1ull << 31)) return fail(KH_ERR_ARG, "%llu start k-mers on one rank (max 2^31)", (unsigned long long)ns);
    uint64_t nsp = 0;
    // splitter segments: every splitter this shard owns seeds a walker too (kh_mseg.hip), on or
    // off the same way on every rank (walkers stop before splitters owned anywhere)
    t->ms_on = mseg_enabled(t) && t->words_split && !t->mw_seg_off;
    if (t->ms_on) {
        nsp = n_splitters;
        if ((rc = ensure_list(t, t->splits, t->splits_cap, nsp))) return rc;
        if (ns + nsp >= (1ull << 31))
            return fail(KH_ERR_ARG, "%llu walk segments on one rank (max 2^31)", (unsigned long long)(ns + nsp));
    }
    const uint64_t nseg = ns + nsp;
    // walkers of every rank: a rank may host (and hold back) at most all of them in a round
    t->mw_wg = total_walkers > nseg ? total_walkers : nseg;
    // text store: a walker appends each k-mer of this shard once, 32 bases per full word record,
    // and leaves at most a partial word, its finish record and a 2-record link where it ends
    // (held-back walkers flush nothing extra): shard / 32 + 4 per walker of every rank, doubled
    uint64_t store_cap = 2 * (t->n_inserted / 32 + 4 * t->mw_wg) + 4096;
    if (store_cap < t->mw_store_min) store_cap = t->mw_store_min;  // a redo sized by the last attempt
    t->mw_seg_off = false;
    t->mw_store_min = 0;
    t->mw_soft = t->mw_soft_next;
    t->mw_soft_next = 0;
    if ((rc = t->mw_misc.ensure(64)) || (rc = t->mw_store.ensure(store_cap * 16)))
        return rc;
    t->ms_ns = ns;
    t->ms_nsp = nsp;
    if (t->ms_on) {
        uint64_t cap2 = 64;
        while (cap2 < 2 * nsp + 64) cap2 <<= 1;
        t->ms_cap2 = cap2;
        if ((rc = t->ms_len.ensure((nseg + 1) * 4)) || (rc = t->ms_hi.ensure((nseg + 1) * 8)) ||
            (rc = t->ms_lo.ensure((nseg + 1) * 8)) || (rc = t->ms_has.ensure(nseg + 1)) ||
            (rc = t->ms_done.ensure(nseg + 1)) || (rc = t->ms_jump.ensure((nseg + 1) * 8)) ||
            (rc = t->ms_acc.ensure((nseg + 1) * 8)) || (rc = t->ms_stab.ensure(cap2 * 16)) ||
            (rc = t->ms_stab_id.ensure(cap2 * 4)) || (rc = t->ms_misc.ensure(64)))
            return rc;
    }
    unsigned long long* ctr = t->ctr.as<unsigned long long>();
    unsigned long long* stats = t->stats.as<unsigned long long>();
    // the caller's counts must be the device's (a mismatch fails the walk at the next sync)
    KH_HIP(kh::launch_fin_check(ctr + kh::CT_N_STARTS, ns, nullptr, 0, stats, t->stream));
    if (t->ms_on) KH_HIP(kh::launch_fin_check(ctr + kh::CT_N_SPLIT, nsp, nullptr, 0, stats, t->stream));
    t->mw_P = (uint32_t)nranks;
    t->mw_rank = (uint32_t)rank;
    t->rw_n = nseg;
    t->rw_total = total_kmers > ns ? total_kmers : ns;
    t->mw_store_n = 0;
    t->mw_store_bound = store_cap;
    t->mw_store_known = false;
    t->mw_cur = 0;
    KH_HIP(hipMemsetAsync(mw_word(t, 2), 0, 8 * 6, t->stream));  // store count, walkers, carries, long walks
    KH_HIP(hipEventRecord(t->ev_walk0, t->stream));
    t->wk_timed = false;
    // chain records: the first round's walkers read the start and splitter lists themselves and
    // look up their own k-mer first (a record covering its run is read next, as on one GPU), and
    // the records' successor runs are resolved beside the first round (k_rec_succ)
    kh::KParams ikp = t->kp;
    if (t->headrec.p && t->hcap && kh::rec_succ_fits(ikp, t->hcap)) {
        hipStream_t rs = t->stream;
        if (kh::rec_succ_side(ikp) && t->side) {
            KH_HIP(hipEventRecord(t->ev_side, t->stream));
            KH_HIP(hipStreamWaitEvent(t->side, t->ev_side, 0));
            rs = t->side;
            t->succ_pending = true;
        }
        KH_HIP(kh::launch_rec_succ(ikp, view(t), t->headrec.as<uint64_t>(), t->hcap, rs,
                                   t->succ_pending ? 1024u : 0u));
    }
    if (t->succ_pending) KH_HIP(hipEventRecord(t->ev_conv, t->side));
    if (t->ms_on) {
        // (on the side stream beside the first round, behind the record resolve, the splitter
        // table's 780K CAS slowed the round as much as they saved: C3 walk init + rounds 1.51 vs
        // 1.53 ms)
        KH_HIP(kh::launch_mseg_init(ns, nseg, (uint32_t)rank, mseg_state(t), t->stream));
        KH_HIP(kh::launch_mseg_stab(t->kp, t->splits.as<uint64_t>(), nsp, t->ms_stab.as<uint64_t>(),
                                    t->ms_stab_id.as<uint32_t>(), t->ms_cap2, t->stream));
    }
    t->mw_live = true;
    t->mw_stepped = false;
    t->assembled = false;
    if (n_walkers) *n_walkers = nseg;
    return KH_OK;
}

int kh_mwalk_round_dev(kh_table* t, const void* in_slots, uint64_t in_cap, void* out_slots, uint64_t out_cap,
                       void* dev_live) {
    if (!t || !t->mw_live) return fail(KH_ERR_STATE, "kh_mwalk_begin first");
    if (!out_slots || !dev_live || out_cap == 0) return fail(KH_ERR_ARG, "null output slots / live word");
    if (t->mw_stepped && !in_slots) return fail(KH_ERR_ARG, "null input slots");
    if (int rc = set_device(t)) return rc;
    const uint32_t P = t->mw_P;
    int rc;
    // this round's walkers: the start and splitter lists (first round), or the P slots received
    const uint64_t* src = nullptr;
    uint64_t nb = t->rw_n;  // bound (every walker is live in the first round)
    unsigned long long* n_dev = mw_word(t, 3);
    if (t->mw_stepped) {
        nb = (uint64_t)P * in_cap;
        if (nb > t->mw_wg) nb = t->mw_wg;  // walkers never multiply
        if ((rc = t->mw_list.ensure((nb + 1) * kh::MSG_WORDS * 8))) return rc;
        KH_HIP(kh::launch_slot_gather((const uint64_t*)in_slots, P, in_cap, t->mw_list.as<uint64_t>(), n_dev, nb,
                                      t->stream, t->stats.as<unsigned long long>()));
        src = t->mw_list.as<uint64_t>();
    } else {
        KH_HIP(kh::launch_add_count(n_dev, t->rw_n, nullptr, 0, t->stream));
    }
    const uint64_t cb = t->mw_wg;  // held-back messages: at most every walker
    if ((rc = t->mw_tmp.ensure((nb + 1) * kh::MSG_WORDS * 8)) || (rc = t->mw_dst.ensure(nb + 1)) ||
        (rc = t->mw_stage.ensure((nb + 1) * kh::MW_REC_SLOTS * 16)) || (rc = t->mw_nrec.ensure(nb + 1)) ||
        (rc = t->mw_off.ensure((nb + 1) * 8)) || (rc = t->scratch.ensure(kh::scan_scratch_words(nb) * 8 + 64)) ||
        (rc = t->mw_cnt.ensure((2 * P + 2) * 8)) ||
        (rc = t->mw_carry[0].ensure((cb + 1) * kh::MSG_WORDS * 8)) ||
        (rc = t->mw_carry[1].ensure((cb + 1) * kh::MSG_WORDS * 8)) || (rc = t->mw_carry_dst[0].ensure(cb + 1)) ||
        (rc = t->mw_carry_dst[1].ensure(cb + 1)) || (rc = ensure_route(t, nb + cb, (int)P)))
        return rc;
    kh::MWalkRound mw;
    mw.P = P;
    mw.rank = t->mw_rank;
    mw.split_bits = t->ms_on ? (uint32_t)mseg_params(t).split_bits : 0u;
    mw.headrec = t->headrec.as<uint64_t>();
    mw.hcap = t->headrec.p ? t->hcap : 0u;
    mw.max_steps = t->rw_total;
    mw.soft_steps = t->mw_soft;
    mw.long_ctr = mw_word(t, 6);
    mw.in = src;
    mw.starts = t->starts.as<uint64_t>();
    mw.splits = t->splits.as<uint64_t>();
    mw.ns = t->ms_ns;
    mw.n_in = nb;
    mw.n_dev = n_dev;
    mw.hot_on = t->ctr.as<unsigned long long>() + kh::CT_HOT;  // the kernel skips the bitmap when 0
    mw.tmp = t->mw_tmp.as<uint64_t>();
    mw.dst = t->mw_dst.as<uint8_t>();
    mw.stage = t->mw_stage.as<uint64_t>();
    mw.nrec = t->mw_nrec.as<uint8_t>();
    KH_HIP(kh::launch_mw_run(t->kp, view(t), mw, t->stats.as<unsigned long long>(), t->stream));
    // text records of this round -> the rank-local store at offsets continuing its device-side
    // count (sized at begin; a walk that would pass it fails instead of overrunning it)
    unsigned long long* store_n = mw_word(t, 2);
    KH_HIP(kh::launch_mw_text_offsets(mw, t->mw_off.as<uint64_t>(), t->scratch.as<uint64_t>(), store_n, t->stream));
    KH_HIP(kh::launch_mw_compact(mw, t->mw_off.as<uint64_t>(), t->mw_store.as<uint64_t>(), t->mw_store_bound,
                                 t->stats.as<unsigned long long>(), t->stream));
    // outgoing walkers (+ the ones held back last round) -> P slots of out_cap; overflow held back
    const int cur = t->mw_cur, nxt = 1 - cur;
    kh::SlotRound r;
    r.P = P;
    r.nb = nb;
    r.n_dev = n_dev;
    r.dst = mw.dst;
    r.tmp = mw.tmp;
    r.cb = t->mw_stepped ? cb : 0;
    r.carry_n = mw_word(t, 4 + cur);
    r.carry_dst = t->mw_carry_dst[cur].as<uint8_t>();
    r.carry = t->mw_carry[cur].as<uint64_t>();
    r.cap = out_cap;
    r.out = (uint64_t*)out_slots;
    r.carry_out = t->mw_carry[nxt].as<uint64_t>();
    r.carry_dst_out = t->mw_carry_dst[nxt].as<uint8_t>();
    r.carry_n_out = mw_word(t, 4 + nxt);
    r.live = (unsigned long long*)dev_live;
    r.cnt = t->mw_cnt.as<uint64_t>();
    KH_HIP(kh::launch_slot_round(r, t->route_hist.as<uint64_t>(), t->route_off.as<uint64_t>(),
                                 t->route_scratch.as<uint64_t>(), t->stream));
    t->mw_cur = nxt;
    t->mw_stepped = true;
    return KH_OK;
}

int kh_mwalk_flags_dev(kh_table* t, void* dev_out) {
    if (!t || !t->mw_live) return fail(KH_ERR_STATE, "kh_mwalk_begin first");
    if (!dev_out) return fail(KH_ERR_ARG, "null output");
    if (int rc = set_device(t)) return rc;
    KH_HIP(kh::launch_mw_flags(t->stats.as<unsigned long long>() + kh::ST_CHUNK_OVF, mw_word(t, 2), (uint64_t*)dev_out,
                               t->stream, t->mw_soft ? mw_word(t, 6) : nullptr));
    return KH_OK;
}

int kh_mwalk_short(kh_table* t, uint64_t total_kmers, uint64_t total_starts, int* armed) {
    if (!t || !armed) return fail(KH_ERR_ARG, "null argument");
    *armed = 0;
    // splitter segments cut the rounds of long contigs; where the mean contig (every rank's k-mers
    // over every rank's starts) is shorter than the splitter spacing (C3: 104 < 256) the walk goes
    // without them first, and a walker past 4 spacings ends it (the hosts then walk segmented)
    if (!mseg_enabled(t) || !t->words_split || t->mw_seg_off || !total_starts) return KH_OK;
    const int sb = mseg_params(t).split_bits;
    if (sb <= 0 || total_kmers / total_starts > (1ull << sb)) return KH_OK;
    t->mw_seg_off = true;
    t->mw_soft_next = 4ull << sb;
    *armed = 1;
    return KH_OK;
}

int kh_mwalk_abandon(kh_table* t) {
    if (!t || !t->mw_live) return fail(KH_ERR_STATE, "kh_mwalk_begin first");
    if (int rc = set_device(t)) return rc;
    if (int rc = join_succ(t)) return rc;
    KH_HIP(hipMemsetAsync(t->stats.as<unsigned long long>() + kh::ST_CHUNK_OVF, 0, 8, t->stream));
    t->mw_live = false;
    t->assembled = false;
    return KH_OK;
}

int kh_mwalk_redo(kh_table* t, uint64_t store_records) {
    if (!t || !t->mw_live) return fail(KH_ERR_STATE, "kh_mwalk_begin first");
    if (int rc = set_device(t)) return rc;
    if (int rc = join_succ(t)) return rc;
    // the overlap / overflow this walk reported is answered by the redo, not an error
    KH_HIP(hipMemsetAsync(t->stats.as<unsigned long long>() + kh::ST_CHUNK_OVF, 0, 8, t->stream));
    t->mw_seg_off = true;
    t->mw_store_min = store_records;
    t->mw_live = false;
    t->assembled = false;
    return KH_OK;
}

int kh_mwalk_text_bound(kh_table* t, uint64_t* n_records) {
    if (!t || !t->mw_live) return fail(KH_ERR_STATE, "kh_mwalk_begin first");
    if (!n_records) return fail(KH_ERR_ARG, "null output");
    *n_records = t->mw_store_bound;
    return KH_OK;
}

int kh_mwalk_text_dev(kh_table* t, void* out, void* counts) {
    if (!t || !t->mw_live) return fail(KH_ERR_STATE, "kh_mwalk_begin first");
    if (int rc = join_succ(t)) return rc;
    if (!counts || (t->mw_store_bound && !out)) return fail(KH_ERR_ARG, "null buffer");
    if (int rc = set_device(t)) return rc;
    if (int rc = ensure_route(t, t->mw_store_bound, (int)t->mw_P)) return rc;
    // the store's records (device count) grouped by origin; out holds kh_mwalk_text_bound records
    KH_HIP(kh::launch_mw_group_text(t->mw_store.as<uint64_t>(), t->mw_store_bound, t->mw_P,
                                    t->route_hist.as<uint64_t>(), t->route_off.as<uint64_t>(),
                                    t->route_scratch.as<uint64_t>(), (uint64_t*)out, (uint64_t*)counts, t->stream,
                                    mw_word(t, 2)));
    return KH_OK;
}

// The origin's line writer (K >= 16): its word-major first chunks (chunk c = contig c, filled by
// the record scan, k_mw_lens / k_mseg_scan), or null at K < 16.
static uint64_t* origin_chunks(kh_table* t, uint64_t nc) {
    if (t->kp.K < 16 || nc == 0 || t->chunk_data.ensure(nc * kh::CHUNK_WORDS * 8)) return nullptr;
    return t->chunk_data.as<uint64_t>();
}

// The origin's text, first part (after the contig offsets): at K >= 16 the line writer stores
// every line whole — heads, each contig's first CHUNK_BASES bases of its start segment (from the
// first chunks origin_chunks gave the record scan), newlines — and the word writers that follow
// cover the rest (start-segment words >= CHUNK_WORDS, splitter segments); at K < 16 the heads
// writer runs and the word writers cover every word. Returns the word writers' first word number
// (kh::WMIN_ERR: no memory). slen[c] + slen_add = k-mers of contig c's start segment.
static uint32_t origin_lines(kh_table* t, uint64_t nc, const uint32_t* clen, int slen_add, const uint32_t* slen,
                             bool chunks) {
    unsigned long long* ctr = t->ctr.as<unsigned long long>();
    if (chunks && t->kp.K >= 16 && nc) {
        if (t->line_first.ensure(kh::line_first_words(t->text.bytes) * 4)) return kh::WMIN_ERR;
        kh::WalkBuffers wb{};
        wb.starts = t->starts.as<uint64_t>();
        wb.n_starts = nc;
        wb.contig_len = const_cast<uint32_t*>(slen);
        wb.chunk_data = t->chunk_data.as<uint64_t>();
        wb.chunk_cap = nc;
        if (kh::launch_text_lines(t->kp, wb, clen, slen_add, t->contig_off.as<uint64_t>(), t->text.as<char>(), ctr,
                                  t->stream, t->text.bytes, t->line_first.as<uint32_t>(), t->text.bytes))
            return kh::CHUNK_WORDS;
    }
    if (kh::launch_write_heads(t->kp, t->starts.as<uint64_t>(), nc, clen, t->contig_off.as<uint64_t>(),
                               t->text.as<char>(), t->stream, t->text.bytes) != hipSuccess)
        return kh::WMIN_ERR;
    return 0;
}

// the contig text bytes: at most K + 1 per contig + 32 per word record (no device read)
static int text_for(kh_table* t, uint64_t nc, uint64_t word_recs) {
    return t->text.ensure(nc * (uint64_t)(t->kp.K + 1) + 32 * word_recs + 64);
}

int kh_mwalk_end_dev(kh_table* t, const void* recs, uint64_t n) {
    if (!t || !t->mw_live) return fail(KH_ERR_STATE, "kh_mwalk_begin first");
    if (t->ms_on && t->ms_nsp)
        return fail(KH_ERR_STATE, "segmented walk: use kh_mwalk_link_dev .. kh_mwalk_end_seg_dev");
    if (n && !recs) return fail(KH_ERR_ARG, "null records");
    if (int rc = set_device(t)) return rc;
    const uint64_t nc = t->ms_ns;
    int rc;
    if ((rc = t->contig_len.ensure((nc + 1) * 4)) || (rc = t->contig_off.ensure((nc + 1) * 8)) ||
        (rc = t->scratch.ensure(kh::scan_scratch_words(nc) * 8 + 64)) || (rc = text_for(t, nc, n)))
        return rc;
    unsigned long long* ctr = t->ctr.as<unsigned long long>();
    KH_HIP(hipEventRecord(t->ev_walk1, t->stream));
    KH_HIP(hipMemsetD32Async((hipDeviceptr_t)t->contig_len.p, 1, nc + 1, t->stream));
    KH_HIP(hipMemsetAsync(ctr + kh::CT_MW_FIN, 0, 8, t->stream));
    uint64_t* chunks = origin_chunks(t, nc);
    KH_HIP(kh::launch_mw_lens((const uint64_t*)recs, n, nc, t->contig_len.as<uint32_t>(), ctr + kh::CT_MW_FIN,
                              t->stream, chunks));
    // every walker came home (else kh_sync reports KH_ERR_NOT_FOUND)
    KH_HIP(kh::launch_fin_check(ctr + kh::CT_MW_FIN, nc, nullptr, 0, t->stats.as<unsigned long long>(), t->stream));
    KH_HIP(kh::launch_contig_offsets(t->kp.K, t->contig_len.as<uint32_t>(), nc, t->contig_off.as<uint64_t>(),
                                     t->scratch.as<uint64_t>(), ctr + kh::CT_OUT_BYTES, t->stream));
    if (nc == 0) KH_HIP(hipMemsetAsync(ctr + kh::CT_OUT_BYTES, 0, 8, t->stream));
    // the text is sized from a host bound (no device read): every writer stops at its end, so a
    // corrupt length or an overflowed store fails at kh_sync instead of writing past it
    const uint32_t wmin = origin_lines(t, nc, t->contig_len.as<uint32_t>(), 0, t->contig_len.as<uint32_t>(), chunks);
    if (wmin == kh::WMIN_ERR) return KH_ERR_NOMEM;
    KH_HIP(kh::launch_mw_words(t->kp.K, (const uint64_t*)recs, n, nc, t->contig_len.as<uint32_t>(),
                               t->contig_off.as<uint64_t>(), t->text.as<char>(), t->text.bytes, t->stream, wmin));
    KH_HIP(hipEventRecord(t->ev_mat1, t->stream));
    t->walk_timed = true;
    t->last_contigs = nc;
    t->assembled = true;
    t->mw_live = false;
    return KH_OK;
}

int kh_mwalk_segments(kh_table* t, uint64_t* n_splitter_segments) {
    if (!t || !t->mw_live) return fail(KH_ERR_STATE, "kh_mwalk_begin first");
    if (!n_splitter_segments) return fail(KH_ERR_ARG, "null output");
    *n_splitter_segments = t->ms_on ? t->ms_nsp : 0;
    return KH_OK;
}

int kh_mwalk_link_dev(kh_table* t, const void* recs, uint64_t n, void* out, void* counts) {
    if (!t || !t->mw_live || !t->ms_on) return fail(KH_ERR_STATE, "no segmented migrating walk");
    if (!counts || (n && !recs)) return fail(KH_ERR_ARG, "null buffer");
    if (int rc = set_device(t)) return rc;
    const uint64_t nseg = t->ms_ns + t->ms_nsp;
    if (nseg && !out) return fail(KH_ERR_ARG, "null output");
    if (int rc = ensure_route(t, nseg, (int)t->mw_P)) return rc;
    unsigned long long* fin = t->ms_misc.as<unsigned long long>();
    // [0] finished segments, [1] the splitter count (kh_mwalk_pred_dev), [2] start-segment words
    // past the line writer's first chunks
    KH_HIP(hipMemsetAsync(fin, 0, 24, t->stream));
    const kh::MSegState st = mseg_state(t);
    t->ms_chunks = origin_chunks(t, t->ms_ns) != nullptr;
    KH_HIP(kh::launch_mseg_scan((const uint64_t*)recs, n, nseg, st, fin, t->stream,
                                t->ms_chunks ? t->chunk_data.as<uint64_t>() : nullptr, t->ms_ns, fin + 2));
    // every segment's walker came home (else kh_sync reports KH_ERR_NOT_FOUND)
    KH_HIP(kh::launch_fin_check(fin, nseg, nullptr, 0, t->stats.as<unsigned long long>(), t->stream));
    KH_HIP(kh::launch_mseg_link(t->kp, st, t->ms_ns, nseg, t->mw_P, t->mw_rank, t->route_hist.as<uint64_t>(),
                                t->route_off.as<uint64_t>(), t->route_scratch.as<uint64_t>(), (uint64_t*)out,
                                (uint64_t*)counts, t->stream));
    return KH_OK;
}

int kh_mwalk_pred_dev(kh_table* t, const void* links, uint64_t m, void* preds_out, uint64_t stride) {
    if (!t || !t->mw_live || !t->ms_on) return fail(KH_ERR_STATE, "no segmented migrating walk");
    if ((m && !links) || (stride && !preds_out)) return fail(KH_ERR_ARG, "null buffer");
    if (stride < t->ms_nsp)
        return fail(KH_ERR_ARG, "stride %llu below this rank's %llu splitter segments", (unsigned long long)stride,
                    (unsigned long long)t->ms_nsp);
    if (int rc = set_device(t)) return rc;
    const kh::MSegState st = mseg_state(t);
    KH_HIP(kh::launch_mseg_pred((const uint64_t*)links, m, t->ms_stab.as<uint64_t>(), t->ms_stab_id.as<uint32_t>(),
                                t->ms_cap2, t->ms_ns, st, t->stats.as<unsigned long long>(), t->stream));
    // nsp on the device: this rank's exact count (the host's, checked at begin)
    unsigned long long* nsp = t->ms_misc.as<unsigned long long>() + 1;
    KH_HIP(kh::launch_add_count(nsp, t->ms_nsp, nullptr, 0, t->stream));
    KH_HIP(kh::launch_mseg_preds_out(st, t->ms_ns, nsp, t->ms_nsp, stride, (uint64_t*)preds_out, t->stream));
    return KH_OK;
}

int kh_mwalk_resolve_dev(kh_table* t, const void* all_preds, uint64_t stride) {
    if (!t || !t->mw_live || !t->ms_on) return fail(KH_ERR_STATE, "no segmented migrating walk");
    const uint64_t N = (uint64_t)t->mw_P * stride;
    if (N && !all_preds) return fail(KH_ERR_ARG, "null predecessor tables");
    if (int rc = set_device(t)) return rc;
    int rc;
    const uint32_t np = kh::mseg_resolve_passes(N);
    if ((rc = t->ms_res[0].ensure((N + 1) * 8)) || (rc = t->ms_res[1].ensure((N + 1) * 8)) ||
        (rc = t->ms_res[2].ensure(N + 1)) || (rc = t->ms_res[3].ensure((N + 1) * 8)) ||
        (rc = t->ms_res[4].ensure((N + 1) * 8)) || (rc = t->ms_res[5].ensure(N + 1)) ||
        (rc = t->ms_pend.ensure((uint64_t)np * 8 + 8)))
        return rc;
    unsigned long long* nsp = t->ms_misc.as<unsigned long long>() + 1;
    KH_HIP(kh::launch_mseg_resolve((const uint64_t*)all_preds, N, stride, t->mw_rank, t->ms_ns, nsp, t->ms_nsp,
                                   mseg_state(t), t->ms_res[0].as<uint64_t>(), t->ms_res[1].as<uint64_t>(),
                                   t->ms_res[2].as<uint8_t>(), t->ms_res[3].as<uint64_t>(),
                                   t->ms_res[4].as<uint64_t>(), t->ms_res[5].as<uint8_t>(),
                                   t->ms_pend.as<unsigned long long>(), t->stream));
    return KH_OK;
}

int kh_mwalk_retag_dev(kh_table* t, const void* recs, uint64_t n, void* out, void* counts) {
    if (!t || !t->mw_live || !t->ms_on) return fail(KH_ERR_STATE, "no segmented migrating walk");
    if (!counts || (n && !recs) || (n + t->ms_nsp && !out)) return fail(KH_ERR_ARG, "null buffer");
    if (int rc = set_device(t)) return rc;
    if (int rc = ensure_route(t, n + t->ms_nsp, (int)t->mw_P)) return rc;
    const kh::MSegState st = mseg_state(t);
    KH_HIP(kh::launch_mseg_check(t->ms_ns, t->ms_ns + t->ms_nsp, st, nullptr, t->stats.as<unsigned long long>(),
                                 t->stream));
    KH_HIP(kh::launch_mseg_retag((const uint64_t*)recs, n, t->ms_ns, t->ms_nsp, st, t->mw_P,
                                 t->route_hist.as<uint64_t>(), t->route_off.as<uint64_t>(),
                                 t->route_scratch.as<uint64_t>(), (uint64_t*)out, (uint64_t*)counts, t->stream));
    return KH_OK;
}

int kh_mwalk_end_seg_dev(kh_table* t, const void* recs, uint64_t n, const void* seg_recs, uint64_t m) {
    if (!t || !t->mw_live || !t->ms_on) return fail(KH_ERR_STATE, "no segmented migrating walk");
    if ((n && !recs) || (m && !seg_recs)) return fail(KH_ERR_ARG, "null records");
    if (int rc = set_device(t)) return rc;
    const uint64_t nc = t->ms_ns;
    int rc;
    if ((rc = t->contig_len.ensure((nc + 1) * 4)) || (rc = t->contig_off.ensure((nc + 1) * 8)) ||
        (rc = t->scratch.ensure(kh::scan_scratch_words(nc) * 8 + 64)) || (rc = text_for(t, nc, n + m)))
        return rc;
    unsigned long long* ctr = t->ctr.as<unsigned long long>();
    const kh::MSegState st = mseg_state(t);
    KH_HIP(hipEventRecord(t->ev_walk1, t->stream));
    KH_HIP(kh::launch_mseg_lens((const uint64_t*)seg_recs, m, nc, st, t->contig_len.as<uint32_t>(), t->stream));
    KH_HIP(kh::launch_contig_offsets(t->kp.K, t->contig_len.as<uint32_t>(), nc, t->contig_off.as<uint64_t>(),
                                     t->scratch.as<uint64_t>(), ctr + kh::CT_OUT_BYTES, t->stream));
    if (nc == 0) KH_HIP(hipMemsetAsync(ctr + kh::CT_OUT_BYTES, 0, 8, t->stream));
    const uint32_t wmin = origin_lines(t, nc, t->contig_len.as<uint32_t>(), 1, st.len, t->ms_chunks);
    if (wmin == kh::WMIN_ERR) return KH_ERR_NOMEM;
    KH_HIP(kh::launch_mseg_words(t->kp.K, (const uint64_t*)recs, n, (const uint64_t*)seg_recs, m, nc, st,
                                 t->contig_off.as<uint64_t>(), t->text.as<char>(), t->text.bytes, t->stream, wmin,
                                 wmin ? t->ms_misc.as<unsigned long long>() + 2 : nullptr));
    KH_HIP(hipEventRecord(t->ev_mat1, t->stream));
    t->walk_timed = true;
    t->last_contigs = nc;
    t->assembled = true;
    t->mw_live = false;
    return KH_OK;
}

}  // extern "C"

