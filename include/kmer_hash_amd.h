/* kmer_hash_amd.h — C ABI of the MI355X-native k-mer hash table + contig walker.
 *
 * Drop-in boundary for the hot path of fractalclockwork/CS267_HW3 (hash_map.hpp / kmer_hash.cpp).
 * Plain C: pointers and sizes only, no C++ or torch types, no exceptions across the boundary.
 * Every entry point returns KH_OK (0) or a negative KH_ERR_*; kh_last_error() gives a message
 * (thread-local). A handle is not thread-safe; use one per host thread / process.
 *
 * Record formats (byte-identical to the reference types, align 1):
 *   key    = pkmer_t   : PACKED = (k+3)/4 bytes, 2 bits/base MSB-first, A=0 C=1 G=2 T=3,
 *                        'A'-padded tail                          (pkmer_t.hpp:6, packing.hpp:77-92)
 *   record = kmer_pair : PACKED key bytes + fb_ext[2] = {backward, forward} chars in {A,C,G,T,F}
 *                        sizeof = PACKED + 2 = 7 (k=19) / 15 (k=51)          (kmer_t.hpp:6-8,43-45)
 *   contig text        : one contig per line, extract_contig() bytes + '\n', in start-node order
 *                        = the bytes of test_<rank>.dat                (read_kmers.hpp:81-92,
 *                                                                       kmer_hash.cpp:60-68)
 * Reference entry points replaced (see INTEGRATION.md for the bindings):
 *   kh_create      <- DistributedHashMap(size, rank, world)  hash_map.hpp:50-52; HashMap(size)
 *   kh_insert*     <- DistributedHashMap::insert_all        hash_map.hpp:55-80; HashMap::insert
 *                     + start-node collection               kmer_hash.cpp:21-33
 *   kh_find*       <- DistributedHashMap::find              hash_map.hpp:83-107; HashMap::find
 *   kh_assemble*   <- assemble_contigs                      kmer_hash.cpp:38-55
 *   kh_contigs_*   <- extract_contig + output_results       read_kmers.hpp:81-92, kmer_hash.cpp:60-68
 *   kh_pack_text   <- read_kmers line parsing               read_kmers.hpp:54-79
 */
#ifndef KMER_HASH_AMD_H
#define KMER_HASH_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KH_ABI_VERSION 3
#define KH_K_MAX 60

enum {
    KH_OK = 0,
    KH_ERR_ARG = -1,        /* bad argument / unsupported k / misaligned device pointer */
    KH_ERR_HIP = -2,        /* HIP runtime error (message has the hipError string) */
    KH_ERR_NOMEM = -3,      /* device or host allocation failed */
    KH_ERR_FULL = -4,       /* more k-mers than the table was created for / probe wrapped */
    KH_ERR_NOT_FOUND = -5,  /* walk: next k-mer missing (kmer_hash.cpp:47-49 throws) */
    KH_ERR_DUPLICATE = -6,  /* insert: key already present (input contract: unique k-mers) */
    KH_ERR_CYCLE = -7,      /* walk: chain longer than the table (no 'F' end) */
    KH_ERR_BAD_BASE = -8,   /* extension byte outside {A,C,G,T,F} */
    KH_ERR_STATE = -9       /* call order (e.g. contigs requested before assemble) */
};

typedef struct kh_table kh_table;

typedef struct kh_stats {
    uint64_t capacity;       /* table slots */
    uint64_t n_inserted;     /* records inserted since create/clear */
    uint64_t n_starts;       /* start k-mers collected (bwd == 'F') or set explicitly */
    uint64_t n_contigs;      /* contigs produced by the last assemble (= n_starts) */
    uint64_t n_lookups;      /* successful walk lookups of the last assemble = sum(len - 1) */
    uint64_t out_bytes;      /* contig text bytes of the last assemble, '\n' included */
    uint64_t n_chunks;       /* 256-base chunks used by the walker */
    uint64_t n_dup, n_full, n_bad_ext, n_missing, n_cycle, n_spin, n_chunk_ovf;
    double ms_insert;        /* device ms, last insert call (table insert + start compaction) */
    double ms_insert_kernel; /* device ms, k_insert alone, last insert call */
    double ms_walk;          /* device ms, k_walk, last assemble */
    double ms_materialize;   /* device ms, offsets scan + contig text, last assemble */
    uint64_t n_bad_base;     /* kh_pack_text_dev lines with a k-mer base outside {A,C,G,T} */
    double ms_build;         /* device ms, region build + overflow inserts of the last partitioned insert */
    double ms_walk_kernel;   /* device ms, k_walk_q alone, last assemble */
    uint64_t n_hot_regions;  /* placement regions remapped (shared minimizers overfilled them): keys by (minimizer, neighbour window) */
    uint64_t n_overflow;     /* keys of the last partitioned build inserted by global CAS (full windows,
                                probe runs that left their region slice) */
    uint64_t n_spread_regions; /* remap targets the remap itself overfilled (a family sharing its
                                  neighbour window too): their remapped keys placed by key hash */
} kh_stats;

/* ---- sizes / info --------------------------------------------------------------------------*/
int kh_abi_version(void);
/* Device bytes the library's buffers hold now in this process (every table) and their high-water
 * mark since the last reset (reset_peak != 0 restarts it at `now` after reading). */
int kh_device_bytes(uint64_t* now, uint64_t* peak, int reset_peak);
int kh_packed_size(int k);   /* sizeof(pkmer_t)   */
int kh_record_size(int k);   /* sizeof(kmer_pair) */
const char* kh_last_error(void);
int kh_device_count(int* n);

/* ---- table lifetime --------------------------------------------------------------------------
 * Capacity = ceil(n_kmers / load_factor) slots (kmer_hash.cpp:108-109 uses load 0.5 -> 2n).
 * Device memory: capacity * (8 B if k <= 29 else 16 B) for the table, plus walker buffers.
 * All work is enqueued on the table's stream (its own, or one set with kh_set_stream). */
int kh_create(kh_table** out, int k, uint64_t n_kmers, double load_factor, int device);
int kh_destroy(kh_table* t);
int kh_clear(kh_table* t);                       /* empty table + start list (async) */
/* Grow an empty table (after create or clear) to hold n_kmers at the creation load factor; a
 * no-op when it already does. The sharded path sizes each shard from the routed counts. */
int kh_reserve(kh_table* t, uint64_t n_kmers);
int kh_set_stream(kh_table* t, void* hip_stream); /* NULL = back to the table's own stream */
int kh_sync(kh_table* t);                        /* wait for the stream; report device errors */
uint64_t kh_capacity(const kh_table* t);
/* blocking host waits on the table's stream so far (device -> host reads of counts, syncs):
 * hosts count the round trips of a sharded step with it (tests/test_gpu_dist.py) */
int kh_host_syncs(const kh_table* t, uint64_t* n);
int kh_get_stats(kh_table* t, kh_stats* out);    /* syncs */

/* ---- insert: records in kmer_pair layout. Start k-mers (bwd == 'F') of every batch are appended
 * to the table's start list in record order (kmer_hash.cpp:27-31). --------------------------*/
int kh_insert(kh_table* t, const uint8_t* host_recs, uint64_t n);   /* synchronous */
int kh_insert_dev(kh_table* t, const void* dev_recs, uint64_t n);   /* async, 16-B aligned */

/* ---- find: keys in pkmer_t layout; out gets kmer_pair records, found[i] = 0/1 ----------------*/
int kh_find(kh_table* t, const uint8_t* host_keys, uint64_t n, uint8_t* host_recs_out,
            uint8_t* host_found);
int kh_find_dev(kh_table* t, const void* dev_keys, uint64_t n, void* dev_recs_out,
                void* dev_found);

/* ---- assemble --------------------------------------------------------------------------------
 * Walks every start k-mer (collected by the inserts, or replaced by kh_set_starts) until its
 * forward extension is 'F', producing the contig text in start-node order on the device. */
int kh_set_starts(kh_table* t, const uint8_t* host_start_recs, uint64_t n);
int kh_assemble_dev(kh_table* t);                 /* async */
int kh_assemble(kh_table* t, uint64_t* n_contigs, uint64_t* out_bytes);  /* sync + checks */
int kh_contigs_text(kh_table* t, char* host_out, uint64_t cap);          /* D2H of the text */
int kh_contigs_text_dev(kh_table* t, const char** dev_text, uint64_t* bytes);
int kh_contigs_offsets(kh_table* t, uint64_t* host_offsets, uint64_t n); /* line starts */

/* ---- sharded multi-GPU path --------------------------------------------------------------------
 * One table per rank (GPU). The key space is split by an owner hash; the caller moves the buffers
 * between ranks (RCCL all-to-all over xGMI: include/cs267_hw3_amd/dist_hash_map.hpp, cs267_hw3_amd/dist.py). Replaces the per-owner batched
 * insert RPCs (hash_map.hpp:38-46,64-77) and the per-step remote find RPCs (hash_map.hpp:94-100).
 * Routed records and query keys are kh_word_count(k) 64-bit words each. counts_out receives
 * nranks + 1 uint64 on the device: per-destination counts, then their total. All async. */
int kh_word_count(int k);
/* Rank (0..nranks-1) owning a pkmer_t key under the table's sharding (the route and the walk use
 * the same function); < 0 on a bad argument. Replaces hash_map.hpp:28-30 get_target_rank. */
int kh_key_owner(const kh_table* t, const uint8_t* packed_key, int nranks);
int kh_collect_starts_dev(kh_table* t, const void* dev_recs, uint64_t n); /* local start k-mers */
/* read_kmers.hpp:62-76 on the GPU: len bytes of fixed-width "KMER BF\n" lines (k+4 bytes each)
 * in device memory -> *n_out = len / (k+4) kmer_pair records at dev_recs (16-byte aligned; NULL:
 * count only), on the table's stream. A line whose k-mer has a base outside {A,C,G,T} makes the
 * next kh_sync fail with KH_ERR_BAD_BASE (the host kh_pack_text fails at once). */
int kh_pack_text_dev(kh_table* t, const void* dev_text, uint64_t len, void* dev_recs, uint64_t* n_out);
int kh_route_dev(kh_table* t, const void* dev_recs, uint64_t n, int nranks, void* dev_words_out,
                 void* dev_counts_out);
/* kh_collect_starts_dev + kh_route_dev in one streaming pass over the records (the start bits
 * come from the route's owner pass); successive calls append starts in call order. */
int kh_route_starts_dev(kh_table* t, const void* dev_recs, uint64_t n, int nranks, void* dev_words_out,
                        void* dev_counts_out);
/* kh_route_starts_dev in ONE pass over the records (no owner pre-pass): owner q's words land in
 * the window dev_words_out + q * win words-per-k-mer (win >= n, < 2^32: a window holds every record,
 * whatever the skew), dev_counts_out[q] = their count, [nranks] = n. The all-to-all sends each
 * window's first counts[q] words. Records of <= 15 bytes (k <= 52; KH_ERR_ARG otherwise: use
 * kh_route_starts_dev). Replaces the same hash_map.hpp:28-30,64-77 routing. */
int kh_route_starts_win_dev(kh_table* t, const void* dev_recs, uint64_t n, int nranks, void* dev_words_out,
                            uint64_t win, void* dev_counts_out);
/* dev_words: internal words as kh_route_dev / kh_route_starts_dev emit them (they carry the
 * k-mer's placement bits: minimizer window, order bits). */
int kh_insert_words_dev(kh_table* t, const void* dev_words, uint64_t m);
/* Staged insert of routed words (one call per received all-to-all chunk, hash_map.hpp:55-80's
 * insert_all split so that partitioning overlaps the exchange): stage partitions m words toward
 * one build of at most total_hint words (the first stage after a clear/finish starts it; keep
 * total_hint the same for every stage of one build); finish builds the table from them. Small
 * builds insert each stage directly. dev_words may be reused once the next stage/finish call
 * has been issued on the table's stream. */
int kh_insert_words_stage_dev(kh_table* t, const void* dev_words, uint64_t m, uint64_t total_hint);
int kh_insert_words_finish(kh_table* t);
/* Splitter k-mers routed to each owner since the last clear (async copy of nranks uint64 into
 * device memory): a shard's splitter count is the sum of its column over the senders, learnt with
 * the route counts instead of by a device read. */
int kh_route_splitters_dev(kh_table* t, void* dev_out, int nranks);
/* Async copy of {start k-mers collected, splitter k-mers collected} (2 uint64) into device memory,
 * for hosts that read them together with their own counts (one host round trip). */
int kh_counters_dev(kh_table* t, void* dev_out);
/* The same two counts read on the host (blocking). After kh_insert_dev they come from the copy
 * made beside the region build, so the read waits for the start / splitter compaction, not for the
 * build (the one-rank sharded step reads them without idling the device). */
int kh_counters(kh_table* t, uint64_t* out2);
/* Migrating-walker rounds. The table is sharded by a hash of each k-mer's minimizer, so
 * consecutive k-mers of a contig mostly share an owner; a walker walks the local shard until its
 * next k-mer is owned elsewhere and is then sent there. Nothing below reads the device on the host:
 *   begin(n_starts, n_splitters, total_walkers)
 *   loop { round(in slots -> out slots, live) -> all-to-all of the fixed-size slot buffers }
 *          (every few rounds the host reads the global sum of live[0]; rounds past the end find
 *           empty slots and do nothing)
 *   -> text_dev (text records grouped by origin rank, counts[P+1]) -> exchange -> end_dev(records)
 * A round's exchange buffer is nranks slots of KH_SLOT_WORDS(cap) int64 words: [count, 0, up to
 * cap messages of KH_MSG_WORDS]; slot q goes to rank q and the received buffer (slot q = what rank q
 * sent) is the next round's input. Messages past cap are held back on the sender and go out in a
 * later round. live: 2 uint64 on the device = [messages in flight after the round (sent + held
 * back), largest per-destination count]. The first round takes in_slots = NULL (the walkers of
 * begin). n_starts / n_splitters: this rank's counts (kh_counters_dev, or the column sums of
 * kh_route_splitters_dev); total_walkers: the sum of n_starts + n_splitters over all ranks.
 * Routing by minimizer must also be used for the inserts: this sharding and the routes agree. */
#define KH_MSG_WORDS 5
#define KH_TEXT_REC_WORDS 2
#define KH_SLOT_WORDS(cap) (2 + (cap) * KH_MSG_WORDS)
int kh_mwalk_begin(kh_table* t, int nranks, int rank, uint64_t total_kmers, uint64_t n_starts, uint64_t n_splitters,
                   uint64_t total_walkers, uint64_t* n_walkers);
int kh_mwalk_round_dev(kh_table* t, const void* dev_in_slots, uint64_t in_cap, void* dev_out_slots, uint64_t out_cap,
                       void* dev_live);
int kh_mwalk_text_bound(kh_table* t, uint64_t* n_records); /* text_dev writes at most this many */
int kh_mwalk_text_dev(kh_table* t, void* dev_out, void* dev_counts_out);
int kh_mwalk_end_dev(kh_table* t, const void* dev_recs, uint64_t n);
/* Splitter segments of the migrating walk (kh_mseg.hip; on when the shard collects splitters,
 * KH_SPLIT_BITS=0 turns them off). kh_mwalk_begin then also seeds a walker at every splitter
 * k-mer this shard owns (n_walkers includes them) and walkers stop before splitters. When
 * kh_mwalk_segments reports > 0 on any rank, after the text records have come home the end of the
 * walk is, instead of kh_mwalk_end_dev:
 *   kh_mwalk_link_dev(recs)  -> KH_LINK_WORDS-word links grouped by owner -> exchange
 *   kh_mwalk_pred_dev(links, preds, stride) -> this rank's table of {predecessor id, length} for
 *        its splitter segments (stride >= every rank's kh_mwalk_segments entries; the tail is "none")
 *   all-gather of the tables (rank q's at q * stride) -> kh_mwalk_resolve_dev(all, stride): every
 *        segment's contig and offset by pointer jumping on the device (no exchange per step)
 *   kh_mwalk_retag_dev(recs) -> KH_SEG_REC_WORDS-word records grouped by contig origin -> exchange
 *   kh_mwalk_end_seg_dev(recs, received segment records)   (this rank's test_<rank>.dat in HBM)
 * Buffers: links <= n_walkers records, preds 2 * stride words, retag output <= n + segments. */
#define KH_LINK_WORDS 4
#define KH_PRED_WORDS 2
#define KH_SEG_REC_WORDS 3
int kh_mwalk_segments(kh_table* t, uint64_t* n_splitter_segments);
/* Malformed input whose start walks overlap (a k-mer reached by two walks): a segmented walk
 * cannot give one splitter segment two contigs, and an unsegmented one may outgrow its text store.
 * kh_mwalk_flags_dev writes 2 uint64 to device memory (async): [overlap / overflow reports of this
 * walk, text records the store needed]; hosts exchange the first with a count exchange they make
 * anyway, and when any rank reports one, every rank calls kh_mwalk_redo (ends this walk, clears the
 * report) and walks again from kh_mwalk_begin: without splitter segments (each start walked to its
 * end, as kmer_hash.cpp:41-53 does) and with a store of at least store_records records. */
int kh_mwalk_flags_dev(kh_table* t, void* dev_out2);
int kh_mwalk_redo(kh_table* t, uint64_t store_records);
/* Short walk first (round 6): splitter segments only pay for long contigs. Called before
 * kh_mwalk_begin with every rank's k-mer and start counts: where the mean contig is shorter than
 * the splitter spacing, *armed = 1 and the next walk runs without splitter segments; a walker that
 * passes 4 spacings ends and adds 2^40 to the first word kh_mwalk_flags_dev reports. When any rank
 * reports it, every rank calls kh_mwalk_abandon and walks again from kh_mwalk_begin, segmented
 * (hosts keep walking segmented on the same input). */
int kh_mwalk_short(kh_table* t, uint64_t total_kmers, uint64_t total_starts, int* armed);
int kh_mwalk_abandon(kh_table* t);
int kh_mwalk_link_dev(kh_table* t, const void* dev_recs, uint64_t n, void* dev_links_out, void* dev_counts_out);
int kh_mwalk_pred_dev(kh_table* t, const void* dev_links, uint64_t m, void* dev_preds_out, uint64_t stride);
int kh_mwalk_resolve_dev(kh_table* t, const void* dev_all_preds, uint64_t stride);
int kh_mwalk_retag_dev(kh_table* t, const void* dev_recs, uint64_t n, void* dev_seg_recs_out, void* dev_counts_out);
int kh_mwalk_end_seg_dev(kh_table* t, const void* dev_recs, uint64_t n, const void* dev_seg_recs, uint64_t m);

/* ---- device memory helpers (for hosts without an allocator of their own) --------------------*/
int kh_dev_malloc(void** p, uint64_t bytes, int device);
int kh_dev_free(void* p);
int kh_memcpy_htod(void* dst, const void* src, uint64_t bytes);
int kh_memcpy_dtoh(void* dst, const void* src, uint64_t bytes);

/* ---- host codec helpers --------------------------------------------------------------------*/
/* read_kmers.hpp:62-76: fixed-width "KMER BF\n" lines (k+4 bytes) -> kmer_pair records. */
int kh_pack_text(int k, const char* text, uint64_t len, uint8_t* recs_out, uint64_t* n_out);
/* packing.hpp:77-107 */
int kh_pack_kmer(int k, const char* kmer, uint8_t* packed_out);
int kh_unpack_kmer(int k, const uint8_t* packed, char* kmer_out);
/* pkmer_t.hpp:31-37 djb2 (API parity; the table places keys with its own mixer) */
uint64_t kh_djb2(int k, const uint8_t* packed);
/* kmer_t.hpp:51-53 next_kmer of a record, as packed bytes */
int kh_next_kmer(int k, const uint8_t* rec, uint8_t* packed_out);

/* ---- synthetic dataset generator ------------------------------------------
 * n k-mers cut from independent uniform-random contigs of len_min..len_max k-mers (plus
 * single_permille / 1000 single-k-mer contigs), every k-mer unique (contigs containing a repeated
 * k-mer are re-drawn), records shuffled by a seeded bijection. Deterministic in all arguments
 * except `threads`. */
typedef struct kh_gen kh_gen;
int kh_gen_create(kh_gen** out, int k, uint64_t n, uint32_t len_min, uint32_t len_max,
                  uint32_t single_permille, uint64_t seed, int shuffle, int threads);
/* C5-style skewed set (BASELINE configs[4]): the first n_long contigs have long_len
 * k-mers, the rest U[len_min, len_max]; front_starts != 0 puts every start k-mer ahead of every
 * other record (so the block split hands all walkers to the first ranks). */
int kh_gen_create_skewed(kh_gen** out, int k, uint64_t n, uint32_t len_min, uint32_t len_max,
                         uint32_t single_permille, uint64_t seed, int shuffle, int threads, uint32_t n_long,
                         uint32_t long_len, int front_starts);
/* Hot-minimizer / hot-bucket variant (BASELINE configs[4] "skewed/hot-bucket"): additionally,
 * hot_permille / 1000 of the contigs (picked by a seeded hash) carry one of n_motifs (1..64) shared
 * M-mers (M = the table's minimizer length: 16 at k >= 31, 12 at k = 19) every K - M + 1 bases, so
 * every k-mer of a hot contig contains one and the motifs (chosen for the smallest minimizer order)
 * are their minimizers: all k-mers of motif h share one minimizer window, hence one placement
 * region and one shard owner before the table's hot-region remap. Uniqueness and the ground
 * truth hold as for kh_gen_create. hot_permille = 0 is kh_gen_create_skewed. */
int kh_gen_create_hot(kh_gen** out, int k, uint64_t n, uint32_t len_min, uint32_t len_max,
                      uint32_t single_permille, uint64_t seed, int shuffle, int threads, uint32_t n_long,
                      uint32_t long_len, int front_starts, uint32_t hot_permille, uint32_t n_motifs);
/* flags: KH_GEN_HOT_FLANK plants a fixed per-motif M-mer right before every motif occurrence (one
 * flank + motif pattern per K bases, k >= 2M + 8): the k-mers holding the whole pattern (20 of 51
 * phases at k=51) share the minimizer and its neighbour window, the worst case of the table's hot
 * remap (a long exact repeat shared by a family). */
#define KH_GEN_HOT_FLANK 1u
int kh_gen_create_hot_ex(kh_gen** out, int k, uint64_t n, uint32_t len_min, uint32_t len_max,
                         uint32_t single_permille, uint64_t seed, int shuffle, int threads, uint32_t n_long,
                         uint32_t long_len, int front_starts, uint32_t hot_permille, uint32_t n_motifs,
                         uint32_t flags);
int kh_gen_destroy(kh_gen* g);
uint64_t kh_gen_num_contigs(const kh_gen* g);
/* records at output positions [pos_begin, pos_end) in kmer_pair layout (block split of
 * read_kmers.hpp:55-58 = positions [r*ceil(n/P), ...)) */
int kh_gen_records(const kh_gen* g, uint64_t pos_begin, uint64_t pos_end, uint8_t* out);
/* the same records produced by the GPU into device memory (R bytes each, contiguous) on a HIP
 * stream (NULL = default stream): a 200M-record C3 set in milliseconds instead of seconds of host
 * work and a PCIe upload. Async; the generator must outlive the work. */
int kh_gen_records_dev(kh_gen* g, uint64_t pos_begin, uint64_t pos_end, void* dev_out, void* hip_stream);
/* ground-truth contig text of the contigs whose start k-mer lies in [pos_begin, pos_end), in
 * start-node order (= expected test_<rank>.dat bytes); bytes_out gets the size. out may be NULL
 * to query the size. */
int kh_gen_truth(const kh_gen* g, uint64_t pos_begin, uint64_t pos_end, char* out, uint64_t cap,
                 uint64_t* bytes_out);

#ifdef __cplusplus
}
#endif
#endif /* KMER_HASH_AMD_H */
