// dist_hash_map.hpp — the sharded table behind DistributedHashMap(size, rank, world) for world > 1
// (hash_map.hpp:12-114 + kmer_hash.cpp:21-55 of the reference), C++ host over the C ABI.
//
// One rank per GPU (or P logical ranks on one GPU for tests), SPMD: every rank calls the same
// collective methods in the same order. The reference's transport (UPC++ RPCs: one batched insert
// RPC per owner, hash_map.hpp:38-46,64-77; one blocking find RPC per remote walk step,
// hash_map.hpp:94-100) becomes bulk exchanges through a kh::Comm (comm.hpp / rccl_comm.hpp):
//
//   insert_all  route every record to its owner on the GPU in one pass into per-owner windows
//               (kh_route_starts_win_dev; the block's start k-mers are collected in the same pass,
//               kmer_hash.cpp:27-31) -> one device all-gather of the counts, read once -> each shard
//               sized from what it receives (kh_reserve) -> all-to-all of the routed words in
//               chunks, each received chunk partitioned while the next is on the wire
//               (kh_insert_words_stage_dev), one region build at the end (kh_insert_words_finish).
//               One rank: the records go straight into the single-GPU records pass.
//   assemble    migrating walkers (kh_mwalk_*): a walker walks the local shard until its next
//               k-mer is owned elsewhere, then moves there in the round's all-to-all of fixed-size
//               slots (no host read per round; the end is checked where the last walk ended); the
//               bases go home in one more all-to-all; splitter segments (long chains) are ranked on
//               the device from an all-gathered predecessor table. Each rank ends with its
//               test_<rank>.dat bytes. A step reads the device at most 8 times (host_syncs()).
//   find        the owner's table answers (the RPC of hash_map.hpp:94-100): ranks that are threads
//               of one process (a peer group) look the owner's table up directly; otherwise every
//               find() is one collective round (all ranks' queries gathered, each owner answers its
//               own, answers gathered), and barrier()/process_requests() keep answering rounds until
//               every rank has reached them -- the UPC++ progress the reference's barrier makes
//               (kmer_hash.cpp:136, hash_map.hpp:110-113) while other ranks still walk
//
// The same protocol has a Python host in cs267_hw3_amd/dist.py (torch.distributed).
#pragma once
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../kmer_hash_amd.h"
#include "comm.hpp"

namespace kh {

inline void abi_check(int rc) {
    if (rc != KH_OK) throw std::runtime_error(kh_last_error());
}

// Grow-only device buffer (25 % headroom when it grows).
class DevBuf {
public:
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void* ensure(size_t bytes) {
        if (bytes <= cap_ && p_) return p_;
        release();
        const size_t want = bytes + bytes / 4 + 256;
        hip_check(hipMalloc(&p_, want), "hipMalloc");
        cap_ = want;
        return p_;
    }
    int64_t* words(size_t n) { return static_cast<int64_t*>(ensure(n * 8)); }
    void* get() const { return p_; }
    size_t capacity() const { return cap_; }
    void release() {
        if (p_) (void)hipFree(p_);
        p_ = nullptr;
        cap_ = 0;
    }

private:
    void* p_ = nullptr;
    size_t cap_ = 0;
};

class ShardedTable;

// The ranks this process drives (one thread each), set by the launcher before the threads start,
// like upcxx::init(): DistributedHashMap(size, rank, world) looks its rank up here.
struct RankContext {
    Comm* comm = nullptr;
    int device = 0;
    const void* peer_group = nullptr;  // in-process peers (owner-side finds); null: none
};
inline std::vector<RankContext>& rank_contexts() {
    static std::vector<RankContext> v;
    return v;
}

// In-process peers of a communicator group (threads of one process), for owner-side finds.
class PeerRegistry {
public:
    static PeerRegistry& get() {
        static PeerRegistry r;
        return r;
    }
    void add(const void* group, int world, int rank, ShardedTable* t) {
        std::lock_guard<std::mutex> g(m_);
        auto& v = peers_[group];
        if ((int)v.size() < world) v.resize(world, nullptr);
        v[rank] = t;
    }
    void remove(const void* group, int rank) {
        std::lock_guard<std::mutex> g(m_);
        auto it = peers_.find(group);
        if (it == peers_.end()) return;
        it->second[rank] = nullptr;
        if (std::all_of(it->second.begin(), it->second.end(), [](ShardedTable* x) { return !x; })) peers_.erase(it);
    }
    ShardedTable* peer(const void* group, int rank) {
        std::lock_guard<std::mutex> g(m_);
        auto it = peers_.find(group);
        return it == peers_.end() || rank >= (int)it->second.size() ? nullptr : it->second[rank];
    }
    // f(peer) with the registry locked, so the peer cannot be destroyed (remove) meanwhile
    template <class F>
    bool with_peer(const void* group, int rank, F f) {
        std::lock_guard<std::mutex> g(m_);
        auto it = peers_.find(group);
        ShardedTable* t = it == peers_.end() || rank >= (int)it->second.size() ? nullptr : it->second[rank];
        if (!t) return false;
        f(t);
        return true;
    }

private:
    std::mutex m_;
    std::map<const void*, std::vector<ShardedTable*>> peers_;
};

class ShardedTable {
public:
    // n_kmers_hint: k-mers this shard is expected to hold (it grows to what it is routed)
    ShardedTable(int k, uint64_t n_kmers_hint, Comm& comm, int device, const void* peer_group = nullptr)
        : k_(k), comm_(comm), P_(comm.size()), rank_(comm.rank()), device_(device), group_(peer_group) {
        hip_check(hipSetDevice(device), "hipSetDevice");
        abi_check(kh_create(&t_, k, n_kmers_hint ? n_kmers_hint : 1, 0.5, device));
        hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
        hip_check(hipStreamCreateWithFlags(&xstream_, hipStreamNonBlocking), "hipStreamCreate");
        abi_check(kh_set_stream(t_, stream_));
        W_ = kh_word_count(k);
        R_ = kh_record_size(k);
        counts_.words(P_ + 1);
        if (group_) PeerRegistry::get().add(group_, P_, rank_, this);
    }
    ~ShardedTable() {
        if (group_) PeerRegistry::get().remove(group_, rank_);
        (void)hipSetDevice(device_);
        if (t_) kh_destroy(t_);
        for (auto* b : {&words_, &recv_, &counts_, &tout_, &trecv_, &lout_, &lin_, &qout_, &qin_, &sout_, &sin_,
                        &recs_, &pack_, &gather_, &live_, &slots_[0], &slots_[1], &recv_slots_[0], &recv_slots_[1]})
            b->release();
        for (auto e : events_) (void)hipEventDestroy(e);
        if (stream_) (void)hipStreamDestroy(stream_);
        if (xstream_) (void)hipStreamDestroy(xstream_);
    }
    ShardedTable(const ShardedTable&) = delete;
    ShardedTable& operator=(const ShardedTable&) = delete;

    kh_table* handle() { return t_; }
    hipStream_t stream() { return stream_; }
    int rank() const { return rank_; }
    int world() const { return P_; }
    int rounds() const { return rounds_; }
    int checks() const { return checks_; }
    // blocking device reads so far: this host's (count exchanges, walk checks) + the library's
    uint64_t host_syncs() const {
        uint64_t lib = 0;
        (void)kh_host_syncs(t_, &lib);
        return syncs_ + lib;
    }
    // tests: slots of at most this many messages (the rest is held back on the sender)
    void set_slot_cap_max(uint64_t c) { slot_cap_max_ = c ? c : 1; }
    std::mutex& mutex() { return m_; }

    void clear() {
        hip_check(hipSetDevice(device_), "hipSetDevice");
        abi_check(kh_clear(t_));
        inserted_ = 0;
    }

    // hash_map.hpp:55-80 insert_all (+ kmer_hash.cpp:27-31 start nodes) for this rank's block of
    // records (host kmer_pair array, R bytes each). Collective. Returns the k-mers this shard got.
    uint64_t insert_all(const void* host_recs, uint64_t n) {
        hip_check(hipSetDevice(device_), "hipSetDevice");
        void* d = recs_.ensure(n * R_ + 16);
        if (n) hip_check(hipMemcpyAsync(d, host_recs, n * R_, hipMemcpyHostToDevice, stream_), "hipMemcpyAsync");
        return insert_all_dev(d, n);
    }

    // Same with the records already in device memory (16-B aligned). Collective.
    uint64_t insert_all_dev(const void* dev_recs, uint64_t n) {
        hip_check(hipSetDevice(device_), "hipSetDevice");
        const uint64_t P = (uint64_t)P_;
        if (P == 1 && !route_one_rank()) {
            // one rank: every key is this shard's and nothing moves, so the records go straight
            // into the single-GPU records pass (start k-mers and splitters in the same pass)
            const int rc = kh_reserve(t_, inserted_ + n);
            if (rc != KH_OK) abi_check(rc);
            abi_check(kh_insert_dev(t_, dev_recs, n));
            inserted_ += n;
            err_.clear();
            uint64_t hv[2];
            abi_check(kh_counters(t_, hv));  // the walk's start / splitter counts (waits for the copy
                                             // made beside the build, not for the build)
            ns_ = hv[0];
            nsp_ = splitters_ = hv[1];
            walkers_ = ns_ + nsp_;
            return done_insert(n);
        }
        uint64_t nch = 1;
        if (P > 1 && n >= kPipelineMin) {
            // per-peer bytes of a chunk <= chunk records * W * 8: every message stays under the
            // transport's per-peer limit whatever the skew
            const uint64_t lim = (512ull << 20);
            nch = std::max<uint64_t>(kInsertChunks, (n * W_ * 8 + lim - 1) / lim);
        }
        std::vector<uint64_t> bounds(nch + 1);
        // chunk starts at multiples of 16 records: every chunk's records stay 16-B aligned
        for (uint64_t c = 0; c < nch; ++c) bounds[c] = std::min<uint64_t>(n, (n * c / nch) & ~15ull);
        bounds[nch] = n;
        // one-pass route (kh_route_starts_win_dev): chunk c's records sorted into P owner windows of
        // (c1 - c0) words each at P * c0 words, while the P windows of the block fit a third of the
        // free device memory; else the two-pass route packs each chunk back to back
        size_t free_b = 0, total_b = 0;
        hip_check(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
        const uint64_t win_bytes = P * std::max<uint64_t>(n, 1) * W_ * 8;
        const bool windows = R_ <= 15 && win_bytes <= words_.capacity() + free_b / (3 * ranks_per_device());
        int64_t* words = windows ? words_.words(P * std::max<uint64_t>(n, 1) * W_)
                                 : words_.words(std::max<uint64_t>(n, 1) * W_);
        int64_t* cnt = counts_.words(nch * (P + 1));
        const uint8_t* recs = static_cast<const uint8_t*>(dev_recs);
        auto win_of = [&](uint64_t c) { return std::max<uint64_t>(bounds[c + 1] - bounds[c], 1); };
        for (uint64_t c = 0; c < nch; ++c) {
            if (windows)
                abi_check(kh_route_starts_win_dev(t_, recs + bounds[c] * R_, bounds[c + 1] - bounds[c], P_,
                                                  words + P * bounds[c] * W_, win_of(c), cnt + c * (P + 1)));
            else
                abi_check(kh_route_starts_dev(t_, recs + bounds[c] * R_, bounds[c + 1] - bounds[c], P_,
                                              words + bounds[c] * W_, cnt + c * (P + 1)));
        }
        // every rank learns the whole [src][chunk][dst] count matrix, the splitters each rank
        // routed to each owner and every rank's start count in one device all-gather, read once
        const uint64_t row = nch * (P + 1) + P + 1;
        int64_t* pk = pack_.words(row * (P + 1));
        hip_check(hipMemcpyAsync(pk, cnt, nch * (P + 1) * 8, hipMemcpyDeviceToDevice, stream_), "hipMemcpyAsync");
        abi_check(kh_route_splitters_dev(t_, pk + nch * (P + 1), P_));
        int64_t* ctr2 = pk + row * P;  // scratch for {starts, splitters collected}
        abi_check(kh_counters_dev(t_, ctr2));
        hip_check(hipMemcpyAsync(pk + nch * (P + 1) + P, ctr2, 8, hipMemcpyDeviceToDevice, stream_), "hipMemcpyAsync");
        int64_t* allp = gather_.words(row * P);
        comm_.allgather_dev(pk, row, allp, stream_);
        std::vector<uint64_t> all(row * P);
        read_host(all.data(), allp, row * P);
        auto M = [&](uint64_t src, uint64_t c, uint64_t dst) { return all[src * row + c * (P + 1) + dst]; };
        auto SPL = [&](uint64_t src, uint64_t dst) { return all[src * row + nch * (P + 1) + dst]; };
        uint64_t m = 0, gmax = 0;
        ns_ = all[(uint64_t)rank_ * row + nch * (P + 1) + P];
        nsp_ = walkers_ = splitters_ = 0;
        for (uint64_t q = 0; q < P; ++q) {
            nsp_ += SPL(q, rank_);
            walkers_ += all[q * row + nch * (P + 1) + P];
            for (uint64_t d = 0; d < P; ++d) splitters_ += SPL(q, d);
            for (uint64_t c = 0; c < nch; ++c) {
                m += M(q, c, rank_);
                for (uint64_t d = 0; d < P; ++d) gmax = std::max(gmax, M(q, c, d));
            }
        }
        walkers_ += splitters_;
        // size the shard from what it holds after this insert (a non-empty shard cannot grow:
        // kh_reserve fails); a rank that cannot still takes part in every exchange, sends no
        // walkers, and every rank raises together at the walk's first check
        const int rc = kh_reserve(t_, inserted_ + m);
        err_ = rc == KH_OK ? "" : kh_last_error();
        const bool ok = rc == KH_OK;
        inserted_ += m;
        if (P == 1) {  // one rank routed anyway (KH_DIST_ROUTE_ONE_RANK=1; one chunk): the words are this shard's
            if (ok) abi_check(kh_insert_words_dev(t_, words, m));
            return done_insert(m);
        }
        int64_t* recv = recv_.words(std::max<uint64_t>(m, 1) * W_);
        std::vector<uint64_t> sc(P), sd(P), rcn(P), rd(P);
        auto plan = [&](uint64_t c, uint64_t pos) {  // chunk c's counts/displacements, in words
            uint64_t so = bounds[c] * W_, ro = pos * W_;
            for (uint64_t q = 0; q < P; ++q) {
                sc[q] = M(rank_, c, q) * W_;
                sd[q] = windows ? (P * bounds[c] + q * win_of(c)) * W_ : so;  // owner window / packed
                so += sc[q];
                rcn[q] = M(q, c, rank_) * W_;
                rd[q] = ro;
                ro += rcn[q];
            }
        };
        if (nch == 1) {
            plan(0, 0);
            comm_.alltoallv(words, sc.data(), sd.data(), recv, rcn.data(), rd.data(), gmax * W_, stream_);
            if (ok) abi_check(kh_insert_words_dev(t_, recv, m));
            return done_insert(m);
        }
        // chunk c moves on the exchange stream while chunk c-1, received, is partitioned on the
        // table's stream; one build at the end
        ensure_events(nch + 1);
        hip_check(hipEventRecord(events_[nch], stream_), "hipEventRecord");  // routed words ready
        hip_check(hipStreamWaitEvent(xstream_, events_[nch], 0), "hipStreamWaitEvent");
        uint64_t pos = 0, prev_pos = 0, prev_m = 0;
        for (uint64_t c = 0; c < nch; ++c) {
            uint64_t mc = 0;
            for (uint64_t q = 0; q < P; ++q) mc += M(q, c, rank_);
            plan(c, pos);
            comm_.alltoallv(words, sc.data(), sd.data(), recv, rcn.data(), rd.data(), gmax * W_, xstream_);
            hip_check(hipEventRecord(events_[c], xstream_), "hipEventRecord");
            if (c > 0 && ok) stage(recv, prev_pos, prev_m, m, events_[c - 1]);
            prev_pos = pos;
            prev_m = mc;
            pos += mc;
        }
        if (ok) {
            stage(recv, prev_pos, prev_m, m, events_[nch - 1]);
            abi_check(kh_insert_words_finish(t_));
        } else {
            hip_check(hipStreamWaitEvent(stream_, events_[nch - 1], 0), "hipStreamWaitEvent");
        }
        return done_insert(m);
    }

    // kmer_hash.cpp:38-55 assemble_contigs for this rank's start k-mers, every rank at once.
    // total_kmers bounds contig length (cycle detection). Collective. Returns walk rounds.
    // Rounds exchange fixed-size slots (KH_SLOT_WORDS): no host read per round; the host reads
    // the global in-flight count first where the last walk ended, then every kCheckEvery rounds.
    int assemble(uint64_t total_kmers) {
        hip_check(hipSetDevice(device_), "hipSetDevice");
        constexpr uint64_t T = KH_TEXT_REC_WORDS;
        const uint64_t P = (uint64_t)P_;
        const bool failed = !err_.empty();  // this shard could not be sized: it sends no walkers
        uint64_t n_in = 0;
        if (!failed) abi_check(kh_mwalk_begin(t_, P_, rank_, total_kmers, ns_, nsp_, walkers_, &n_in));
        rounds_ = checks_ = 0;
        const int64_t* in = nullptr;
        uint64_t cap_in = 0;
        // caps learnt from a walk of another walker count describe another input: start over
        if (caps_walkers_ != walkers_) {
            caps_.clear();
            rounds_hint_ = 0;
        }
        cap_floor_ = 0;
        int check_at = rounds_hint_ ? rounds_hint_ : kCheckEvery;
        // rounds without splitter segments (KH_SPLIT_BITS=0) grow with the longest chain; a
        // walker advances every round it is not held back, so total_kmers bounds them
        const uint64_t limit = splitters_ ? (uint64_t)kMaxRounds : std::max<uint64_t>(kMaxRounds, total_kmers + kMaxRounds);
        // [in flight, largest per-destination count] of the rounds since the last check
        int64_t* live = live_.words(2 * (uint64_t)std::max(check_at, kCheckEvery) + 2);
        std::vector<uint64_t> maxes, flights, used;
        int base = 0;
        for (;;) {
            const uint64_t cap = slot_cap(rounds_), sw = KH_SLOT_WORDS(cap);
            used.push_back(cap);
            int64_t* out = slots_[rounds_ & 1].words(P * sw);
            int64_t* lv = live + 2 * (rounds_ - base);
            if (failed) {
                hip_check(hipMemset2DAsync(out, sw * 8, 0, 8, P, stream_), "hipMemset2DAsync");
                hip_check(hipMemsetAsync(lv, 0, 16, stream_), "hipMemsetAsync");
            } else {
                abi_check(kh_mwalk_round_dev(t_, in, cap_in, out, cap, lv));
            }
            int64_t* nxt = out;  // one rank: slot 0 is the next round's input
            if (P > 1) {
                nxt = recv_slots_[rounds_ & 1].words(P * sw);
                std::vector<uint64_t> cnt(P, sw), dsp(P);
                for (uint64_t q = 0; q < P; ++q) dsp[q] = q * sw;
                comm_.alltoallv(out, cnt.data(), dsp.data(), nxt, cnt.data(), dsp.data(), sw, stream_);
            }
            in = nxt;
            cap_in = cap;
            ++rounds_;
            if (rounds_ >= check_at || (uint64_t)rounds_ >= limit) {
                // every rank's window of [in flight, largest per-destination] + errors
                const uint64_t nw = 2 * (uint64_t)(rounds_ - base), w = nw + 1;
                int64_t* mine = pack_.words(w);
                hip_check(hipMemcpyAsync(mine, live, nw * 8, hipMemcpyDeviceToDevice, stream_), "hipMemcpyAsync");
                put_word(mine + w - 1, failed ? 1 : 0);
                int64_t* allg = gather_.words(w * P);
                comm_.allgather_dev(mine, w, allg, stream_);
                std::vector<uint64_t> h(w * P);
                read_host(h.data(), allg, w * P);
                ++checks_;
                std::vector<uint64_t> mx(w, 0);
                for (uint64_t q = 0; q < P; ++q)
                    for (uint64_t i = 0; i < w; ++i) mx[i] = std::max(mx[i], h[q * w + i]);
                if (mx[w - 1]) throw std::runtime_error(failed ? err_ : "another rank failed to size its shard");
                for (uint64_t i = 1; i < nw; i += 2) maxes.push_back(mx[i]);
                for (uint64_t i = 0; i < nw; i += 2) flights.push_back(mx[i]);
                if (mx[nw - 2] == 0) break;
                // a round whose demand passed its slots held messages back: later rounds get
                // slots for that demand, so the surplus drains in a few rounds, not thousands
                for (int r = base; r < rounds_; ++r)
                    if (maxes[r] > used[r]) cap_floor_ = std::max<uint64_t>(cap_floor_, maxes[r] * 5 / 4 + 256);
                if ((uint64_t)rounds_ >= limit) throw std::runtime_error("migrating walk did not end in its round limit");
                base = rounds_;
                check_at = rounds_ + kCheckEvery;
            }
        }
        // the next assemble: slots sized by what each round carried, and its first check at the
        // round after which nothing was in flight (rounds past it are empty)
        caps_.assign(maxes.size(), 0);
        for (size_t r = 0; r < maxes.size(); ++r) caps_[r] = std::max<uint64_t>(256, maxes[r] * 5 / 4 + 256);
        rounds_hint_ = rounds_;
        for (size_t r = 0; r < flights.size(); ++r)
            if (flights[r] == 0) {
                rounds_hint_ = (int)r + 1;
                break;
            }
        caps_walkers_ = walkers_;
        uint64_t tb = 0;
        abi_check(kh_mwalk_text_bound(t_, &tb));
        int64_t* tout = tout_.words(std::max<uint64_t>(tb, 1) * T);
        abi_check(kh_mwalk_text_dev(t_, tout, counts_.words(P + 1)));
        Exchange ex;
        exchange_counts(ex);
        const uint64_t r = ex.recv_total;
        int64_t* trecv = tout;
        if (P > 1) {
            trecv = trecv_.words(std::max<uint64_t>(r, 1) * T);
            move(tout, trecv, ex, T);
        }
        // every rank takes the same branch (a rank without splitters still links and answers)
        if (splitters_)
            segments_end(trecv, r, ns_ + nsp_);
        else
            abi_check(kh_mwalk_end_dev(t_, trecv, r));
        abi_check(kh_sync(t_));
        return rounds_;
    }

    // This rank's contig text (= test_<rank>.dat bytes) of the last assemble.
    std::string contigs_text() {
        hip_check(hipSetDevice(device_), "hipSetDevice");
        const char* d = nullptr;
        uint64_t bytes = 0;
        abi_check(kh_contigs_text_dev(t_, &d, &bytes));
        std::string s(bytes, '\0');
        if (bytes) hip_check(hipMemcpy(&s[0], d, bytes, hipMemcpyDeviceToHost), "hipMemcpy");
        return s;
    }

    // Single-key find (hash_map.hpp:83-107): the owner's table answers. Ranks of a peer group
    // (threads of one process) look the owner's table up directly; without one (one process per
    // GPU) every find() is one collective round, so every rank must keep calling find() or
    // barrier() (process_requests) until all are done, as the reference's own loop does.
    bool find(const uint8_t* packed_key, uint8_t* rec_out) {
        if (!group_ && P_ > 1) return find_round(packed_key, rec_out, false);
        const int owner = kh_key_owner(t_, packed_key, P_);
        if (owner < 0) abi_check(owner);
        int prev = 0;
        hip_check(hipGetDevice(&prev), "hipGetDevice");
        uint8_t found = 0;
        int rc = KH_OK;
        auto look = [&](ShardedTable* o) {
            std::lock_guard<std::mutex> g(o->m_);
            if (hipSetDevice(o->device_) != hipSuccess) rc = KH_ERR_HIP;
            else rc = kh_find(o->t_, packed_key, 1, rec_out, &found);
        };
        bool ok = true;
        if (owner == rank_ || !group_)
            look(this);
        else
            ok = PeerRegistry::get().with_peer(group_, owner, look);  // registry locked: the peer stays
        (void)hipSetDevice(prev);  // the caller's device, whichever table answered
        if (!ok) throw std::runtime_error("DistributedHashMap::find: the owner rank is not in this process");
        abi_check(rc);
        return found != 0;
    }

    // hash_map.hpp:110-113 process_requests (progress + barrier) / upcxx::barrier(): collective.
    // Without a peer group it answers find rounds until every rank has arrived here.
    void barrier() {
        if (!group_ && P_ > 1) {
            while (!find_round(nullptr, nullptr, true)) {
            }
            return;
        }
        comm_.barrier();
    }

    // processes sharing one device (KH_DIST_DEVICE rehearsals) split its free memory
    void set_ranks_per_device(int n) { ranks_per_device_ = n > 0 ? n : 1; }
    uint64_t ranks_per_device() const { return (uint64_t)ranks_per_device_; }

    static constexpr uint64_t kInsertChunks = 4;
    static constexpr int kCheckEvery = 4;
    static constexpr int kMaxRounds = 4096;
    static constexpr uint64_t kPipelineMin = 1ull << 22;  // records per rank below: one transfer

private:
    static bool route_one_rank() {
        const char* e = getenv("KH_DIST_ROUTE_ONE_RANK");
        return e && !strcmp(e, "1");
    }

    // hash_map.hpp:79: insert_all ends in a barrier, so a find() right after it sees every
    // rank's keys (the shard's build has finished before any rank leaves)
    uint64_t done_insert(uint64_t m) {
        abi_check(kh_sync(t_));
        comm_.barrier();
        return m;
    }

    // One collective find round: every rank contributes {flags (1 = query, 2 = done), owner, key}
    // (4 words), each owner answers the queries it owns with one batched kh_find, and the answers
    // {found, record} (4 words per asker) are gathered back. done: this rank only serves (barrier);
    // returns true when every rank was done in this round. Otherwise returns `found` for the query.
    bool find_round(const uint8_t* key, uint8_t* rec_out, bool done) {
        hip_check(hipSetDevice(device_), "hipSetDevice");
        const uint64_t P = (uint64_t)P_, Pk = (uint64_t)((k_ + 3) / 4);
        std::vector<uint64_t> q(4, 0), all(4 * P);
        if (!done) {
            const int owner = kh_key_owner(t_, key, P_);
            if (owner < 0) abi_check(owner);
            q[0] = 1;
            q[1] = (uint64_t)owner;
            std::memcpy(&q[2], key, Pk);
        } else {
            q[0] = 2;
        }
        comm_.allgather(q.data(), 4, all.data(), stream_);
        bool any = false, all_done = true;
        std::vector<uint8_t> keys, recs, found;
        std::vector<int> asker;
        for (uint64_t r = 0; r < P; ++r) {
            const uint64_t* a = &all[4 * r];
            all_done = all_done && (a[0] & 2);
            if (!(a[0] & 1)) continue;
            any = true;
            if (a[1] != (uint64_t)rank_) continue;
            keys.insert(keys.end(), reinterpret_cast<const uint8_t*>(&a[2]), reinterpret_cast<const uint8_t*>(&a[2]) + Pk);
            asker.push_back((int)r);
        }
        if (!any) return all_done;  // nobody asked: every rank sees the same and skips the answers
        std::vector<uint64_t> rep(4 * P, 0), rall(4 * P * P);
        if (!asker.empty()) {
            recs.assign(asker.size() * R_, 0);
            found.assign(asker.size(), 0);
            std::lock_guard<std::mutex> g(m_);
            abi_check(kh_find(t_, keys.data(), asker.size(), recs.data(), found.data()));
            for (size_t i = 0; i < asker.size(); ++i) {
                rep[4 * asker[i]] = found[i];
                std::memcpy(&rep[4 * asker[i] + 1], &recs[i * R_], R_);
            }
        }
        comm_.allgather(rep.data(), 4 * P, rall.data(), stream_);
        if (done) return false;
        const uint64_t* ans = &rall[(q[1] * P + (uint64_t)rank_) * 4];
        std::memcpy(rec_out, &ans[1], R_);
        return ans[0] != 0;
    }

    struct Exchange {
        std::vector<uint64_t> send, recv;  // per peer, in items
        uint64_t send_total = 0, recv_total = 0, total_all = 0, gmax = 0;
        std::vector<uint64_t> extra;       // every rank's extra word
    };

    // counts_ holds [P+1] device words (per destination, total) -> every rank's view, with one
    // extra word of this rank's (e.g. its splitter count): one device all-gather, read once
    void exchange_counts(Exchange& ex, uint64_t extra = 0) {
        const uint64_t P = (uint64_t)P_, w = P + 2;
        int64_t* mine = pack_.words(w);
        hip_check(hipMemcpyAsync(mine, counts_.get(), (P + 1) * 8, hipMemcpyDeviceToDevice, stream_), "hipMemcpyAsync");
        put_word(mine + P + 1, extra);
        int64_t* allg = gather_.words(w * P);
        comm_.allgather_dev(mine, w, allg, stream_);
        std::vector<uint64_t> all(w * P);
        read_host(all.data(), allg, w * P);
        ex.send.assign(P, 0);
        ex.recv.resize(P);
        ex.extra.resize(P);
        ex.send_total = ex.recv_total = ex.total_all = ex.gmax = 0;
        for (uint64_t q = 0; q < P; ++q) {
            ex.send[q] = all[(uint64_t)rank_ * w + q];
            ex.recv[q] = all[q * w + rank_];
            ex.extra[q] = all[q * w + P + 1];
            ex.send_total += ex.send[q];
            ex.recv_total += ex.recv[q];
            ex.total_all += all[q * w + P];
            for (uint64_t d = 0; d < P; ++d) ex.gmax = std::max(ex.gmax, all[q * w + d]);
        }
    }

    // one blocking device -> host read (counted: host_syncs())
    void read_host(void* dst, const void* dev, uint64_t words) {
        hip_check(hipMemcpyAsync(dst, dev, words * 8, hipMemcpyDeviceToHost, stream_), "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
        ++syncs_;
    }

    uint64_t slot_cap(int r) const {
        uint64_t c;
        if (r < (int)caps_.size())
            c = caps_[r];
        else if (!caps_.empty())
            c = caps_.back();
        else {
            const uint64_t P = (uint64_t)P_;
            c = P > 1 ? std::max<uint64_t>(1024, (walkers_ + P * P - 1) / (P * P) * 5 / 4 + 1024) : walkers_ + 16;
        }
        return std::max<uint64_t>(1, std::min<uint64_t>(std::max(c, cap_floor_), slot_cap_max_));
    }

    // items of `width` words grouped by destination (ex.send) -> received (ex.recv); reverse:
    // the replies of a query exchange go back the way the queries came
    void move(const int64_t* send, int64_t* recv, const Exchange& ex, uint64_t width, bool reverse = false) {
        const uint64_t P = (uint64_t)P_;
        const std::vector<uint64_t>& s = reverse ? ex.recv : ex.send;
        const std::vector<uint64_t>& r = reverse ? ex.send : ex.recv;
        std::vector<uint64_t> sc(P), sd(P), rc(P), rd(P);
        uint64_t so = 0, ro = 0;
        for (uint64_t q = 0; q < P; ++q) {
            sc[q] = s[q] * width;
            sd[q] = so;
            so += sc[q];
            rc[q] = r[q] * width;
            rd[q] = ro;
            ro += rc[q];
        }
        comm_.alltoallv(send, sc.data(), sd.data(), recv, rc.data(), rd.data(), ex.gmax * width, stream_);
    }

    // a host value into device memory without a host-side copy (two 32-bit fills: async)
    void put_word(int64_t* dev, uint64_t v) {
        hip_check(hipMemsetD32Async((hipDeviceptr_t)dev, (int)(uint32_t)v, 1, stream_), "hipMemsetD32Async");
        hip_check(hipMemsetD32Async((hipDeviceptr_t)((char*)dev + 4), (int)(uint32_t)(v >> 32), 1, stream_),
                  "hipMemsetD32Async");
    }

    void stage(const int64_t* recv, uint64_t pos, uint64_t m, uint64_t total, hipEvent_t arrived) {
        hip_check(hipStreamWaitEvent(stream_, arrived, 0), "hipStreamWaitEvent");
        abi_check(kh_insert_words_stage_dev(t_, recv + pos * W_, m, total));
    }

    void ensure_events(size_t n) {
        while (events_.size() < n) {
            hipEvent_t e;
            hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
            events_.push_back(e);
        }
    }

    // Splitter segments: link each segment to its successor's owner, all-gather every rank's
    // predecessor table, rank the chains on the device, send the segments' text to the contig
    // origins, materialise.
    void segments_end(const int64_t* trecv, uint64_t r, uint64_t nseg) {
        constexpr uint64_t L = KH_LINK_WORDS, S = KH_SEG_REC_WORDS, PW = KH_PRED_WORDS;
        const bool local = P_ == 1;
        Exchange ex;
        int64_t* lout = lout_.words(std::max<uint64_t>(nseg, 1) * L);
        abi_check(kh_mwalk_link_dev(t_, trecv, r, lout, counts_.words(P_ + 1)));
        exchange_counts(ex, nsp_);
        int64_t* lin = lout;
        if (!local) {
            lin = lin_.words(std::max<uint64_t>(ex.recv_total, 1) * L);
            move(lout, lin, ex, L);
        }
        uint64_t stride = 0;
        for (uint64_t x : ex.extra) stride = std::max(stride, x);
        int64_t* preds = qout_.words(std::max<uint64_t>(stride, 1) * PW);
        abi_check(kh_mwalk_pred_dev(t_, lin, ex.recv_total, preds, stride));
        int64_t* allp = preds;
        if (!local) {
            allp = qin_.words(std::max<uint64_t>(stride * P_, 1) * PW);
            comm_.allgather_dev(preds, stride * PW, allp, stream_);
        }
        abi_check(kh_mwalk_resolve_dev(t_, allp, stride));
        int64_t* tout = sout_.words(std::max<uint64_t>(r + nseg, 1) * S);
        abi_check(kh_mwalk_retag_dev(t_, trecv, r, tout, counts_.words(P_ + 1)));
        exchange_counts(ex);
        int64_t* tin = tout;
        if (!local) {
            tin = sin_.words(std::max<uint64_t>(ex.recv_total, 1) * S);
            move(tout, tin, ex, S);
        }
        abi_check(kh_mwalk_end_seg_dev(t_, trecv, r, tin, ex.recv_total));
    }

    int k_;
    Comm& comm_;
    int P_, rank_, device_;
    const void* group_;
    kh_table* t_ = nullptr;
    hipStream_t stream_ = nullptr, xstream_ = nullptr;
    uint64_t W_ = 2, R_ = 15;
    int rounds_ = 0, checks_ = 0, rounds_hint_ = 0;
    uint64_t inserted_ = 0;  // k-mers this shard holds since the last clear
    int ranks_per_device_ = 1;
    uint64_t syncs_ = 0;     // blocking device reads by this host (host_syncs() adds the library's)
    uint64_t ns_ = 0, nsp_ = 0, walkers_ = 0, splitters_ = 0;  // of the last insert_all
    std::string err_;        // this shard could not be sized by the last insert_all
    std::vector<uint64_t> caps_;  // slot capacity per round, learnt from the last assemble
    uint64_t caps_walkers_ = 0;   // ... whose walker count (another count: caps_ not used)
    uint64_t cap_floor_ = 0;      // this assemble: the demand of rounds that held messages back
    uint64_t slot_cap_max_ = ~0ull;
    std::mutex m_;
    std::vector<hipEvent_t> events_;
    DevBuf words_, recv_, counts_, tout_, trecv_, lout_, lin_, qout_, qin_, sout_, sin_, recs_, pack_, gather_, live_;
    DevBuf slots_[2], recv_slots_[2];
};

}  // namespace kh
