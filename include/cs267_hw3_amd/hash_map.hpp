// hash_map.hpp (drop-in) — the reference's table surfaces, backed by the GPU table of the C ABI.
//
//   DistributedHashMap(size_t table_size, int rank_id, int world_size)   hash_map.hpp:50-52
//   void insert_all(const std::vector<kmer_pair>&)                       hash_map.hpp:55-80
//   bool find(const std::string& key, kmer_pair& result)                 hash_map.hpp:83-107
//   void process_requests()                                              hash_map.hpp:110-113
//   HashMap(size_t size); bool insert(const kmer_pair&);                 stock starter surface
//   bool find(const pkmer_t&, kmer_pair&); size_t size() const           (README.md:95,99)
//
// GPU additions: assemble() walks every start k-mer collected by the inserts on the device and
// returns the test_<rank>.dat bytes (kmer_hash.cpp:38-68 in one call). Compile with
// -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include and link -lkmerhash_amd -lamdhip64.
// Single-key insert() calls are buffered on the host and flushed as one batch before the next
// find()/size()/assemble(), so starter-style loops stay correct without a device call per k-mer.
#pragma once
#include <memory>
#include <stdexcept>
#include <algorithm>
#include <string>
#include <vector>

#include "dist_hash_map.hpp"
#include "kmer_t.hpp"

namespace kh_detail {
inline void check(int rc) {
    if (rc != KH_OK) throw std::runtime_error(kh_last_error());
}
}  // namespace kh_detail

class HashMap {
public:
    // Stock starter semantics (README.md:95): the table holds up to `size` k-mers and insert()
    // returns false ("HashMap is full") beyond that. The GPU table behind it has 2 * size slots
    // (load 0.5).
    explicit HashMap(size_t size, int device = 0) : HashMap(size, size, device) {}
    // Table allocated for n_kmers (<= size); a bulk insert_all into the empty table grows it
    // (DistributedHashMap at world_size 1: size = 2 * k-mers, kmer_hash.cpp:108-109).
    HashMap(size_t size, uint64_t n_kmers, int device) : size_(size), n_kmers_(n_kmers ? n_kmers : 1) {
        kh_detail::check(kh_create(&t_, KMER_LEN, n_kmers_, 0.5, device));
    }
    ~HashMap() { kh_destroy(t_); }
    HashMap(const HashMap&) = delete;
    HashMap& operator=(const HashMap&) = delete;

    bool insert(const kmer_pair& kmer) {
        if (inserted_ + pending_.size() >= size_) return false;  // "HashMap is full!"
        pending_.push_back(kmer);
        return true;
    }
    bool find(const pkmer_t& key, kmer_pair& val) {
        flush();
        uint8_t found = 0;
        kh_detail::check(kh_find(t_, key.data, 1, reinterpret_cast<uint8_t*>(&val), &found));
        return found != 0;
    }
    size_t size() const { return size_; }

    void insert_all(const std::vector<kmer_pair>& items) {
        flush();
        if (inserted_ == 0) grow(items.size());
        kh_detail::check(kh_insert(t_, reinterpret_cast<const uint8_t*>(items.data()), items.size()));
        inserted_ += items.size();
    }
    // Contig text (one line per contig, start-node order) of every start k-mer inserted so far.
    std::string assemble() {
        flush();
        uint64_t nc = 0, nb = 0;
        kh_detail::check(kh_assemble(t_, &nc, &nb));
        std::string s(nb, '\0');
        if (nb) kh_detail::check(kh_contigs_text(t_, &s[0], nb));
        return s;
    }
    kh_table* handle() { return t_; }

private:
    void grow(uint64_t n) {
        if (n <= n_kmers_) return;
        kh_detail::check(kh_reserve(t_, n));
        n_kmers_ = n;
    }
    void flush() {
        if (pending_.empty()) return;
        // the first flush sizes the table for everything insert() may still accept (size_):
        // a table holding k-mers cannot grow (kh_reserve), so a later flush must fit
        if (inserted_ == 0) grow(std::max<uint64_t>(pending_.size(), size_));
        kh_detail::check(kh_insert(t_, reinterpret_cast<const uint8_t*>(pending_.data()), pending_.size()));
        inserted_ += pending_.size();
        pending_.clear();
    }
    kh_table* t_ = nullptr;
    size_t size_ = 0, inserted_ = 0;
    uint64_t n_kmers_ = 1;
    std::vector<kmer_pair> pending_;
};

// DistributedHashMap (hash_map.hpp:12-114). world_size == 1: one GPU table (HashMap above).
// world_size > 1: one shard per rank (kh::ShardedTable, dist_hash_map.hpp) over the rank's
// kh::Comm, found in kh::rank_contexts() — the launcher fills it before starting one thread per
// rank, as upcxx::init() would (tools/kmer_hash.cpp) — or passed explicitly.
class DistributedHashMap {
public:
    DistributedHashMap(size_t table_size, int rank_id, int world_size, int device = -1)
        : size_(table_size ? table_size : 2), rank_(rank_id), world_(world_size) {
        if (world_size == 1) {
            map_.reset(new HashMap(size_, size_ / 2, device < 0 ? 0 : device));
            return;
        }
        auto& ctx = kh::rank_contexts();
        if ((int)ctx.size() != world_size || rank_id < 0 || rank_id >= world_size || !ctx[rank_id].comm)
            throw std::runtime_error("DistributedHashMap: world_size > 1 needs kh::rank_contexts() set up by "
                                     "the launcher (one kh::Comm per rank)");
        make_shard(*ctx[rank_id].comm, device < 0 ? ctx[rank_id].device : device, ctx[rank_id].peer_group);
    }
    DistributedHashMap(size_t table_size, kh::Comm& comm, int device, const void* peer_group = nullptr)
        : size_(table_size ? table_size : 2), rank_(comm.rank()), world_(comm.size()) {
        make_shard(comm, device, peer_group);
    }

    // hash_map.hpp:55-80 (collective at world_size > 1; ends like the reference's barrier)
    void insert_all(const std::vector<kmer_pair>& items) {
        if (map_) return map_->insert_all(items);
        shard_->insert_all(items.data(), items.size());
    }
    // hash_map.hpp:83-107: the owner's table answers (one device round trip per call)
    bool find(const pkmer_t& key, kmer_pair& result) {
        if (map_) return map_->find(key, result);
        return shard_->find(key.data, reinterpret_cast<uint8_t*>(&result));
    }
    bool find(const std::string& key, kmer_pair& result) { return find(pkmer_t(key), result); }
    // hash_map.hpp:110-113 (upcxx::progress + barrier): collective at world_size > 1; a rank that
    // has finished its finds answers the others' until every rank is here
    void process_requests() { barrier(); }

    // kmer_hash.cpp:38-68 in one call: walk every start k-mer collected by insert_all on the
    // device and return this rank's test_<rank>.dat bytes (collective at world_size > 1).
    std::string assemble() {
        if (map_) return map_->assemble();
        shard_->assemble(size_ / 2);  // the reference sizes the table at 2 x the k-mer count
        return shard_->contigs_text();
    }
    void barrier() {
        if (shard_) shard_->barrier();
    }
    kh_table* handle() { return map_ ? map_->handle() : shard_->handle(); }
    kh::ShardedTable* shard() { return shard_.get(); }
    int rank() const { return rank_; }
    int world() const { return world_; }

private:
    void make_shard(kh::Comm& comm, int device, const void* peer_group) {
        // expected share of the k-mers (size_ / 2 in all); the shard grows to what it receives
        const uint64_t hint = size_ / 2 / (uint64_t)world_ + 1024;
        shard_.reset(new kh::ShardedTable(KMER_LEN, hint, comm, device, peer_group));
        // ranks driven by this process on the same device share its free memory
        int same = 1;
        const auto& ctx = kh::rank_contexts();
        if ((int)ctx.size() == world_) {
            same = 0;
            for (const auto& c : ctx) same += c.device == device;
        } else if (peer_group) {
            same = world_;
        }
        shard_->set_ranks_per_device(same);
    }
    size_t size_;
    int rank_, world_;
    std::unique_ptr<HashMap> map_;
    std::unique_ptr<kh::ShardedTable> shard_;
};
