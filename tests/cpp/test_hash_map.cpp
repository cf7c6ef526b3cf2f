// C++ tests of the drop-in headers (include/cs267_hw3_amd/*.hpp), driven by tests/test_cpp_api.py.
//   test_hash_map_<K> stock   <kmer_file>                 HashMap(size): insert/find/size/full
//   test_hash_map_<K> refloop <kmer_file> <P> <prefix>    the reference's own initialize_kmers +
//        assemble_contigs + output_results (kmer_hash.cpp:21-68) over DistributedHashMap, P ranks
//        as threads on GPU 0 (kh::ThreadComm; P = 1: the single-GPU table), one find() per step
//   test_hash_map_<K> refloopc <kmer_file> <P> <prefix>   the same without a peer group and without
//        the caller's barriers: every find() a collective round, process_requests() serving the rest
//   test_hash_map_<K> rccl1loop <kmer_file> <prefix>      the reference loop over a one-rank RCCL
//        communicator without a peer group (one process per GPU)
//   test_hash_map_<K> rccl1   <kmer_file> <prefix>        DistributedHashMap over a one-rank RCCL
//        communicator (sharded code path, RCCL all-gathers) -> <prefix>_0.dat
//   test_hash_map_<K> gen     <n> <P> <len_min> <len_max> kh::ShardedTable at P ranks (threads, one
//        GPU) on n generated k-mers (records made in HBM by kh_gen_records_dev); large enough per
//        rank for the chunked, overlapped insert; each rank's text == its block's ground truth
//   test_hash_map_<K> gen2    <n_small> <n> <P>           one kh::ShardedTable per rank walks a small
//        generated set, is cleared, and walks a set of n (slot capacities learnt per input), then
//        the small one again; every text == its block's truth
// Exit status 0 = pass; a failed check prints it and exits 1.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <list>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "cs267_hw3_amd/hash_map.hpp"
#include "cs267_hw3_amd/rccl_comm.hpp"
#include "cs267_hw3_amd/read_kmers.hpp"

#define CHECK(c)                                                                 \
    do {                                                                         \
        if (!(c)) {                                                              \
            fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

namespace {

// README.md:95,99 stock surface: every k-mer inserted one by one, found again; absent keys are
// not found; size() is the constructor's; a full table refuses inserts.
int stock(const std::string& fname) {
    std::vector<kmer_pair> kmers = read_kmers(fname);
    const size_t n = kmers.size();
    HashMap hm(n * 2);
    CHECK(hm.size() == n * 2);
    for (const auto& k : kmers) CHECK(hm.insert(k));
    for (const auto& k : kmers) {
        kmer_pair got;
        CHECK(hm.find(k.kmer, got));
        CHECK(got == k);
    }
    // absent keys: the next k-mer of each contig end ('F' forward) is not in the set
    int absent = 0;
    for (const auto& k : kmers)
        if (k.forwardExt() == 'F') {
            kmer_pair got;
            std::string s = k.kmer_str().substr(1) + "A";
            bool present = false;
            for (const auto& o : kmers) present |= o.kmer_str() == s;
            if (!present) {
                CHECK(!hm.find(pkmer_t(s), got));
                ++absent;
            }
            if (absent > 20) break;
        }
    CHECK(absent > 0);
    // "HashMap is full": a table of n slots takes exactly n k-mers
    HashMap small(n / 2);
    size_t ok = 0;
    for (const auto& k : kmers) ok += small.insert(k);
    CHECK(ok == n / 2);
    for (size_t i = 0; i < n / 2; ++i) {
        kmer_pair got;
        CHECK(small.find(kmers[i].kmer, got) && got == kmers[i]);
    }
    kmer_pair got;
    CHECK(!small.find(kmers[n - 1].kmer, got));
    // assemble() on the stock table == one line per start k-mer
    std::string text = hm.assemble();
    size_t starts = 0, lines = 0;
    for (const auto& k : kmers) starts += k.backwardExt() == 'F';
    for (char c : text) lines += c == '\n';
    CHECK(lines == starts);
    printf("stock ok: %zu k-mers, %d absent probes, %zu contigs\n", n, absent, lines);
    return 0;
}

// kmer_hash.cpp:21-68, verbatim in structure (find per step), for one rank. sync: the explicit
// barriers of a careful caller; without them the map's own collective points must do (insert_all
// ends in a barrier, hash_map.hpp:79; process_requests() answers finds until every rank is done,
// hash_map.hpp:110-113).
void ref_rank(const std::string& fname, DistributedHashMap& hashmap, int rank, int world, const std::string& prefix,
              bool sync) {
    std::vector<kmer_pair> kmers = read_kmers(fname, world, rank);
    if (sync) hashmap.barrier();
    // initialize_kmers
    std::vector<kmer_pair> start_nodes;
    hashmap.insert_all(kmers);
    for (const auto& kmer : kmers)
        if (kmer.backwardExt() == 'F') start_nodes.push_back(kmer);
    if (sync) hashmap.barrier();
    // assemble_contigs
    std::list<std::list<kmer_pair>> contigs;
    for (const auto& start_kmer : start_nodes) {
        std::list<kmer_pair> contig;
        contig.push_back(start_kmer);
        while (contig.back().forwardExt() != 'F') {
            kmer_pair found;
            bool success = hashmap.find(contig.back().next_kmer().get(), found);
            if (!success) throw std::runtime_error("Error: k-mer not found in Distributed HashMap.");
            contig.push_back(found);
        }
        contigs.push_back(contig);
    }
    // every rank's finds are answered before any table goes away
    if (sync) hashmap.barrier();
    else hashmap.process_requests();
    // output_results
    std::ofstream fout(prefix + "_" + std::to_string(rank) + ".dat");
    for (const auto& contig : contigs) fout << extract_contig(contig) << std::endl;
}

// mode "refloop": ranks as threads with a peer group (finds read the owner's table directly);
// "refloopc": no peer group and no explicit barriers -- every find is a collective round (the
// one-process-per-GPU protocol), driven by P threads over kh::ThreadComm
int refloop(const std::string& fname, int world, const std::string& prefix, bool collective) {
    const size_t n = line_count(fname);
    if (world == 1) {
        DistributedHashMap hashmap(n * 2, 0, 1, 0);
        ref_rank(fname, hashmap, 0, 1, prefix, !collective);
        return 0;
    }
    kh::ThreadComm::Group group(world);
    auto& ctx = kh::rank_contexts();
    ctx.assign(world, kh::RankContext{});
    for (int r = 0; r < world; ++r) ctx[r] = kh::RankContext{group.comm(r), 0, collective ? nullptr : &group};
    std::vector<std::thread> th;
    int failed = 0;
    for (int r = 0; r < world; ++r)
        th.emplace_back([&, r] {
            try {
                DistributedHashMap hashmap(n * 2, r, world, 0);
                ref_rank(fname, hashmap, r, world, prefix, !collective);
            } catch (const std::exception& ex) {
                fprintf(stderr, "rank %d: %s\n", r, ex.what());
                failed = 1;
                group.abort();
            }
        });
    for (auto& t : th) t.join();
    return failed;
}

// the reference's find loop over an RCCL communicator without a peer group (the
// one-process-per-GPU shape, RcclComm(rank, world, id, device)), at one rank
int rccl1loop(const std::string& fname, const std::string& prefix) {
    auto comms = kh::RcclComm::init_all({0});
    const size_t n = line_count(fname);
    DistributedHashMap hashmap(n * 2, *comms[0], 0, nullptr);
    ref_rank(fname, hashmap, 0, 1, prefix, false);
    return 0;
}

int rccl1(const std::string& fname, const std::string& prefix) {
    auto comms = kh::RcclComm::init_all({0});
    const size_t n = line_count(fname);
    DistributedHashMap hashmap(n * 2, *comms[0], 0, comms.data());
    CHECK(hashmap.shard() != nullptr);
    hashmap.insert_all(read_kmers(fname));
    std::string text = hashmap.assemble();
    std::ofstream(prefix + "_0.dat", std::ios::binary).write(text.data(), (std::streamsize)text.size());
    // a single-key find through the sharded surface
    std::vector<kmer_pair> kmers = read_kmers(fname);
    kmer_pair got;
    CHECK(hashmap.find(kmers[0].kmer_str(), got) && got == kmers[0]);
    printf("rccl1 ok: %zu bytes, %d rounds\n", text.size(), hashmap.shard()->rounds());
    return 0;
}

// read_kmers.hpp:55-58 block split
void block(uint64_t n, int P, int r, uint64_t& b, uint64_t& e) {
    const uint64_t split = (n + P - 1) / P;
    b = std::min<uint64_t>(split * r, n);
    e = std::min<uint64_t>(b + split, n);
}

int gen(uint64_t n, int P, uint32_t lmin, uint32_t lmax) {
    kh_gen* g = nullptr;
    kh::abi_check(kh_gen_create(&g, KMER_LEN, n, lmin, lmax, 10, 4242, 1, 0));
    kh::ThreadComm::Group group(P);
    std::vector<std::thread> th;
    std::vector<int> ok(P, 0);
    std::vector<int> rounds(P, 0);
    for (int r = 0; r < P; ++r)
        th.emplace_back([&, r] {
            try {
                kh::hip_check(hipSetDevice(0), "hipSetDevice");
                uint64_t b, e;
                block(n, P, r, b, e);
                kh::ShardedTable st(KMER_LEN, n / P + 1, *group.comm(r), 0, &group);
                kh::DevBuf recs;
                void* d = recs.ensure((e - b) * kh_record_size(KMER_LEN) + 16);
                kh::abi_check(kh_gen_records_dev(g, b, e, d, st.stream()));
                st.insert_all_dev(d, e - b);
                rounds[r] = st.assemble(n);
                const std::string text = st.contigs_text();
                uint64_t bytes = 0;
                kh::abi_check(kh_gen_truth(g, b, e, nullptr, 0, &bytes));
                std::string want(bytes, '\0');
                kh::abi_check(kh_gen_truth(g, b, e, &want[0], bytes, &bytes));
                ok[r] = text == want;
            } catch (const std::exception& ex) {
                fprintf(stderr, "rank %d: %s\n", r, ex.what());
                group.abort();
            }
        });
    for (auto& t : th) t.join();
    kh_gen_destroy(g);
    for (int r = 0; r < P; ++r)
        if (!ok[r]) {
            fprintf(stderr, "rank %d differs from the truth of its block\n", r);
            return 1;
        }
    printf("gen ok: n=%llu P=%d rounds=%d\n", (unsigned long long)n, P, rounds[0]);
    return 0;
}

// small input, clear, large input, clear, small again on the same maps (slot
// capacities learnt from one input must not size another's rounds)
int gen2(uint64_t n_small, uint64_t n, int P) {
    kh_gen* gs = nullptr;
    kh_gen* gl = nullptr;
    kh::abi_check(kh_gen_create(&gs, KMER_LEN, n_small, 8, 200, 0, 3, 1, 0));
    kh::abi_check(kh_gen_create(&gl, KMER_LEN, n, 8, 200, 0, 4, 1, 0));
    kh::ThreadComm::Group group(P);
    std::vector<std::thread> th;
    std::vector<int> ok(P, 0);
    std::vector<int> rounds(P, 0);
    for (int r = 0; r < P; ++r)
        th.emplace_back([&, r] {
            try {
                kh::hip_check(hipSetDevice(0), "hipSetDevice");
                kh::ShardedTable st(KMER_LEN, n_small / P + 1, *group.comm(r), 0, &group);
                kh::DevBuf recs;
                int good = 1;
                for (kh_gen* g : {gs, gl, gs}) {
                    const uint64_t m = g == gs ? n_small : n;
                    uint64_t b, e;
                    block(m, P, r, b, e);
                    void* d = recs.ensure((e - b) * kh_record_size(KMER_LEN) + 16);
                    st.clear();
                    kh::abi_check(kh_gen_records_dev(g, b, e, d, st.stream()));
                    st.insert_all_dev(d, e - b);
                    rounds[r] = std::max(rounds[r], st.assemble(m));
                    const std::string text = st.contigs_text();
                    uint64_t bytes = 0;
                    kh::abi_check(kh_gen_truth(g, b, e, nullptr, 0, &bytes));
                    std::string want(bytes, '\0');
                    kh::abi_check(kh_gen_truth(g, b, e, &want[0], bytes, &bytes));
                    good &= text == want;
                }
                ok[r] = good;
            } catch (const std::exception& ex) {
                fprintf(stderr, "rank %d: %s\n", r, ex.what());
                group.abort();
            }
        });
    for (auto& t : th) t.join();
    kh_gen_destroy(gs);
    kh_gen_destroy(gl);
    for (int r = 0; r < P; ++r)
        if (!ok[r]) {
            fprintf(stderr, "rank %d differs from the truth of its block\n", r);
            return 1;
        }
    printf("gen2 ok: n_small=%llu n=%llu P=%d max rounds=%d\n", (unsigned long long)n_small, (unsigned long long)n, P,
           rounds[0]);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s stock|refloop|rccl1 <kmer_file> ...\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1], fname = argv[2];
    try {
        if (mode == "gen" && argc >= 6)
            return gen(strtoull(argv[2], nullptr, 10), atoi(argv[3]), (uint32_t)atoi(argv[4]), (uint32_t)atoi(argv[5]));
        if (mode == "gen2" && argc >= 5)
            return gen2(strtoull(argv[2], nullptr, 10), strtoull(argv[3], nullptr, 10), atoi(argv[4]));
        if (mode == "stock") return stock(fname);
        if (mode == "refloop" && argc >= 5) return refloop(fname, atoi(argv[3]), argv[4], false);
        if (mode == "refloopc" && argc >= 5) return refloop(fname, atoi(argv[3]), argv[4], true);
        if (mode == "rccl1loop" && argc >= 4) return rccl1loop(fname, argv[3]);
        if (mode == "rccl1" && argc >= 4) return rccl1(fname, argv[3]);
    } catch (const std::exception& ex) {
        fprintf(stderr, "%s\n", ex.what());
        return 1;
    }
    fprintf(stderr, "bad arguments\n");
    return 2;
}
