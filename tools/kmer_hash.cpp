// kmer_hash.cpp (drop-in driver) — same argv, stdout lines and test_<rank>.dat outputs as the
// reference's kmer_hash.cpp:60-150, with the insert + walk done by the GPU table.
//   [KH_RANKS=P] ./kmer_hash_<K> kmer_file [verbose|test [prefix]]
// The reference runs P UPC++ processes; here one process drives P ranks, one thread each, as the
// reference's main body (kmer_hash.cpp:84-150) per thread:
//   * P GPUs visible and KH_COMM != thread: RCCL over xGMI, rank r on GPU r (ncclCommInitAll)
//   * otherwise: P logical ranks sharing the GPUs round-robin, exchanges by device copies
//     (kh::ThreadComm) — same protocol, used to test P > #GPUs on one card
// Timed region as in the reference (kmer_hash.cpp:129-137): records parsed in host memory at the
// start, each rank's contigs in host memory at the end (H2D of the records and D2H of the text
// included). Device of a single rank: $KH_DEVICE (default 0).
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <fstream>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "cs267_hw3_amd/hash_map.hpp"
#include "cs267_hw3_amd/rccl_comm.hpp"
#include "cs267_hw3_amd/read_kmers.hpp"

namespace {

// BUtil::print (butil.hpp:6-14): a collective; rank 0 prints
void rank0_print(DistributedHashMap& h, const std::string& s) {
    fflush(stdout);
    h.barrier();
    if (h.rank() == 0) {
        fputs(s.c_str(), stdout);
        fflush(stdout);
    }
    h.barrier();
}

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, f);
    vsnprintf(buf, sizeof buf, f, ap);
    va_end(ap);
    return buf;
}

struct Args {
    std::string fname, run_type, prefix = "test";
    size_t n_kmers = 0, table_size = 0;
};

// kmer_hash.cpp:111-148 for one rank
void rank_main(const Args& a, int rank, int world, int device) {
    if (world == 1 && a.run_type == "verbose")
        printf("Initializing hash table of size %lu for %lu kmers.\n", a.table_size, a.n_kmers);
    DistributedHashMap hashmap(a.table_size, rank, world, device);
    if (world > 1 && a.run_type == "verbose")
        rank0_print(hashmap, fmt("Initializing hash table of size %lu for %lu kmers.\n", a.table_size, a.n_kmers));
    std::vector<kmer_pair> kmers = read_kmers(a.fname, world, rank);
    if (a.run_type == "verbose") {
        if (world > 1)
            rank0_print(hashmap, "Finished reading kmers.\n");
        else
            printf("Finished reading kmers.\n");
    }
    hashmap.barrier();

    auto t0 = std::chrono::high_resolution_clock::now();
    hashmap.insert_all(kmers);  // + start-node collection on the device (kmer_hash.cpp:21-33)
    auto t1 = std::chrono::high_resolution_clock::now();
    std::string text = hashmap.assemble();  // kmer_hash.cpp:38-55 + the contigs in host memory
    hashmap.barrier();
    auto t2 = std::chrono::high_resolution_clock::now();

    const double ins = std::chrono::duration<double>(t1 - t0).count();
    const double asm_ = std::chrono::duration<double>(t2 - t1).count();
    const double tot = std::chrono::duration<double>(t2 - t0).count();
    std::string out;
    if (a.run_type != "test") {
        out = fmt("Finished inserting in %lf sec\n", ins) + fmt("Assembled in %lf total\n", tot);
    } else {
        std::ofstream fout(a.prefix + "_" + std::to_string(rank) + ".dat", std::ios::binary);
        fout.write(text.data(), (std::streamsize)text.size());
        fout.close();
        size_t contigs = 0;
        for (char c : text) contigs += c == '\n';
        const size_t nodes = text.size() - contigs * KMER_LEN;  // a line: K + len - 1 bases + '\n'
        // kmer_hash.cpp:71-78 verbatim (argument order included)
        out = fmt("Rank %d reconstructed %d contigs with %d nodes from %d start nodes. (%lf read, %lf insert, %lf total)\n",
                  rank, (int)contigs, (int)nodes, 0, asm_, ins, tot);
    }
    if (world > 1)
        rank0_print(hashmap, out);
    else
        fputs(out.c_str(), stdout);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        printf("Usage: ./kmer_hash kmer_file [verbose|test [prefix]]\n");
        return 1;
    }
    Args a;
    a.fname = argv[1];
    a.run_type = argc >= 3 ? argv[2] : "";
    if (a.run_type == "test" && argc >= 4) a.prefix = argv[3];
    const int ks = kmer_size(a.fname);
    if (ks != KMER_LEN)
        throw std::runtime_error("Error: " + a.fname + " contains " + std::to_string(ks) +
                                 "-mers, while this binary is compiled for " + std::to_string(KMER_LEN) +
                                 "-mers. Modify packing.hpp and recompile.");
    a.n_kmers = line_count(a.fname);
    a.table_size = a.n_kmers * 2;  // load factor 0.5 (kmer_hash.cpp:108-109)

    const char* er = getenv("KH_RANKS");
    const int world = er ? atoi(er) : 1;
    if (world < 1) throw std::runtime_error("KH_RANKS must be >= 1");
    if (world == 1) {
        const char* dev = getenv("KH_DEVICE");
        rank_main(a, 0, 1, dev ? atoi(dev) : 0);
        return 0;
    }
    int ngpu = 0;
    kh::hip_check(hipGetDeviceCount(&ngpu), "hipGetDeviceCount");
    if (ngpu < 1) throw std::runtime_error("no GPU visible");
    const char* ec = getenv("KH_COMM");
    const bool rccl = ngpu >= world && !(ec && std::string(ec) == "thread");
    std::vector<int> devices(world);
    for (int r = 0; r < world; ++r) devices[r] = r % ngpu;
    std::unique_ptr<kh::ThreadComm::Group> tgroup;
    std::vector<std::unique_ptr<kh::RcclComm>> rcomms;
    auto& ctx = kh::rank_contexts();
    ctx.assign(world, kh::RankContext{});
    if (rccl) {
        rcomms = kh::RcclComm::init_all(devices);
        for (int r = 0; r < world; ++r) ctx[r] = kh::RankContext{rcomms[r].get(), devices[r], rcomms.data()};
    } else {
        tgroup.reset(new kh::ThreadComm::Group(world));
        for (int r = 0; r < world; ++r) ctx[r] = kh::RankContext{tgroup->comm(r), devices[r], tgroup.get()};
    }
    std::mutex em;
    std::exception_ptr first;
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r)
        th.emplace_back([&, r] {
            try {
                rank_main(a, r, world, devices[r]);
            } catch (const std::exception& ex) {
                if (!tgroup) {  // the other ranks would wait in RCCL collectives forever
                    fprintf(stderr, "rank %d: %s\n", r, ex.what());
                    fflush(stderr);
                    std::_Exit(1);
                }
                std::lock_guard<std::mutex> g(em);
                if (!first) first = std::current_exception();
                tgroup->abort();
            }
        });
    for (auto& t : th) t.join();
    if (first) std::rethrow_exception(first);
    return 0;
}
