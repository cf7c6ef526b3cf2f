// kh_bench_cpp.cpp — the sharded step timed through the C++ host (dist_hash_map.hpp), beside the
// Python host's bench line (bench.py / cs267_hw3_amd/dist.py bench_main).
//
// One step = clear + insert_all_dev of the rank's block + assemble (migrating walk, contig text in
// HBM), every rank at once: the collective body of the reference's timed region
// (kmer_hash.cpp:119-137) with the records already on the device. P ranks are threads of this
// process, rank r on GPU r % #GPUs: RCCL over xGMI (ncclCommInitAll) when every rank has its own
// GPU, else kh::ThreadComm (device copies; P logical ranks on one GPU). Timing brackets every step
// with a barrier + device sync on both sides and takes the max over ranks, as bench.py does.
//
//   ./kh_bench_cpp [--ranks P] [--comm rccl|thread] [--k 51] [--n 200000000] [--len-min 8]
//                  [--len-max 200] [--seed 51] [--steps 5] [--warmup 2] [--no-verify]
// --n is per rank (weak scaling, like bench.py's default). Prints one JSON line.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "cs267_hw3_amd/dist_hash_map.hpp"
#include "cs267_hw3_amd/rccl_comm.hpp"

namespace {

struct Opt {
    int ranks = 1, k = 51, steps = 5, warmup = 2;
    uint64_t n = 200000000ull, seed = 51;
    uint32_t len_min = 8, len_max = 200;
    std::string comm = "auto";
    bool verify = true;
};

void gen_check(int rc) {
    if (rc != KH_OK) throw std::runtime_error(kh_last_error());
}

}  // namespace

int main(int argc, char** argv) {
    Opt o;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
            return argv[++i];
        };
        if (a == "--ranks") o.ranks = atoi(val());
        else if (a == "--comm") o.comm = val();
        else if (a == "--k") o.k = atoi(val());
        else if (a == "--n") o.n = strtoull(val(), nullptr, 10);
        else if (a == "--len-min") o.len_min = (uint32_t)atoi(val());
        else if (a == "--len-max") o.len_max = (uint32_t)atoi(val());
        else if (a == "--seed") o.seed = strtoull(val(), nullptr, 10);
        else if (a == "--steps") o.steps = atoi(val());
        else if (a == "--warmup") o.warmup = atoi(val());
        else if (a == "--no-verify") o.verify = false;
        else throw std::runtime_error("unknown option " + a);
    }
    const int P = o.ranks;
    int ngpu = 0;
    kh::hip_check(hipGetDeviceCount(&ngpu), "hipGetDeviceCount");
    if (ngpu < 1) throw std::runtime_error("no GPU visible");
    const bool rccl = o.comm == "rccl" || (o.comm == "auto" && ngpu >= P);
    std::vector<int> devices(P);
    for (int r = 0; r < P; ++r) devices[r] = r % ngpu;
    const uint64_t n_total = o.n * (uint64_t)P;
    kh_gen* g = nullptr;
    const auto tg = std::chrono::steady_clock::now();
    gen_check(kh_gen_create(&g, o.k, n_total, o.len_min, o.len_max, 0, o.seed, 1, 16));
    const double gen_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tg).count();
    std::unique_ptr<kh::ThreadComm::Group> tgroup;
    std::vector<std::unique_ptr<kh::RcclComm>> rcomms;
    std::vector<kh::Comm*> comms(P);
    if (rccl) {
        rcomms = kh::RcclComm::init_all(devices);
        for (int r = 0; r < P; ++r) comms[r] = rcomms[r].get();
    } else {
        tgroup.reset(new kh::ThreadComm::Group(P));
        for (int r = 0; r < P; ++r) comms[r] = tgroup->comm(r);
    }
    const uint64_t split = (n_total + P - 1) / P;  // read_kmers.hpp:55-58 block split
    std::vector<double> mean_s(P, 0.0);
    std::vector<std::vector<double>> step_ms(P);
    std::vector<int> ok(P, 1), rounds(P, 0), checks(P, 0);
    std::vector<uint64_t> syncs(P, 0);
    std::vector<uint64_t> lookups(P, 0), contigs(P, 0);
    std::mutex em;
    std::exception_ptr first;
    std::vector<std::thread> th;
    for (int r = 0; r < P; ++r)
        th.emplace_back([&, r] {
            try {
                kh::hip_check(hipSetDevice(devices[r]), "hipSetDevice");
                const uint64_t b = std::min<uint64_t>(split * r, n_total), e = std::min<uint64_t>(b + split, n_total);
                const int R = kh_record_size(o.k);
                void* recs = nullptr;
                kh::hip_check(hipMalloc(&recs, (e - b) * R + 16), "hipMalloc");
                kh::ShardedTable sh(o.k, (uint64_t)((double)split * 1.02) + 4096, *comms[r], devices[r]);
                sh.set_ranks_per_device(rccl ? 1 : (P + ngpu - 1) / ngpu);
                gen_check(kh_gen_records_dev(g, b, e, recs, sh.stream()));
                kh::hip_check(hipStreamSynchronize(sh.stream()), "hipStreamSynchronize");
                auto step = [&] {
                    sh.clear();
                    const uint64_t s0 = sh.host_syncs();
                    sh.insert_all_dev(recs, e - b);
                    rounds[r] = sh.assemble(n_total);
                    syncs[r] = sh.host_syncs() - s0;  // blocking device reads of this step
                    checks[r] = sh.checks();
                };
                for (int i = 0; i < o.warmup; ++i) step();
                double sum = 0;
                for (int i = 0; i < o.steps; ++i) {
                    comms[r]->barrier();
                    kh::hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
                    const auto t0 = std::chrono::steady_clock::now();
                    step();
                    kh::hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
                    comms[r]->barrier();
                    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                    step_ms[r].push_back(1e3 * s);
                    sum += s;
                }
                mean_s[r] = sum / std::max(o.steps, 1);
                kh_stats st{};
                kh::abi_check(kh_get_stats(sh.handle(), &st));
                lookups[r] = st.n_lookups;
                contigs[r] = st.n_starts;
                if (o.verify) {
                    uint64_t nb = 0;
                    gen_check(kh_gen_truth(g, b, e, nullptr, 0, &nb));
                    std::string want(nb, '\0');
                    gen_check(kh_gen_truth(g, b, e, nb ? &want[0] : nullptr, nb, &nb));
                    ok[r] = sh.contigs_text() == want;
                }
                kh::hip_check(hipFree(recs), "hipFree");
            } catch (const std::exception& ex) {
                fprintf(stderr, "rank %d: %s\n", r, ex.what());
                fflush(stderr);
                if (!tgroup) std::_Exit(1);  // RCCL peers would wait forever
                std::lock_guard<std::mutex> lk(em);
                if (!first) first = std::current_exception();
                tgroup->abort();
            }
        });
    for (auto& t : th) t.join();
    if (first) std::rethrow_exception(first);
    const double tmax = *std::max_element(mean_s.begin(), mean_s.end());
    uint64_t nl = 0, nc = 0;
    for (int r = 0; r < P; ++r) {
        nl += lookups[r];
        nc += contigs[r];
    }
    bool all_ok = true;
    for (int r = 0; r < P; ++r) all_ok = all_ok && ok[r];
    std::string steps_s;
    for (double x : step_ms[0]) steps_s += (steps_s.empty() ? "" : ", ") + std::to_string(x);
    printf("{\"metric\": \"k-mer inserts+lookups/sec (k=%d)\", \"value\": %.6e, \"unit\": \"ops/s\", \"host\": \"cpp\", "
           "\"n_gpus\": %d, \"ranks\": %d, \"comm\": \"%s\", \"steps\": %d, \"warmup\": %d, \"ms_per_step\": %.4f, "
           "\"step_ms_rank0\": [%s], \"higher_is_better\": true, \"scaling\": \"weak\", \"dtype\": \"u64\", "
           "\"data\": \"synthetic\", \"config\": {\"workload\": \"contigs U[%u,%u] k-mers, %llu k-mers per rank\", "
           "\"k\": %d, \"n_kmers_total\": %llu, \"contigs\": %llu, \"lookups\": %llu, \"walk_rounds\": %d}, "
           "\"verified_vs_truth\": %s, \"host_syncs_per_step_max\": %llu, \"walk_checks\": %d, \"gen_s\": %.1f}\n",
           o.k, (double)(n_total + nl) / tmax, std::min(P, ngpu), P, rccl ? "rccl" : "thread", o.steps, o.warmup,
           1e3 * tmax, steps_s.c_str(), o.len_min, o.len_max, (unsigned long long)o.n, o.k,
           (unsigned long long)n_total, (unsigned long long)nc, (unsigned long long)nl, rounds[0],
           o.verify ? (all_ok ? "true" : "false") : "null",
           (unsigned long long)*std::max_element(syncs.begin(), syncs.end()),
           *std::max_element(checks.begin(), checks.end()), gen_s);
    kh_gen_destroy(g);
    return all_ok ? 0 : 3;
}
