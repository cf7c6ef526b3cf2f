// ref_harness.cpp — TEST INFRASTRUCTURE ONLY. Builds against the reference's OWN headers
// (/root/reference/{packing,pkmer_t,kmer_t,read_kmers}.hpp, compiled in place, never copied) so
// that the golden vectors in tests/golden/ come from the reference codec itself:
//   kat <kmer> <fb>   -> "<packed hex> <djb2> <next packed hex|->"  (packing.hpp, pkmer_t.hpp:31-37,
//                        kmer_t.hpp:51-53)
//   assemble <file>   -> contigs on stdout, one per line, start-node order (test_0.dat bytes)
// The reference driver (kmer_hash.cpp) needs <upcxx/upcxx.hpp>, which this image lacks, so it is
// not built; its world_size==1 control flow (kmer_hash.cpp:21-55, hash_map.hpp:33-35,86-91: a
// std::unordered_map<std::string,kmer_pair> keyed by kmer_str()) is restated in main() below.
#include <cstdint>
#include <cstdio>
#include <list>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "read_kmers.hpp"  // pulls kmer_t.hpp, pkmer_t.hpp, packing.hpp from /root/reference

static std::string hex(const unsigned char* d, int n) {
    static const char* H = "0123456789abcdef";
    std::string s;
    for (int i = 0; i < n; ++i) {
        s += H[d[i] >> 4];
        s += H[d[i] & 15];
    }
    return s;
}

int main(int argc, char** argv) {
    if (argc >= 4 && std::string(argv[1]) == "kat") {
        kmer_pair kp(argv[2], argv[3]);
        std::string nx = "-";
        if (kp.forwardExt() != 'F') {
            pkmer_t n = kp.next_kmer();
            nx = hex(n.data, PACKED_KMER_LEN);
        }
        printf("%s %llu %s\n", hex(kp.kmer.data, PACKED_KMER_LEN).c_str(),
               (unsigned long long)kp.hash(), nx.c_str());
        return 0;
    }
    if (argc >= 3 && std::string(argv[1]) == "assemble") {
        std::vector<kmer_pair> kmers = read_kmers(argv[2], 1, 0);
        std::unordered_map<std::string, kmer_pair> map;
        std::vector<kmer_pair> starts;
        for (const auto& k : kmers) {
            map[k.kmer_str()] = k;
            if (k.backwardExt() == 'F') starts.push_back(k);
        }
        for (const auto& s : starts) {
            std::list<kmer_pair> contig;
            contig.push_back(s);
            while (contig.back().forwardExt() != 'F') {
                auto it = map.find(contig.back().next_kmer().get());
                if (it == map.end()) {
                    fprintf(stderr, "k-mer not found\n");
                    return 2;
                }
                contig.push_back(it->second);
            }
            std::string c = extract_contig(contig);
            fwrite(c.data(), 1, c.size(), stdout);
            fputc('\n', stdout);
        }
        return 0;
    }
    fprintf(stderr, "usage: %s kat <kmer> <fb> | assemble <file>\n", argv[0]);
    return 1;
}
