// Spread of hot minimizer families over the placement regions (host only, kh_codec.hpp rules):
// level 1 remaps a region whose minimizer family overfills it to hot_region(minimizer window,
// neighbour window); level 2 sends the remapped keys of a target region that the remap itself
// overfills (a family sharing its neighbour window too: the generator's flank mode) to a region of
// their key hash. Prints the largest region counts after each level.
//   ./tools/hot_spread [n] [flank 0|1]
#include <algorithm>
#include <string>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kh_codec.hpp"
#include "kmer_hash_amd.h"
using namespace kh;

static void top(const char* what, std::vector<uint32_t> c) {
    std::sort(c.rbegin(), c.rend());
    printf("%s: largest region counts %u %u %u, 10th %u\n", what, c[0], c[1], c[2], c[10]);
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 20000000ull;
    const uint32_t flags = argc > 2 && atoi(argv[2]) ? KH_GEN_HOT_FLANK : 0u;
    kh_gen* g;
    if (kh_gen_create_hot_ex(&g, 51, n, 8, 200, 0, 5198, 1, 8, 0, 0, 0, 300, 8, flags)) {
        fprintf(stderr, "%s\n", kh_last_error());
        return 1;
    }
    KParams p = make_params(51);
    const uint64_t cap = (uint64_t)(n / 0.5);
    set_region_bits(p, cap);
    const uint32_t NR = 1u << p.rbits;
    std::vector<uint8_t> recs(n * p.R);
    kh_gen_records(g, 0, n, recs.data());
    std::vector<uint32_t> l0(NR, 0), wins(n), fwd(n);
    std::vector<int> js(n);
    std::vector<Key> keys(n);
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t ext;
        parse_record(&recs[i * p.R], p, keys[i], ext);
        fwd[i] = ext_fwd(ext);
        const uint32_t mn = mini_scan(keys[i], p);
        wins[i] = mini_window(keys[i], mn, p);
        js[i] = (int)(mn & 63u);
        ++l0[mini_region(wins[i], p)];
    }
    const double mean = (double)n / NR, thr = 2.0 * mean;  // the marks' threshold, roughly
    std::vector<uint32_t> hot(2 * HOT_LEVEL_WORDS, 0);
    uint64_t h1 = 0, h2 = 0;
    for (uint32_t r = 0; r < NR; ++r)
        if (l0[r] > thr) hot[r >> 5] |= 1u << (r & 31), ++h1;
    p.hot = hot.data();
    std::vector<uint32_t> l1(NR, 0);
    for (uint64_t i = 0; i < n; ++i) ++l1[place_w(wins[i], keys[i], p, js[i]).r];
    for (uint32_t r = 0; r < NR; ++r)
        if (l1[r] > thr) hot[HOT_LEVEL_WORDS + (r >> 5)] |= 1u << (r & 31), ++h2;
    std::vector<uint32_t> l2(NR, 0);
    for (uint64_t i = 0; i < n; ++i) ++l2[place_w(wins[i], keys[i], p, js[i]).r];
    // runs: k-mers whose successor lands in another region (each costs the walker a lookup)
    auto breaks = [&]() {
        uint64_t b = 0;
        for (uint64_t i = 0; i < n; ++i) {
            if (fwd[i] > 3) continue;
            const Key y = key_next(keys[i], fwd[i], p);
            b += place(y, p).r != place_w(wins[i], keys[i], p, js[i]).r;
        }
        return (unsigned long long)b;
    };
    printf("region changes along contigs (walker lookups): %llu of %llu k-mers\n", breaks(), (unsigned long long)n);
    // per contig (ground-truth lines): lookups along it = 1 + region changes; the longest contigs
    // of lookups bound the walk (one dependent request each)
    {
        uint64_t bytes = 0;
        kh_gen_truth(g, 0, n, nullptr, 0, &bytes);
        std::string text(bytes, '\0');
        kh_gen_truth(g, 0, n, &text[0], bytes, &bytes);
        std::vector<uint32_t> per;
        size_t a = 0;
        while (a < text.size()) {
            size_t b = text.find('\n', a);
            const int L = (int)(b - a);
            uint32_t look = 1;
            uint32_t prev = ~0u;
            for (int t = 0; t + p.K <= L; ++t) {
                uint8_t pk[32] = {0};
                for (int q = 0; q < p.K; ++q) {
                    const char c = text[a + t + q];
                    const uint32_t code = c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3;
                    pk[q / 4] |= (uint8_t)(code << (6 - 2 * (q % 4)));
                }
                pk[p.P] = 'A';
                pk[p.P + 1] = 'A';
                Key k;
                uint32_t ext;
                parse_record(pk, p, k, ext);
                const uint32_t r = place(k, p).r;
                if (t && r != prev) ++look;
                prev = r;
            }
            per.push_back(look);
            a = b + 1;
        }
        std::sort(per.rbegin(), per.rend());
        double mean = 0;
        for (auto x : per) mean += x;
        printf("lookups per contig: mean %.2f, top %u %u %u, 100th %u, 1000th %u (of %zu contigs)\n",
               mean / per.size(), per[0], per[1], per[2], per[99], per[999], per.size());
    }
    printf("n=%llu flank=%u regions=%u mean=%.0f level-1 marks %llu level-2 marks %llu\n", (unsigned long long)n,
           flags, NR, mean, (unsigned long long)h1, (unsigned long long)h2);
    top("minimizer regions", l0);
    top("after level 1", l1);
    top("after level 2", l2);
    // keys by the fill of their region's slice (equal ranges: 2x the mean slots at load 0.5), and
    // the mean linear-probe length of a successful lookup at that fill, (1 + 1/(1 - a)) / 2
    {
        const double bins[] = {0.5, 0.67, 0.8, 0.9, 1.0};
        uint64_t nb[6] = {0};
        double probe = 0;
        for (uint32_t r = 0; r < NR; ++r) {
            const double a = l2[r] / (2.0 * mean);
            int b = 0;
            while (b < 5 && a > bins[b]) ++b;
            nb[b] += l2[r];
            const double ac = a < 0.99 ? a : 0.99;
            probe += l2[r] * 0.5 * (1.0 + 1.0 / (1.0 - ac));
        }
        printf("keys by slice fill: <=0.5 %.3f, 0.5-0.67 %.3f, 0.67-0.8 %.3f, 0.8-0.9 %.3f, 0.9-1 %.3f, >1 %.3f;"
               " mean probe %.2f slots\n", nb[0] / (double)n, nb[1] / (double)n, nb[2] / (double)n,
               nb[3] / (double)n, nb[4] / (double)n, nb[5] / (double)n, probe / n);
    }
    kh_gen_destroy(g);
}
