// Spread of a hot minimizer family (the C5 hot-bucket set) over the remap target regions: the
// secondary-window rule of kh_codec.hpp (second_window: the M-mer next to the minimizer occurrence)
// against the rule it replaced (the lowest-order other window, which often overlaps the shared
// motif and so takes few distinct values). Host only: ./tools/hot_spread [n]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "kmer_hash_amd.h"
#include "kh_codec.hpp"
using namespace kh;
static uint32_t old_second(Key k, uint32_t win, const KParams& p) {
    uint32_t best = 0xFFFFFFFFu, bw = win;
    for (int j = 0; j <= p.K - p.M; ++j) {
        const uint32_t w = win_bits(k, j, p);
        const uint32_t o = (win_order(w) << 6) | (uint32_t)j;
        if (w != win && o < best) { best = o; bw = w; }
    }
    return bw;
}
int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 20000000ull;
    kh_gen* g;
    if (kh_gen_create_hot(&g, 51, n, 8, 200, 0, 5198, 1, 8, 0, 0, 0, 300, 8)) return 1;
    KParams p = make_params(51);
    uint64_t cap = (uint64_t)(n / 0.5);
    int rb = 9; while (rb < 17 && (cap >> (rb + 1)) >= REGION_SLOTS) ++rb;
    p.rbits = rb;
    const uint32_t NR = 1u << rb;
    std::vector<uint8_t> recs(n * p.R);
    kh_gen_records(g, 0, n, recs.data());
    std::vector<uint32_t> cnt(NR, 0), wins(n);
    std::vector<Key> keys(n);
    for (uint64_t i = 0; i < n; ++i) {
        uint32_t ext; parse_record(&recs[i * p.R], p, keys[i], ext);
        wins[i] = mini_window(keys[i], mini_scan(keys[i], p), p);
        ++cnt[mini_region(wins[i], p)];
    }
    const double mean = (double)n / NR;
    std::vector<uint32_t> tn(NR, 0), to(NR, 0);
    uint64_t nhot = 0, hotr = 0;
    for (uint32_t r = 0; r < NR; ++r) hotr += cnt[r] > 4 * mean;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = mini_region(wins[i], p);
        if (cnt[r] <= 4 * mean) continue;
        ++nhot;
        ++tn[mix32((wins[i] * 0x9E3779B1u) ^ second_window(keys[i], wins[i], p) ^ 0x2545F491u) >> (32 - rb)];
        ++to[mix32((wins[i] * 0x9E3779B1u) ^ old_second(keys[i], wins[i], p) ^ 0x2545F491u) >> (32 - rb)];
    }
    std::sort(tn.rbegin(), tn.rend()); std::sort(to.rbegin(), to.rend());
    printf("n=%llu regions=%u mean=%.0f slots/region=%.0f hot regions=%llu hot keys=%llu\n",
           (unsigned long long)n, NR, mean, (double)cap / NR, (unsigned long long)hotr, (unsigned long long)nhot);
    printf("new: top target counts %u %u %u %u ; old: %u %u %u %u\n", tn[0], tn[1], tn[2], tn[10], to[0], to[1], to[2], to[10]);
    kh_gen_destroy(g);
}
