// kh_gen.hpp — the synthetic dataset's math, shared by the host generator
// (kh_host.cpp) and the device record generator (kh_gen.hip): contig i's bases come from a
// counter-based hash, k-mer t of contig i is recomputed from them, and record positions are a
// seeded Feistel bijection of the global k-mer index. Everything is a pure function of the
// parameters and three per-contig arrays (len, off, salt), so any position range can be produced
// independently on either side.
#pragma once
#include <stdint.h>

#include "kh_codec.hpp"

namespace kh {

KH_HD uint64_t splitmix(uint64_t x) {
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// Seeded Feistel bijection on [0, n) by cycle walking over the next even power of two.
struct Perm {
    uint64_t n = 1, seed = 0;
    int half = 1;
    uint64_t mask = 1;
    void init(uint64_t n_, uint64_t seed_) {
        n = n_ ? n_ : 1;
        seed = seed_;
        int bits = 2;
        while (bits < 64 && (1ull << bits) < n) ++bits;
        if (bits & 1) ++bits;
        half = bits / 2;
        mask = (1ull << half) - 1;
    }
    KH_HD uint64_t round_f(uint64_t x, int r) const { return splitmix(x ^ (seed + 0x51ed27ull * (r + 1))) & mask; }
    KH_HD uint64_t fwd1(uint64_t x) const {
        uint64_t L = x >> half, R = x & mask;
        for (int r = 0; r < 4; ++r) {
            const uint64_t t = L ^ round_f(R, r);
            L = R;
            R = t;
        }
        return (L << half) | R;
    }
    KH_HD uint64_t inv1(uint64_t y) const {
        uint64_t L = y >> half, R = y & mask;
        for (int r = 3; r >= 0; --r) {
            const uint64_t t = R ^ round_f(L, r);
            R = L;
            L = t;
        }
        return (L << half) | R;
    }
    KH_HD uint64_t fwd(uint64_t x) const {
        uint64_t y = fwd1(x);
        while (y >= n) y = fwd1(y);
        return y;
    }
    KH_HD uint64_t inv(uint64_t y) const {
        uint64_t x = inv1(y);
        while (x >= n) x = inv1(x);
        return x;
    }
};

// last i with a[i] <= x (a sorted, a[0] <= x < a[m-1] + ...): std::upper_bound - 1
KH_HD uint64_t upper_index(const uint64_t* a, uint64_t m, uint64_t x) {
    uint64_t lo = 0, hi = m;  // first index with a[idx] > x in [lo, hi]
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (a[mid] <= x)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo - 1;
}

// Hot-minimizer stress (BASELINE configs[4] "hot-bucket"): up to this many shared M-mer motifs.
static constexpr int GEN_MAX_MOTIFS = 64;

// The generator's parameters and per-contig arrays (host or device pointers).
struct GenView {
    int K = 0;
    KParams kp{};
    uint64_t n = 0, seed = 0, C = 0;  // k-mers, seed, contigs
    bool shuffle = true, front_starts = false;
    const uint32_t* len = nullptr;    // k-mers per contig [C]
    const uint64_t* off = nullptr;    // first global k-mer index of each contig [C + 1]
    const uint32_t* salt = nullptr;   // re-draw counter per contig [C] (uniqueness)
    const uint64_t* nb = nullptr;     // front_starts: non-start k-mers before contig i [C]
    Perm perm, perm_s, perm_n;
    // Hot contigs (hot_pm per mille of contigs, chosen by a hash of the contig index): the motif
    // motif[h] (M bases, first base in the top bits) is planted at every position j with
    // j % period < M, period = K - M + 1 when that leaves >= 8 free bases between occurrences
    // (k=51: every k-mer of the contig holds exactly one full occurrence), else K (k=19, 31).
    // The motifs are the M-mers of smallest minimizer order among 2^16 seeded draws,
    // so the occurrence is (almost always) the k-mer's minimizer: all k-mers of the hot contigs
    // of motif h share one minimizer window, one placement region and one shard owner.
    // flank mode (the worst case of the table's hot remap): a fixed per-motif M-mer
    // flank[h] is planted right before every occurrence (pattern = flank then motif, plen = 2M, one
    // per K bases), so the k-mers holding the whole pattern share the minimizer AND its neighbour
    // window (kh_codec.hpp second_window): the remap alone would pile them into one region.
    uint32_t hot_pm = 0, n_motifs = 0, period = 0, M = 0, plen = 0;
    uint32_t motif[GEN_MAX_MOTIFS] = {};
    uint32_t flank[GEN_MAX_MOTIFS] = {};

    KH_HD uint64_t hot_hash(uint64_t i) const { return splitmix(seed ^ 0x3f84d5b5b5470917ull ^ (i * 0xd1b54a32d192ed03ull)); }
    // motif index of contig i, or -1 when the contig is not hot
    KH_HD int hot_motif(uint64_t i) const {
        if (!hot_pm) return -1;
        const uint64_t h = hot_hash(i);
        return (h % 1000) < hot_pm ? (int)((h >> 32) % n_motifs) : -1;
    }
    // 32 bases of contig i per 64-bit word: base j = bits 2(j%32).. of word(i, j/32).
    KH_HD uint64_t word(uint64_t i, uint64_t b) const {
        uint64_t r = splitmix(splitmix(seed ^ 0x6a09e667f3bcc908ull ^ (i * 0x9e3779b97f4a7c15ull)) ^
                              ((uint64_t)salt[i] << 40) ^ b);
        const int h = hot_motif(i);
        if (h < 0) return r;
        // pattern bases, first base in the top bits: flank (flank mode) then motif
        const uint64_t pat = plen > M ? ((uint64_t)flank[h] << (2 * M)) | motif[h] : (uint64_t)motif[h];
        uint32_t q = (uint32_t)((b * 32) % period);
        for (int x = 0; x < 32; ++x) {
            if (q < plen) {
                const uint64_t base = (pat >> (2 * (plen - 1 - q))) & 3u;
                r = (r & ~(3ull << (2 * x))) | (base << (2 * x));
            }
            if (++q == period) q = 0;
        }
        return r;
    }
    KH_HD uint32_t base(uint64_t i, uint64_t j) const { return (uint32_t)(word(i, j >> 5) >> (2 * (j & 31))) & 3u; }
    // k-mer t of contig i as (hi, lo) plus the ext code.
    KH_HD void kmer(uint64_t i, uint64_t t, Key& k, uint32_t& ext) const {
        unsigned __int128 V = 0;
        uint64_t wb = ~0ull, w = 0;
        for (int q = 0; q < K; ++q) {
            const uint64_t j = t + q;
            if ((j >> 5) != wb) {
                wb = j >> 5;
                w = word(i, wb);
            }
            V = (V << 2) | ((w >> (2 * (j & 31))) & 3u);
        }
        k.lo = (uint64_t)V & LO_MASK;
        k.hi = (uint64_t)(V >> 62);
        const uint32_t bwd = t == 0 ? EXT_F : base(i, t - 1);
        const uint32_t fwd = (t + 1 == len[i]) ? EXT_F : base(i, t + K);
        ext = bwd | (fwd << 3);
    }
    KH_HD uint64_t contig_of(uint64_t g) const { return upper_index(off, C + 1, g); }
    // C5 record order (front_starts): every start k-mer (t = 0) before every other k-mer, each
    // group in its own seeded shuffle.
    KH_HD uint64_t pos_of(uint64_t g) const {
        if (!front_starts) return shuffle ? perm.fwd(g) : g;
        const uint64_t i = contig_of(g);
        if (g == off[i]) return shuffle ? perm_s.fwd(i) : i;
        const uint64_t q = g - i - 1;
        return C + (shuffle ? perm_n.fwd(q) : q);
    }
    KH_HD uint64_t g_of(uint64_t p) const {
        if (!front_starts) return shuffle ? perm.inv(p) : p;
        if (p < C) return off[shuffle ? perm_s.inv(p) : p];
        const uint64_t q = shuffle ? perm_n.inv(p - C) : p - C;
        const uint64_t i = upper_index(nb, C, q);
        return off[i] + 1 + (q - nb[i]);
    }
    // the record at output position p
    KH_HD void record(uint64_t p, uint8_t* out) const {
        const uint64_t gi = g_of(p);
        const uint64_t i = contig_of(gi);
        Key k;
        uint32_t ext;
        kmer(i, gi - off[i], k, ext);
        write_record(out, k, ext, kp);
    }
};

}  // namespace kh
