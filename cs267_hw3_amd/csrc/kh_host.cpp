// kh_host.cpp — host-side C ABI pieces: the reference codec helpers (packing.hpp, pkmer_t.hpp,
// kmer_t.hpp, read_kmers.hpp) and the deterministic synthetic dataset generator.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kmer_hash_amd.h"
#include "kh_codec.hpp"
#include "kh_internal.hpp"

namespace {

int hfail(int code, const char* msg) {
    kh_set_error_internal(msg);
    return code;
}

int pick_threads(int threads) {
    int hc = (int)std::thread::hardware_concurrency();
    if (hc <= 0) hc = 1;
    if (threads <= 0) threads = hc < 16 ? hc : 16;
    return threads;
}

template <class F>
void parallel_for(uint64_t n, int threads, F f) {
    if (n == 0) return;
    threads = (int)std::min<uint64_t>((uint64_t)threads, (n + 4095) / 4096);
    if (threads <= 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> th;
    const uint64_t chunk = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const uint64_t b = (uint64_t)t * chunk, e = std::min(n, b + chunk);
        if (b >= e) break;
        th.emplace_back([=] { f(b, e); });
    }
    for (auto& x : th) x.join();
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Codec helpers.
extern "C" {

int kh_pack_kmer(int k, const char* kmer, uint8_t* out) {
    if (k < 1 || k > KH_K_MAX || !kmer || !out) return hfail(KH_ERR_ARG, "bad argument");
    kh::KParams p = kh::make_params(k);
    kh::Key key{0, 0};
    unsigned __int128 V = 0;
    for (int i = 0; i < k; ++i) {
        uint32_t c = kh::base_code((uint8_t)kmer[i]);
        if (c > 3) return hfail(KH_ERR_BAD_BASE, "k-mer base outside {A,C,G,T}");
        V = (V << 2) | c;
    }
    key.lo = (uint64_t)V & kh::LO_MASK;
    key.hi = (uint64_t)(V >> 62);
    kh::key_to_packed(key, out, p);
    return KH_OK;
}

int kh_unpack_kmer(int k, const uint8_t* packed, char* out) {
    if (k < 1 || k > KH_K_MAX || !packed || !out) return hfail(KH_ERR_ARG, "bad argument");
    kh::KParams p = kh::make_params(k);
    kh::Key key = kh::key_from_packed(packed, p);
    for (int i = 0; i < k; ++i) out[i] = (char)kh::code_char(kh::key_base(key, i, p));
    return KH_OK;
}

uint64_t kh_djb2(int k, const uint8_t* packed) {
    if (k < 1 || k > KH_K_MAX || !packed) return 0;
    return kh::djb2(packed, (k + 3) / 4);
}

int kh_next_kmer(int k, const uint8_t* rec, uint8_t* out) {
    if (k < 1 || k > KH_K_MAX || !rec || !out) return hfail(KH_ERR_ARG, "bad argument");
    kh::KParams p = kh::make_params(k);
    kh::Key key;
    uint32_t ext;
    kh::parse_record(rec, p, key, ext);
    uint32_t f = kh::ext_fwd(ext);
    if (f > 3) return hfail(KH_ERR_BAD_BASE, "forward extension is not a base");
    kh::key_to_packed(kh::key_next(key, f, p), out, p);
    return KH_OK;
}

int kh_pack_text(int k, const char* text, uint64_t len, uint8_t* recs, uint64_t* n_out) {
    if (k < 1 || k > KH_K_MAX || (!text && len) || !n_out) return hfail(KH_ERR_ARG, "bad argument");
    const uint64_t line = (uint64_t)k + 4;
    const uint64_t n = len / line;  // read_kmers.hpp:64 fixed line length
    *n_out = n;
    if (!recs) return KH_OK;
    kh::KParams p = kh::make_params(k);
    int bad = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const char* l = text + i * line;
        uint8_t* r = recs + i * (uint64_t)p.R;
        if (kh_pack_kmer(k, l, r) != KH_OK) bad = 1;
        r[p.P] = (uint8_t)l[k + 1];
        r[p.P + 1] = (uint8_t)l[k + 2];
    }
    return bad ? hfail(KH_ERR_BAD_BASE, "k-mer text has a base outside {A,C,G,T}") : KH_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------------
// Synthetic generator.
namespace {

uint64_t splitmix(uint64_t x) {
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
    uint64_t round_f(uint64_t x, int r) const { return splitmix(x ^ (seed + 0x51ed27ull * (r + 1))) & mask; }
    uint64_t fwd1(uint64_t x) const {
        uint64_t L = x >> half, R = x & mask;
        for (int r = 0; r < 4; ++r) {
            uint64_t t = L ^ round_f(R, r);
            L = R;
            R = t;
        }
        return (L << half) | R;
    }
    uint64_t inv1(uint64_t y) const {
        uint64_t L = y >> half, R = y & mask;
        for (int r = 3; r >= 0; --r) {
            uint64_t t = R ^ round_f(L, r);
            R = L;
            L = t;
        }
        return (L << half) | R;
    }
    uint64_t fwd(uint64_t x) const {
        uint64_t y = fwd1(x);
        while (y >= n) y = fwd1(y);
        return y;
    }
    uint64_t inv(uint64_t y) const {
        uint64_t x = inv1(y);
        while (x >= n) x = inv1(x);
        return x;
    }
};

}  // namespace

struct kh_gen {
    int K = 0;
    kh::KParams kp{};
    uint64_t n = 0, seed = 0;
    bool shuffle = true;
    int threads = 1;
    std::vector<uint32_t> len;   // k-mers per contig
    std::vector<uint64_t> off;   // first global k-mer index of each contig (size C+1)
    std::vector<uint32_t> salt;  // re-draw counter per contig (uniqueness)
    Perm perm;

    // 32 bases of contig i per 64-bit word: base j = bits 2(j%32).. of word(i, j/32).
    uint64_t word(uint64_t i, uint64_t b) const {
        return splitmix(splitmix(seed ^ 0x6a09e667f3bcc908ull ^ (i * 0x9e3779b97f4a7c15ull)) ^
                        ((uint64_t)salt[i] << 40) ^ b);
    }
    uint32_t base(uint64_t i, uint64_t j) const { return (uint32_t)(word(i, j >> 5) >> (2 * (j & 31))) & 3u; }
    // k-mer t of contig i as (hi, lo) plus the ext code.
    void kmer(uint64_t i, uint64_t t, kh::Key& k, uint32_t& ext) const {
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
        k.lo = (uint64_t)V & kh::LO_MASK;
        k.hi = (uint64_t)(V >> 62);
        const uint32_t bwd = t == 0 ? kh::EXT_F : base(i, t - 1);
        const uint32_t fwd = (t + 1 == len[i]) ? kh::EXT_F : base(i, t + K);
        ext = bwd | (fwd << 3);
    }
    // C5 record order (front_starts): every start k-mer (t = 0) before every other k-mer, each
    // group in its own seeded shuffle; nb[i] = off[i] - i = non-start k-mers before contig i.
    bool front_starts = false;
    Perm perm_s, perm_n;
    std::vector<uint64_t> nb;
    uint64_t pos_of(uint64_t g) const {
        if (!front_starts) return shuffle ? perm.fwd(g) : g;
        const uint64_t i = (uint64_t)(std::upper_bound(off.begin(), off.end(), g) - off.begin()) - 1;
        const uint64_t C = len.size();
        if (g == off[i]) return shuffle ? perm_s.fwd(i) : i;
        const uint64_t q = g - i - 1;
        return C + (shuffle ? perm_n.fwd(q) : q);
    }
    uint64_t g_of(uint64_t p) const {
        if (!front_starts) return shuffle ? perm.inv(p) : p;
        const uint64_t C = len.size();
        if (p < C) return off[shuffle ? perm_s.inv(p) : p];
        const uint64_t q = shuffle ? perm_n.inv(p - C) : p - C;
        const uint64_t i = (uint64_t)(std::upper_bound(nb.begin(), nb.end(), q) - nb.begin()) - 1;
        return off[i] + 1 + (q - nb[i]);
    }
};

namespace {

struct KeyRef {
    uint64_t hi, lo;
    uint32_t contig;
    bool operator<(const KeyRef& o) const { return hi != o.hi ? hi < o.hi : lo < o.lo; }
};

void psort(std::vector<KeyRef>& v, int threads) {
    const uint64_t n = v.size();
    if (threads <= 1 || n < (1u << 16)) {
        std::sort(v.begin(), v.end());
        return;
    }
    int parts = 1;
    while (parts * 2 <= threads) parts *= 2;
    std::vector<uint64_t> b(parts + 1);
    for (int i = 0; i <= parts; ++i) b[i] = n * i / parts;
    std::vector<std::thread> th;
    for (int i = 0; i < parts; ++i)
        th.emplace_back([&, i] { std::sort(v.begin() + b[i], v.begin() + b[i + 1]); });
    for (auto& x : th) x.join();
    for (int w = 1; w < parts; w *= 2) {
        th.clear();
        for (int i = 0; i + w < parts; i += 2 * w) {
            int hiidx = std::min(i + 2 * w, parts);
            th.emplace_back([&, i, w, hiidx] {
                std::inplace_merge(v.begin() + b[i], v.begin() + b[i + w], v.begin() + b[hiidx]);
            });
        }
        for (auto& x : th) x.join();
    }
}

}  // namespace

extern "C" {

int kh_gen_create(kh_gen** out, int k, uint64_t n, uint32_t len_min, uint32_t len_max,
                  uint32_t single_permille, uint64_t seed, int shuffle, int threads) {
    return kh_gen_create_skewed(out, k, n, len_min, len_max, single_permille, seed, shuffle, threads, 0, 0, 0);
}

int kh_gen_create_skewed(kh_gen** out, int k, uint64_t n, uint32_t len_min, uint32_t len_max,
                         uint32_t single_permille, uint64_t seed, int shuffle, int threads, uint32_t n_long,
                         uint32_t long_len, int front_starts) {
    if (!out) return hfail(KH_ERR_ARG, "out is NULL");
    *out = nullptr;
    if (k < 1 || k > KH_K_MAX || len_min < 1 || len_max < len_min || single_permille > 1000)
        return hfail(KH_ERR_ARG, "bad generator parameters");
    kh_gen* g = new (std::nothrow) kh_gen();
    if (!g) return hfail(KH_ERR_NOMEM, "host allocation failed");
    g->K = k;
    g->kp = kh::make_params(k);
    g->n = n;
    g->seed = seed;
    g->shuffle = shuffle != 0;
    g->threads = pick_threads(threads);
    // 1) contig lengths until n k-mers (last one truncated); the first n_long contigs have
    //    long_len k-mers (C5: a handful of 10^6-k-mer chains among short contigs)
    uint64_t sum = 0;
    const uint64_t span = (uint64_t)len_max - len_min + 1;
    for (uint64_t i = 0; sum < n; ++i) {
        const uint64_t u = splitmix(seed * 0x2545f4914f6cdd1dull + i + 1);
        uint64_t L = ((u % 1000) < single_permille) ? 1 : len_min + (u >> 10) % span;
        if (i < n_long && long_len) L = long_len;
        if (L > n - sum) L = n - sum;
        g->len.push_back((uint32_t)L);
        g->off.push_back(sum);
        sum += L;
    }
    g->off.push_back(sum);
    g->salt.assign(g->len.size(), 0);
    g->perm.init(n, splitmix(seed ^ 0x3c6ef372fe94f82bull));
    if (front_starts) {
        const uint64_t C = g->len.size();
        g->front_starts = true;
        g->nb.resize(C);
        for (uint64_t i = 0; i < C; ++i) g->nb[i] = g->off[i] - i;
        g->perm_s.init(C, splitmix(seed ^ 0x510e527fade682d1ull));
        g->perm_n.init(n - C, splitmix(seed ^ 0x9b05688c2b3e6c1full));
    }
    // 2) uniqueness: re-draw every contig holding a k-mer that occurs more than once, until none.
    //    Skipped when the expected number of repeats n^2 / (2 * 4^k) is below 1e-9 (k=51 and
    //    anything below 10^12 k-mers); the table's duplicate counter still checks it on insert.
    const double expect = (double)n * (double)n / 2.0 / __builtin_powi(4.0, k);
    if (expect > 1e-9 && n > 1) {
        const uint64_t C = g->len.size();
        std::vector<uint8_t> redo(C, 1);
        for (int round = 0; round < 256; ++round) {
            std::vector<KeyRef> keys(n);
            parallel_for(C, g->threads, [&](uint64_t b, uint64_t e) {
                for (uint64_t i = b; i < e; ++i)
                    for (uint64_t t = 0; t < g->len[i]; ++t) {
                        kh::Key kk;
                        uint32_t ext;
                        g->kmer(i, t, kk, ext);
                        keys[g->off[i] + t] = KeyRef{kk.hi, kk.lo, (uint32_t)i};
                    }
            });
            psort(keys, g->threads);
            std::fill(redo.begin(), redo.end(), 0);
            uint64_t bad = 0;
            for (uint64_t a = 0; a < n;) {
                uint64_t b = a + 1;
                while (b < n && keys[b].hi == keys[a].hi && keys[b].lo == keys[a].lo) ++b;
                if (b - a > 1)
                    for (uint64_t q = a; q < b; ++q) {
                        if (!redo[keys[q].contig]) ++bad;
                        redo[keys[q].contig] = 1;
                    }
                a = b;
            }
            if (!bad) break;
            for (uint64_t i = 0; i < C; ++i)
                if (redo[i]) ++g->salt[i];
            if (round == 255) {
                kh_gen_destroy(g);
                return hfail(KH_ERR_ARG, "could not draw unique k-mers (k too small for n?)");
            }
        }
    }
    *out = g;
    return KH_OK;
}

int kh_gen_destroy(kh_gen* g) {
    delete g;
    return KH_OK;
}

uint64_t kh_gen_num_contigs(const kh_gen* g) { return g ? g->len.size() : 0; }

int kh_gen_records(const kh_gen* g, uint64_t pb, uint64_t pe, uint8_t* out) {
    if (!g || (!out && pe > pb) || pe < pb || pe > g->n) return hfail(KH_ERR_ARG, "bad range");
    const int R = g->kp.R;
    parallel_for(pe - pb, g->threads, [&](uint64_t b, uint64_t e) {
        for (uint64_t q = b; q < e; ++q) {
            const uint64_t gi = g->g_of(pb + q);
            const uint64_t i = (uint64_t)(std::upper_bound(g->off.begin(), g->off.end(), gi) -
                                          g->off.begin()) - 1;
            kh::Key k;
            uint32_t ext;
            g->kmer(i, gi - g->off[i], k, ext);
            kh::write_record(out + q * (uint64_t)R, k, ext, g->kp);
        }
    });
    return KH_OK;
}

int kh_gen_truth(const kh_gen* g, uint64_t pb, uint64_t pe, char* out, uint64_t cap,
                 uint64_t* bytes_out) {
    if (!g || pe < pb || pe > g->n) return hfail(KH_ERR_ARG, "bad range");
    const uint64_t C = g->len.size();
    std::vector<std::pair<uint64_t, uint32_t>> sel;  // (start position, contig)
    for (uint64_t i = 0; i < C; ++i) {
        const uint64_t p = g->front_starts ? (g->shuffle ? g->perm_s.fwd(i) : i) : g->pos_of(g->off[i]);
        if (p >= pb && p < pe) sel.emplace_back(p, (uint32_t)i);
    }
    std::sort(sel.begin(), sel.end());
    std::vector<uint64_t> o(sel.size() + 1, 0);
    for (size_t s = 0; s < sel.size(); ++s) o[s + 1] = o[s] + g->len[sel[s].second] + (uint64_t)g->K;
    if (bytes_out) *bytes_out = o.back();
    if (!out) return KH_OK;
    if (cap < o.back()) return hfail(KH_ERR_ARG, "truth buffer too small");
    parallel_for(sel.size(), g->threads, [&](uint64_t b, uint64_t e) {
        for (uint64_t s = b; s < e; ++s) {
            const uint64_t i = sel[s].second;
            char* d = out + o[s];
            const uint64_t nb = g->len[i] + (uint64_t)g->K - 1;
            uint64_t w = 0;
            for (uint64_t j = 0; j < nb; ++j) {
                if ((j & 31) == 0) w = g->word(i, j >> 5);
                d[j] = (char)kh::code_char((uint32_t)(w >> (2 * (j & 31))) & 3u);
            }
            d[nb] = '\n';
        }
    });
    return KH_OK;
}

}  // extern "C"
