// kh_host.cpp — host-side C ABI pieces: the reference codec helpers (packing.hpp, pkmer_t.hpp,
// kmer_t.hpp, read_kmers.hpp) and the deterministic synthetic dataset generator.
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kmer_hash_amd.h"
#include "kh_codec.hpp"
#include "kh_gen.hpp"
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
// Synthetic generator (math in kh_gen.hpp, shared with the device generator kh_gen.hip).
struct kh_gen {
    int threads = 1;
    std::vector<uint32_t> len;   // k-mers per contig
    std::vector<uint64_t> off;   // first global k-mer index of each contig (size C+1)
    std::vector<uint32_t> salt;  // re-draw counter per contig (uniqueness)
    std::vector<uint64_t> nb;    // front_starts: non-start k-mers before contig i
    kh::GenView v;               // host pointers into the vectors above
    kh_gen_dev* dev[KH_GEN_MAX_DEVICES] = {};  // per-device copies of the arrays (kh_gen.hip), made on first use
    std::mutex dev_m;            // ranks (threads) may generate their blocks concurrently
    void bind() {
        v.C = len.size();
        v.len = len.data();
        v.off = off.data();
        v.salt = salt.data();
        v.nb = nb.empty() ? nullptr : nb.data();
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
    return kh_gen_create_hot(out, k, n, len_min, len_max, single_permille, seed, shuffle, threads, n_long, long_len,
                             front_starts, 0, 0);
}

int kh_gen_create_hot(kh_gen** out, int k, uint64_t n, uint32_t len_min, uint32_t len_max,
                      uint32_t single_permille, uint64_t seed, int shuffle, int threads, uint32_t n_long,
                      uint32_t long_len, int front_starts, uint32_t hot_permille, uint32_t n_motifs) {
    return kh_gen_create_hot_ex(out, k, n, len_min, len_max, single_permille, seed, shuffle, threads, n_long, long_len,
                                front_starts, hot_permille, n_motifs, 0u);
}

int kh_gen_create_hot_ex(kh_gen** out, int k, uint64_t n, uint32_t len_min, uint32_t len_max,
                         uint32_t single_permille, uint64_t seed, int shuffle, int threads, uint32_t n_long,
                         uint32_t long_len, int front_starts, uint32_t hot_permille, uint32_t n_motifs,
                         uint32_t flags) {
    if (!out) return hfail(KH_ERR_ARG, "out is NULL");
    const bool flank = (flags & KH_GEN_HOT_FLANK) != 0;
    *out = nullptr;
    if (k < 1 || k > KH_K_MAX || len_min < 1 || len_max < len_min || single_permille > 1000)
        return hfail(KH_ERR_ARG, "bad generator parameters");
    if (hot_permille > 1000 || (hot_permille && (n_motifs < 1 || n_motifs > (uint32_t)kh::GEN_MAX_MOTIFS)))
        return hfail(KH_ERR_ARG, "bad hot-motif parameters (hot_permille <= 1000, 1 <= n_motifs <= 64)");
    kh_gen* g = new (std::nothrow) kh_gen();
    if (!g) return hfail(KH_ERR_NOMEM, "host allocation failed");
    kh::GenView& v = g->v;
    v.K = k;
    v.kp = kh::make_params(k);
    v.n = n;
    v.seed = seed;
    v.shuffle = shuffle != 0;
    g->threads = pick_threads(threads);
    if (hot_permille && v.kp.M < k) {
        // motifs: per motif the M-mer of smallest minimizer order among 2^16 seeded draws
        v.hot_pm = hot_permille;
        v.n_motifs = n_motifs;
        v.M = (uint32_t)v.kp.M;
        v.plen = v.M;
        // every k-mer holds a full occurrence when the period is K - M + 1, which needs
        // K >= 2M + 7 to leave 8 free bases between occurrences (k=51: 20); shorter k (19, 31)
        // plant one motif per K bases: every k-mer keeps K - M free bases (4^7 at k=19) and
        // K - M + 1 of the K phases hold a full occurrence
        const uint32_t full = (uint32_t)(k - v.kp.M + 1);
        v.period = full >= v.M + 8 ? full : (uint32_t)k;
        if (flank) {
            // flank + motif (2M bases) once per K bases: K - 2M + 1 of the K phases (k=51: 20)
            // hold the whole pattern, the others keep >= K - 2M free bases
            if ((uint32_t)k < 2 * v.M + 8) {
                delete g;
                return hfail(KH_ERR_ARG, "hot flank mode needs k >= 2M + 8 (k=51 at M=16)");
            }
            v.plen = 2 * v.M;
            v.period = (uint32_t)k;
        }
        const uint32_t mmask = (uint32_t)((1ull << (2 * v.M)) - 1);
        for (uint32_t h = 0; h < n_motifs; ++h) {
            uint32_t best = 0, bo = 0xFFFFFFFFu;
            for (uint32_t t = 0; t < (1u << 16); ++t) {
                const uint32_t c = (uint32_t)kh::splitmix(seed ^ 0x7a5c9e1bd4f30c2dull ^ ((uint64_t)h << 20) ^ t) & mmask;
                const uint32_t o = kh::win_order(c);
                if (o < bo) {
                    bo = o;
                    best = c;
                }
            }
            v.motif[h] = best;
            // flank: any M-mer ordered above the motif (the motif stays the minimizer)
            for (uint32_t t = 0; flank; ++t) {
                const uint32_t c = (uint32_t)kh::splitmix(seed ^ 0x1f83d9abfb41bd6bull ^ ((uint64_t)h << 20) ^ t) & mmask;
                if (kh::win_order(c) > bo) {
                    v.flank[h] = c;
                    break;
                }
            }
        }
    }
    // 1) contig lengths until n k-mers (last one truncated); the first n_long contigs have
    //    long_len k-mers (C5: a handful of 10^6-k-mer chains among short contigs)
    uint64_t sum = 0;
    const uint64_t span = (uint64_t)len_max - len_min + 1;
    for (uint64_t i = 0; sum < n; ++i) {
        const uint64_t u = kh::splitmix(seed * 0x2545f4914f6cdd1dull + i + 1);
        uint64_t L = ((u % 1000) < single_permille) ? 1 : len_min + (u >> 10) % span;
        if (i < n_long && long_len) L = long_len;
        if (L > n - sum) L = n - sum;
        g->len.push_back((uint32_t)L);
        g->off.push_back(sum);
        sum += L;
    }
    g->off.push_back(sum);
    g->salt.assign(g->len.size(), 0);
    v.perm.init(n, kh::splitmix(seed ^ 0x3c6ef372fe94f82bull));
    if (front_starts) {
        const uint64_t C = g->len.size();
        v.front_starts = true;
        g->nb.resize(C);
        for (uint64_t i = 0; i < C; ++i) g->nb[i] = g->off[i] - i;
        v.perm_s.init(C, kh::splitmix(seed ^ 0x510e527fade682d1ull));
        v.perm_n.init(n - C, kh::splitmix(seed ^ 0x9b05688c2b3e6c1full));
    }
    g->bind();
    // 2) uniqueness: re-draw every contig holding a k-mer that occurs more than once, until none.
    //    Skipped when the expected number of repeats n^2 / (2 * 4^k) is below 1e-9 (k=51 and
    //    anything below 10^12 k-mers); the table's duplicate counter still checks it on insert.
    //    Hot contigs draw only K - M bases per k-mer (one of n_motifs motifs at one of `period`
    //    phases): their expected repeats are counted on that space (checked above 1e-6; the
    //    table's duplicate counter still reports any on insert).
    const double expect = (double)n * (double)n / 2.0 / __builtin_powi(4.0, k);
    double expect_hot = 0.0;
    if (v.hot_pm) {
        // a k-mer of a hot contig spans one period plus K - period bases that may repeat motif
        // bases: the phase with the most motif bases leaves the fewest free ones (k=51: 20, not
        // K - M = 35; 12 repeated hot k-mers at 1B before this was counted)
        int free_min = k;
        for (uint32_t t = 0; t < v.period; ++t) {
            int fixed = 0;
            for (int q = 0; q < k; ++q) fixed += (t + (uint32_t)q) % v.period < v.plen;
            free_min = k - fixed < free_min ? k - fixed : free_min;
        }
        const double nh = (double)n * v.hot_pm / 1000.0;
        expect_hot = nh * nh / 2.0 / ((double)v.n_motifs * v.period * __builtin_powi(4.0, free_min));
    }
    if ((expect > 1e-9 || expect_hot > 1e-6) && n > 1) {
        const uint64_t C = g->len.size();
        // only hot contigs can repeat a k-mer when the whole set cannot (k=51): check just those
        const bool hot_only = expect <= 1e-9;
        std::vector<uint64_t> koff(C + 1, 0);
        for (uint64_t i = 0; i < C; ++i) koff[i + 1] = koff[i] + ((!hot_only || v.hot_motif(i) >= 0) ? g->len[i] : 0);
        const uint64_t nk = koff[C];
        std::vector<uint8_t> redo(C, 1);
        for (int round = 0; round < 256; ++round) {
            std::vector<KeyRef> keys(nk);
            parallel_for(C, g->threads, [&](uint64_t b, uint64_t e) {
                for (uint64_t i = b; i < e; ++i)
                    for (uint64_t t = 0; t < koff[i + 1] - koff[i]; ++t) {
                        kh::Key kk;
                        uint32_t ext;
                        v.kmer(i, t, kk, ext);
                        keys[koff[i] + t] = KeyRef{kk.hi, kk.lo, (uint32_t)i};
                    }
            });
            psort(keys, g->threads);
            std::fill(redo.begin(), redo.end(), 0);
            uint64_t bad = 0;
            for (uint64_t a = 0; a < nk;) {
                uint64_t b = a + 1;
                while (b < nk && keys[b].hi == keys[a].hi && keys[b].lo == keys[a].lo) ++b;
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
    if (g)
        for (auto* d : g->dev) kh_gen_dev_free(d);
    delete g;
    return KH_OK;
}

uint64_t kh_gen_num_contigs(const kh_gen* g) { return g ? g->len.size() : 0; }

int kh_gen_records(const kh_gen* g, uint64_t pb, uint64_t pe, uint8_t* out) {
    if (!g || (!out && pe > pb) || pe < pb || pe > g->v.n) return hfail(KH_ERR_ARG, "bad range");
    const int R = g->v.kp.R;
    parallel_for(pe - pb, g->threads, [&](uint64_t b, uint64_t e) {
        for (uint64_t q = b; q < e; ++q) g->v.record(pb + q, out + q * (uint64_t)R);
    });
    return KH_OK;
}

int kh_gen_records_dev(kh_gen* g, uint64_t pb, uint64_t pe, void* dev_out, void* stream) {
    if (!g || (!dev_out && pe > pb) || pe < pb || pe > g->v.n) return hfail(KH_ERR_ARG, "bad range");
    if (pe == pb) return KH_OK;
    std::lock_guard<std::mutex> lk(g->dev_m);
    if (int rc = kh_gen_dev_records(g->v, g->dev, pb, pe, (uint8_t*)dev_out, stream)) return rc;
    return KH_OK;
}

int kh_gen_truth(const kh_gen* g, uint64_t pb, uint64_t pe, char* out, uint64_t cap,
                 uint64_t* bytes_out) {
    if (!g || pe < pb || pe > g->v.n) return hfail(KH_ERR_ARG, "bad range");
    const kh::GenView& v = g->v;
    const uint64_t C = g->len.size();
    std::vector<std::pair<uint64_t, uint32_t>> sel;  // (start position, contig)
    for (uint64_t i = 0; i < C; ++i) {
        const uint64_t p = v.front_starts ? (v.shuffle ? v.perm_s.fwd(i) : i) : v.pos_of(g->off[i]);
        if (p >= pb && p < pe) sel.emplace_back(p, (uint32_t)i);
    }
    std::sort(sel.begin(), sel.end());
    std::vector<uint64_t> o(sel.size() + 1, 0);
    for (size_t s = 0; s < sel.size(); ++s) o[s + 1] = o[s] + g->len[sel[s].second] + (uint64_t)v.K;
    if (bytes_out) *bytes_out = o.back();
    if (!out) return KH_OK;
    if (cap < o.back()) return hfail(KH_ERR_ARG, "truth buffer too small");
    parallel_for(sel.size(), g->threads, [&](uint64_t b, uint64_t e) {
        for (uint64_t s = b; s < e; ++s) {
            const uint64_t i = sel[s].second;
            char* d = out + o[s];
            const uint64_t nb = g->len[i] + (uint64_t)v.K - 1;
            uint64_t w = 0;
            for (uint64_t j = 0; j < nb; ++j) {
                if ((j & 31) == 0) w = v.word(i, j >> 5);
                d[j] = (char)kh::code_char((uint32_t)(w >> (2 * (j & 31))) & 3u);
            }
            d[nb] = '\n';
        }
    });
    return KH_OK;
}

}  // extern "C"
