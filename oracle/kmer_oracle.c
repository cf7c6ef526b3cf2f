/* kmer_oracle.c — TEST INFRASTRUCTURE ONLY (see kmer_oracle.h).
 * CPU restatement of the reference's serial path; every function cites what it follows in
 * /root/reference. Deliberately written the slow, obvious way (string round trips, djb2, modulo
 * linear probing) so that it mirrors the reference rather than the GPU design.
 */
#include "kmer_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int packed_len(int K) { return (K + 3) / 4; } /* packing.hpp:9 */

/* packing.hpp:50-75 packFourMer: A=0 C=1 G=2 T=3, first base most significant. */
static uint8_t pack_four(const char* four) {
    int v = 0;
    for (int i = 0; i < 4; ++i) {
        int code = 0;
        switch (four[i]) {
        case 'A': code = 0; break;
        case 'C': code = 1; break;
        case 'G': code = 2; break;
        case 'T': code = 3; break;
        default: code = 0; break; /* reference leaves `code` uninitialised: undefined input */
        }
        v = v * 4 + code;
    }
    return (uint8_t)v;
}

/* packing.hpp:77-92 */
void ko_pack(int K, const char* kmer, uint8_t* packed) {
    int i = 0, j = 0;
    for (; j <= K - 4; ++i, j += 4) packed[i] = pack_four(kmer + j);
    char block[4] = {'A', 'A', 'A', 'A'};
    int rem = K % 4;
    for (int r = 0; r < rem; ++r) block[r] = kmer[j + r];
    packed[i] = pack_four(block);
}

/* packing.hpp:16-48 + 94-107 (LUT of 4-mers), truncated to K chars. */
void ko_unpack(int K, const uint8_t* packed, char* kmer) {
    static const char bases[4] = {'A', 'C', 'G', 'T'};
    int P = packed_len(K);
    for (int i = 0; i < P; ++i) {
        for (int s = 0; s < 4; ++s) {
            int pos = 4 * i + s;
            if (pos < K) kmer[pos] = bases[(packed[i] >> (6 - 2 * s)) & 3];
        }
    }
}

/* pkmer_t.hpp:31-37 */
uint64_t ko_djb2(int K, const uint8_t* packed) {
    unsigned long h = 5381;
    int P = packed_len(K);
    for (int i = 0; i < P; ++i) h = packed[i] + (h << 5) + h;
    return (uint64_t)h;
}

/* kmer_t.hpp:51-53: pkmer_t(kmer_str().substr(1) + forwardExt()) */
void ko_next_kmer(int K, const uint8_t* rec, uint8_t* next_packed) {
    char buf[128];
    int P = packed_len(K);
    ko_unpack(K, rec, buf);
    memmove(buf, buf + 1, (size_t)(K - 1));
    buf[K - 1] = (char)rec[P + 1];
    ko_pack(K, buf, next_packed);
}

/* read_kmers.hpp:62-76: line = K chars, ' ', bwd, fwd, '\n'; kmer_pair(kmer, fb_ext) */
size_t ko_parse_text(int K, const char* text, size_t len, uint8_t* recs) {
    size_t line = (size_t)K + 4, n = len / line;
    int P = packed_len(K), R = P + 2;
    for (size_t i = 0; i < n; ++i) {
        const char* l = text + i * line;
        uint8_t* r = recs + i * (size_t)R;
        ko_pack(K, l, r);
        r[P] = (uint8_t)l[K + 1];     /* fb_ext[0] = backward */
        r[P + 1] = (uint8_t)l[K + 2]; /* fb_ext[1] = forward  */
    }
    return n;
}

/* ---- stock open addressing HashMap (README.md:95,99; test/distributed_hashmap_test.cpp:34-65) */
struct ko_table {
    int K, P, R;
    size_t size;
    uint8_t* data; /* size * R */
    uint8_t* used; /* size */
};

ko_table* ko_table_new(int K, size_t size) {
    ko_table* t = (ko_table*)calloc(1, sizeof(ko_table));
    if (!t) return NULL;
    t->K = K;
    t->P = packed_len(K);
    t->R = t->P + 2;
    t->size = size ? size : 1;
    t->data = (uint8_t*)malloc(t->size * (size_t)t->R);
    t->used = (uint8_t*)calloc(t->size, 1);
    if (!t->data || !t->used) {
        ko_table_free(t);
        return NULL;
    }
    return t;
}

void ko_table_free(ko_table* t) {
    if (!t) return;
    free(t->data);
    free(t->used);
    free(t);
}

/* insert: probe (hash + probe) % size until an unused slot; "HashMap is full" if none. */
int ko_table_insert(ko_table* t, const uint8_t* rec) {
    uint64_t h = ko_djb2(t->K, rec);
    for (size_t probe = 0; probe < t->size; ++probe) {
        size_t slot = (size_t)((h + probe) % t->size);
        if (!t->used[slot]) {
            t->used[slot] = 1;
            memcpy(t->data + slot * (size_t)t->R, rec, (size_t)t->R);
            return 1;
        }
    }
    return 0;
}

/* find: probe from the djb2 home slot, compare pkmer_t bytes (pkmer_t.hpp:41-43); an unused
 * slot ends the search (test/distributed_hashmap_test.cpp:59-61). */
int ko_table_find(const ko_table* t, const uint8_t* key, uint8_t* rec) {
    uint64_t h = ko_djb2(t->K, key);
    for (size_t probe = 0; probe < t->size; ++probe) {
        size_t slot = (size_t)((h + probe) % t->size);
        if (!t->used[slot]) return 0;
        const uint8_t* d = t->data + slot * (size_t)t->R;
        if (memcmp(d, key, (size_t)t->P) == 0) {
            memcpy(rec, d, (size_t)t->R);
            return 1;
        }
    }
    return 0;
}

void ko_free(void* p) { free(p); }

/* kmer_hash.cpp:21-55 + read_kmers.hpp:81-92 */
int ko_assemble(int K, const uint8_t* recs, size_t n, char** out, size_t* out_len,
                size_t* n_contigs, size_t* n_lookups, double* t_insert, double* t_walk) {
    int P = packed_len(K), R = P + 2;
    *out = NULL;
    *out_len = 0;
    ko_table* t = ko_table_new(K, 2 * n); /* kmer_hash.cpp:109 table = 2 * n_kmers, built before */
    if (!t) return -4;                    /* the timer starts (kmer_hash.cpp:119 vs :129)       */
    double t0 = now_s();
    size_t* starts = (size_t*)malloc((n ? n : 1) * sizeof(size_t));
    if (!starts) {
        ko_table_free(t);
        return -4;
    }
    size_t ns = 0;
    for (size_t i = 0; i < n; ++i) {
        if (!ko_table_insert(t, recs + i * (size_t)R)) {
            free(starts);
            ko_table_free(t);
            return -2;
        }
        if (recs[i * (size_t)R + P] == 'F') starts[ns++] = i; /* kmer_hash.cpp:27-31 */
    }
    double t1 = now_s();
    /* the output when walks are disjoint (every k-mer contributes <= 1 char, every contig K +
       '\n'); walks that overlap (malformed input) grow it */
    size_t cap = n + ns * ((size_t)K + 1) + 1;
    char* o = (char*)malloc(cap);
    if (!o) {
        free(starts);
        ko_table_free(t);
        return -4;
    }
    size_t pos = 0, lookups = 0;
    uint8_t cur[32], nxt[32];
    int rc = 0;
    for (size_t s = 0; s < ns && rc == 0; ++s) {
        if (pos + (size_t)K + 2 >= cap) {
            char* g = (char*)realloc(o, 2 * cap + (size_t)K + 2);
            if (!g) { rc = -4; break; }
            o = g;
            cap = 2 * cap + (size_t)K + 2;
        }
        memcpy(cur, recs + starts[s] * (size_t)R, (size_t)R);
        ko_unpack(K, cur, o + pos); /* extract_contig: front().kmer_str() */
        pos += (size_t)K;
        size_t steps = 0;
        while (cur[P + 1] != 'F') { /* kmer_hash.cpp:44 */
            if (pos + 2 >= cap) { /* overlapping walks: grow */
                char* g = (char*)realloc(o, 2 * cap);
                if (!g) { rc = -4; break; }
                o = g;
                cap *= 2;
            }
            o[pos++] = (char)cur[P + 1]; /* extract_contig: every non-F forward ext */
            ko_next_kmer(K, cur, nxt);
            if (!ko_table_find(t, nxt, cur)) { rc = -1; break; } /* kmer_hash.cpp:47-49 */
            ++lookups;
            if (++steps > n) { rc = -3; break; }
        }
        o[pos++] = '\n'; /* std::endl in output_results, kmer_hash.cpp:66 */
    }
    double t2 = now_s();
    free(starts);
    ko_table_free(t);
    if (rc) {
        free(o);
        return rc;
    }
    o[pos] = 0;
    *out = o;
    *out_len = pos;
    if (n_contigs) *n_contigs = ns;
    if (n_lookups) *n_lookups = lookups;
    if (t_insert) *t_insert = t1 - t0;
    if (t_walk) *t_walk = t2 - t1;
    return 0;
}
