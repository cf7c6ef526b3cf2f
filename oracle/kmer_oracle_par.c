/* kmer_oracle_par.c — TEST INFRASTRUCTURE / CPU BASELINE ONLY (see kmer_oracle.h).
 *
 * Thread-parallel restatement of the reference's DistributedHashMap path on the host cores
 * (BASELINE.md "CPU baseline plan" item 2): P threads play the P UPC++ ranks.
 *
 *   rank r reads the block split of read_kmers.hpp:55-58 (split = ceil(n/P), start = split*r);
 *   insert_all (hash_map.hpp:55-80): every rank partitions its records by owner into one batch
 *     per target rank (hash_map.hpp:57-62), then every owner applies the batches addressed to it
 *     (the RPC bodies of hash_map.hpp:38-46, run by the owner thread itself: no locks), barrier
 *     (hash_map.hpp:79);
 *   start nodes (kmer_hash.cpp:27-31): backward extension 'F', in block (file) order;
 *   assemble_contigs (kmer_hash.cpp:38-55): every rank walks its own start nodes; find
 *     (hash_map.hpp:83-107) reads the owner's shard directly (shared memory stands in for the
 *     RPC); a missing k-mer is an error (kmer_hash.cpp:47-49).
 *
 * Each shard is the stock open-addressing table of kmer_oracle.c (djb2 home, linear probing,
 * 2x the k-mers it receives = load 0.5). The owner is a multiplicative mix of the djb2 hash
 * (the reference uses std::hash<std::string> % P, hash_map.hpp:28-30; a plain djb2 % P would
 * correlate with the shard's own djb2 % size slot and cluster it). Ownership never changes the
 * output: the concatenation of the ranks' texts in rank order is the serial test_0.dat.
 */
#include "kmer_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int owner_of(uint64_t h, int P) {
    return (int)(((h * 0x9E3779B97F4A7C15ull) >> 32) % (uint64_t)P);
}

typedef struct {
    int K, P, R, np;          /* np = packed bytes */
    const uint8_t* recs;
    size_t n;
    pthread_barrier_t bar;
    size_t** batch;           /* batch[r*P + o] = record indices rank r sends to owner o */
    size_t* batch_n;
    ko_table** shard;
    int rc;                   /* first error (shared; set under lock) */
    pthread_mutex_t m;
    double t0, t1, t2;
    char** text;              /* per rank */
    size_t* text_len;
    size_t* n_contigs;
    size_t* n_lookups;
} par_job;

typedef struct {
    par_job* j;
    int r;
} par_arg;

static void set_rc(par_job* j, int rc) {
    pthread_mutex_lock(&j->m);
    if (!j->rc) j->rc = rc;
    pthread_mutex_unlock(&j->m);
}

static int append(char** buf, size_t* len, size_t* cap, const char* s, size_t k) {
    if (*len + k > *cap) {
        size_t nc = *cap ? *cap : 4096;
        while (nc < *len + k) nc *= 2;
        char* nb = (char*)realloc(*buf, nc);
        if (!nb) return -4;
        *buf = nb;
        *cap = nc;
    }
    memcpy(*buf + *len, s, k);
    *len += k;
    return 0;
}

static void* par_rank(void* argp) {
    par_arg* a = (par_arg*)argp;
    par_job* j = a->j;
    const int r = a->r, P = j->P, K = j->K, R = j->R, np = j->np;
    size_t split = (j->n + (size_t)P - 1) / (size_t)P;
    size_t b = split * (size_t)r, e = b + split;
    if (b > j->n) b = j->n;
    if (e > j->n) e = j->n;

    if (r == 0) j->t0 = now_s();
    /* ---- insert_all: partition by owner (one batch per target), collect start nodes ---- */
    uint8_t* own = (uint8_t*)malloc((e - b) ? (e - b) : 1);
    size_t* cnt = (size_t*)calloc((size_t)P, sizeof(size_t));
    size_t* starts = NULL;
    size_t ns = 0;
    int rc = (own && cnt) ? 0 : -4;
    for (size_t i = b; i < e && !rc; ++i) {
        const uint8_t* rec = j->recs + i * (size_t)R;
        int o = owner_of(ko_djb2(K, rec), P);
        own[i - b] = (uint8_t)o;
        ++cnt[o];
        if (rec[np] == 'F') ++ns;
    }
    if (!rc) {
        starts = (size_t*)malloc((ns ? ns : 1) * sizeof(size_t));
        if (!starts) rc = -4;
        for (int o = 0; o < P && !rc; ++o) {
            j->batch[(size_t)r * P + o] = (size_t*)malloc((cnt[o] ? cnt[o] : 1) * sizeof(size_t));
            if (!j->batch[(size_t)r * P + o]) rc = -4;
        }
    }
    if (!rc) {
        size_t s = 0;
        for (size_t i = b; i < e; ++i) {
            int o = own[i - b];
            j->batch[(size_t)r * P + o][j->batch_n[(size_t)r * P + o]++] = i;
            if (j->recs[i * (size_t)R + np] == 'F') starts[s++] = i;
        }
    }
    if (rc) set_rc(j, rc);
    pthread_barrier_wait(&j->bar);
    /* ---- every owner applies the batches addressed to it, in rank order ---- */
    if (!j->rc) {
        size_t tot = 0;
        for (int s = 0; s < P; ++s) tot += j->batch_n[(size_t)s * P + r];
        ko_table* t = ko_table_new(K, 2 * tot);
        j->shard[r] = t;
        if (!t) set_rc(j, -4);
        for (int s = 0; s < P && t; ++s) {
            const size_t* idx = j->batch[(size_t)s * P + r];
            size_t m = j->batch_n[(size_t)s * P + r];
            for (size_t q = 0; q < m; ++q)
                if (!ko_table_insert(t, j->recs + idx[q] * (size_t)R)) {
                    set_rc(j, -2);
                    break;
                }
        }
    }
    pthread_barrier_wait(&j->bar); /* hash_map.hpp:79 */
    if (r == 0) j->t1 = now_s();
    /* ---- assemble_contigs over this rank's start nodes ---- */
    char* o = NULL;
    size_t ol = 0, oc = 0, lookups = 0;
    if (!j->rc) {
        uint8_t cur[32], nxt[32];
        char kbuf[128];
        for (size_t s = 0; s < ns && !rc; ++s) {
            memcpy(cur, j->recs + starts[s] * (size_t)R, (size_t)R);
            ko_unpack(K, cur, kbuf);
            if ((rc = append(&o, &ol, &oc, kbuf, (size_t)K))) break;
            size_t steps = 0;
            while (cur[np + 1] != 'F') {
                char c = (char)cur[np + 1];
                if ((rc = append(&o, &ol, &oc, &c, 1))) break;
                ko_next_kmer(K, cur, nxt);
                const ko_table* t = j->shard[owner_of(ko_djb2(K, nxt), P)];
                if (!ko_table_find(t, nxt, cur)) { rc = -1; break; }
                ++lookups;
                if (++steps > j->n) { rc = -3; break; }
            }
            if (!rc) rc = append(&o, &ol, &oc, "\n", 1);
        }
        if (rc) set_rc(j, rc);
    }
    pthread_barrier_wait(&j->bar);
    if (r == 0) j->t2 = now_s();
    j->text[r] = o;
    j->text_len[r] = ol;
    j->n_contigs[r] = ns;
    j->n_lookups[r] = lookups;
    free(own);
    free(cnt);
    free(starts);
    return NULL;
}

int ko_assemble_par(int K, const uint8_t* recs, size_t n, int P, char** out, size_t* out_len,
                    size_t* n_contigs, size_t* n_lookups, double* t_insert, double* t_walk) {
    *out = NULL;
    *out_len = 0;
    if (P < 1 || P > 256) return -5;
    par_job j;
    memset(&j, 0, sizeof j);
    j.K = K;
    j.P = P;
    j.np = (K + 3) / 4;
    j.R = j.np + 2;
    j.recs = recs;
    j.n = n;
    pthread_barrier_init(&j.bar, NULL, (unsigned)P);
    pthread_mutex_init(&j.m, NULL);
    j.batch = (size_t**)calloc((size_t)P * P, sizeof(size_t*));
    j.batch_n = (size_t*)calloc((size_t)P * P, sizeof(size_t));
    j.shard = (ko_table**)calloc((size_t)P, sizeof(ko_table*));
    j.text = (char**)calloc((size_t)P, sizeof(char*));
    j.text_len = (size_t*)calloc((size_t)P, sizeof(size_t));
    j.n_contigs = (size_t*)calloc((size_t)P, sizeof(size_t));
    j.n_lookups = (size_t*)calloc((size_t)P, sizeof(size_t));
    pthread_t* th = (pthread_t*)calloc((size_t)P, sizeof(pthread_t));
    par_arg* args = (par_arg*)calloc((size_t)P, sizeof(par_arg));
    int rc = 0;
    if (!j.batch || !j.batch_n || !j.shard || !j.text || !j.text_len || !j.n_contigs ||
        !j.n_lookups || !th || !args)
        rc = -4;
    int started = 0;
    for (int r = 0; r < P && !rc; ++r) {
        args[r].j = &j;
        args[r].r = r;
        if (pthread_create(&th[r], NULL, par_rank, &args[r])) rc = -4;
        else ++started;
    }
    if (rc && started) {
        /* cannot run the barriers short-handed: this only happens on thread exhaustion */
        abort();
    }
    for (int r = 0; r < started; ++r) pthread_join(th[r], NULL);
    if (!rc) rc = j.rc;
    if (!rc) {
        size_t tot = 0, nc = 0, nl = 0;
        for (int r = 0; r < P; ++r) {
            tot += j.text_len[r];
            nc += j.n_contigs[r];
            nl += j.n_lookups[r];
        }
        char* o = (char*)malloc(tot + 1);
        if (!o) rc = -4;
        else {
            size_t pos = 0;
            for (int r = 0; r < P; ++r) {
                if (j.text_len[r]) memcpy(o + pos, j.text[r], j.text_len[r]);
                pos += j.text_len[r];
            }
            o[pos] = 0;
            *out = o;
            *out_len = pos;
            if (n_contigs) *n_contigs = nc;
            if (n_lookups) *n_lookups = nl;
            if (t_insert) *t_insert = j.t1 - j.t0;
            if (t_walk) *t_walk = j.t2 - j.t1;
        }
    }
    for (int r = 0; j.text && r < P; ++r) free(j.text[r]);
    for (size_t q = 0; j.batch && q < (size_t)P * P; ++q) free(j.batch[q]);
    for (int r = 0; j.shard && r < P; ++r) ko_table_free(j.shard[r]);
    free(j.batch);
    free(j.batch_n);
    free(j.shard);
    free(j.text);
    free(j.text_len);
    free(j.n_contigs);
    free(j.n_lookups);
    free(th);
    free(args);
    pthread_barrier_destroy(&j.bar);
    pthread_mutex_destroy(&j.m);
    return rc;
}
