/* asan_main.c — TEST INFRASTRUCTURE ONLY: the oracle under AddressSanitizer (CPU).
 *
 * Built by `make -C oracle asan` with -fsanitize=address into oracle/_asan/oracle_asan and run by
 * tests/test_oracle.py::test_oracle_asan_merging_walks. Reads a fixed-width k-mer text file
 * (read_kmers.hpp:54-79 layout), assembles it with the serial oracle (ko_assemble) and the
 * thread-parallel one (ko_assemble_par, P ranks), checks the two texts agree and writes the
 * serial text to the output file. Round 5's GPU box lost a test process to a SIGSEGV that was a
 * heap overflow in ko_assemble on overlapping walks (text longer than n + starts * (K + 1));
 * this run keeps that class of bug visible on the CPU. Exit status: 0 ok, 1 usage / IO, 2 oracle
 * error code, 3 serial and parallel texts differ. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "kmer_oracle.h"

static char* slurp(const char* path, size_t* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* b = (char*)malloc((size_t)n + 1);
    if (b && fread(b, 1, (size_t)n, f) != (size_t)n) {
        free(b);
        b = NULL;
    }
    fclose(f);
    *len = (size_t)n;
    return b;
}

int main(int argc, char** argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s K P in.txt out.dat\n", argv[0]);
        return 1;
    }
    const int K = atoi(argv[1]), P = atoi(argv[2]);
    size_t len = 0;
    char* text = slurp(argv[3], &len);
    if (!text) return 1;
    const size_t R = (size_t)(K + 3) / 4 + 2, nmax = len / (size_t)(K + 4) + 1;
    uint8_t* recs = (uint8_t*)malloc(nmax * R);
    const size_t n = ko_parse_text(K, text, len, recs);
    char *a = NULL, *b = NULL;
    size_t la = 0, lb = 0, nc = 0, nl = 0;
    double ti, tw;
    int rc = ko_assemble(K, recs, n, &a, &la, &nc, &nl, &ti, &tw);
    if (rc) return 2;
    rc = ko_assemble_par(K, recs, n, P, &b, &lb, &nc, &nl, &ti, &tw);
    if (rc) return 2;
    const int same = la == lb && memcmp(a, b, la) == 0;
    FILE* o = fopen(argv[4], "wb");
    if (!o || fwrite(a, 1, la, o) != la) return 1;
    fclose(o);
    printf("records %zu contigs %zu bytes %zu\n", n, nc, la);
    ko_free(a);
    ko_free(b);
    free(recs);
    free(text);
    return same ? 0 : 3;
}
