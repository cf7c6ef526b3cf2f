// read_kmers.hpp (drop-in) — kmer_size / line_count / read_kmers / extract_contig with the
// semantics of the reference's read_kmers.hpp:14-92 (block split, fixed K+4-byte lines).
#pragma once
#include <cstdio>
#include <fstream>
#include <list>
#include <stdexcept>
#include <string>
#include <vector>

#include "kmer_t.hpp"

inline int kmer_size(const std::string& fname) {
    std::ifstream fin(fname);
    if (!fin.is_open()) throw std::runtime_error("kmer_size: could not open " + fname);
    std::string buf;
    fin >> buf;
    return (int)buf.size();
}

inline size_t line_count(const std::string& fname) {
    FILE* f = fopen(fname.c_str(), "r");
    if (!f) throw std::runtime_error("line_count: could not open " + fname);
    size_t n = 0;
    char buf[1 << 16];
    size_t r;
    while ((r = fread(buf, 1, sizeof buf, f)) > 0)
        for (size_t i = 0; i < r; ++i) n += buf[i] == '\n';
    fclose(f);
    return n;
}

inline std::vector<kmer_pair> read_kmers(const std::string& fname, int nprocs = 1, int rank = 0) {
    const size_t n = line_count(fname);
    const size_t split = (n + nprocs - 1) / nprocs;
    const size_t start = std::min(split * (size_t)rank, n);
    const size_t size = std::min(split, n - start);
    const size_t line = KMER_LEN + 4;
    std::vector<char> buf(line * size);
    FILE* f = fopen(fname.c_str(), "r");
    if (!f) throw std::runtime_error("read_kmers: could not open " + fname);
    fseek(f, (long)(line * start), SEEK_SET);
    const size_t got = fread(buf.data(), 1, buf.size(), f);
    fclose(f);
    if (got != buf.size()) throw std::runtime_error("read_kmers: short read of " + fname);
    std::vector<kmer_pair> kmers(size);
    uint64_t parsed = 0;
    if (kh_pack_text(KMER_LEN, buf.data(), buf.size(), reinterpret_cast<uint8_t*>(kmers.data()),
                     &parsed) != KH_OK)
        throw std::runtime_error(kh_last_error());
    return kmers;
}

inline std::string extract_contig(const std::list<kmer_pair>& contig) {
    std::string s = contig.front().kmer_str();
    for (const auto& k : contig)
        if (k.forwardExt() != 'F') s += k.forwardExt();
    return s;
}
