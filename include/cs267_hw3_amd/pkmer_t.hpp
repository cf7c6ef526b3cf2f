// pkmer_t.hpp (drop-in) — layout and methods of the reference's pkmer_t.hpp:5-51.
#pragma once
#include <cstring>
#include <string>

#include "packing.hpp"

struct pkmer_t {
    unsigned char data[PACKED_KMER_LEN];

    std::string get() const noexcept {
        char buf[KMER_LEN];
        unpackKmer(data, buf);
        return std::string(buf, KMER_LEN);
    }
    // djb2 over the packed bytes (pkmer_t.hpp:31-37)
    uint64_t hash() const noexcept { return kh_djb2(KMER_LEN, data); }

    pkmer_t(const std::string& kmer) { packKmer(kmer.data(), data); }
    pkmer_t() = default;
    pkmer_t(const pkmer_t&) = default;
    pkmer_t& operator=(const pkmer_t&) = default;

    bool operator==(const pkmer_t& o) const noexcept { return std::memcmp(o.data, data, PACKED_KMER_LEN) == 0; }
    bool operator!=(const pkmer_t& o) const noexcept { return !(*this == o); }

    void init(const unsigned char d[PACKED_KMER_LEN]) { std::memcpy(data, d, PACKED_KMER_LEN); }
};
static_assert(sizeof(pkmer_t) == PACKED_KMER_LEN, "pkmer_t must stay byte-packed");
