// kmer_t.hpp (drop-in) — layout and methods of the reference's kmer_t.hpp:6-82:
// { pkmer_t kmer; char fb_ext[2]; }, fb_ext[0] = backward, fb_ext[1] = forward extension.
#pragma once
#include <cstdio>
#include <string>

#include "pkmer_t.hpp"

struct kmer_pair {
    pkmer_t kmer;
    char fb_ext[2];

    std::string kmer_str() const noexcept { return kmer.get(); }
    std::string fb_ext_str() const noexcept { return std::string(fb_ext, 2); }
    // kmer_t.hpp:51-53, computed as a 2-bit shift of the packed key (no string round trip)
    pkmer_t next_kmer() const noexcept {
        pkmer_t n;
        kh_next_kmer(KMER_LEN, reinterpret_cast<const uint8_t*>(this), n.data);
        return n;
    }
    pkmer_t last_kmer() const noexcept {
        return pkmer_t(std::string(1, backwardExt()) + kmer_str().substr(0, KMER_LEN - 1));
    }
    char forwardExt() const noexcept { return fb_ext[1]; }
    char backwardExt() const noexcept { return fb_ext[0]; }
    void print() const noexcept { printf("%s %s\n", kmer_str().c_str(), fb_ext_str().c_str()); }
    uint64_t hash() const noexcept { return kmer.hash(); }

    kmer_pair(const std::string& k, const std::string& fb) { init(k, fb); }
    kmer_pair() = default;
    kmer_pair(const kmer_pair&) = default;
    kmer_pair& operator=(const kmer_pair&) = default;

    void init(const std::string& k, const std::string& fb) {
        if (k.length() != KMER_LEN || fb.length() != 2) {
            fprintf(stderr, "error: tried to initialize a kmer pair with too short a string.\n");
            return;
        }
        kmer = pkmer_t(k);
        fb_ext[0] = fb[0];
        fb_ext[1] = fb[1];
    }
    void init(const kmer_pair& o) { *this = o; }

    bool operator==(const kmer_pair& o) const noexcept {
        return o.kmer == kmer && fb_ext[0] == o.fb_ext[0] && fb_ext[1] == o.fb_ext[1];
    }
    bool operator!=(const kmer_pair& o) const noexcept { return !(o == *this); }
};
static_assert(sizeof(kmer_pair) == PACKED_KMER_LEN + 2, "kmer_pair must match the reference layout");
