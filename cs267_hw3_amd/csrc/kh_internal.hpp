// kh_internal.hpp — symbols shared between the library's translation units (not part of the ABI).
#pragma once

// Sets the thread-local message returned by kh_last_error().
void kh_set_error_internal(const char* msg);

// Device copies of a synthetic generator's per-contig arrays (kh_gen.hip).
#include <stdint.h>
namespace kh {
struct GenView;
}
struct kh_gen_dev;
// records at positions [pb, pe) into device memory (R bytes each) on `stream` (a hipStream_t);
// dev[d] caches the arrays on device d (made on first use on the current device)
static constexpr int KH_GEN_MAX_DEVICES = 64;
int kh_gen_dev_records(const kh::GenView& v, kh_gen_dev** dev, uint64_t pb, uint64_t pe, uint8_t* out,
                       void* stream);
void kh_gen_dev_free(kh_gen_dev* d);
