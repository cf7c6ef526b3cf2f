// kh_gen.hip — the synthetic generator's records produced on the GPU (kh_gen_records_dev): one
// thread per record position, the same pure functions as the host generator (kh_gen.hpp), so a
// C3/C4-size dataset (200M-1B records) appears in HBM in milliseconds instead of a minute of host
// work plus a PCIe upload. Test and benchmark input only; the table never calls it.
#include <hip/hip_runtime.h>

#include "../../include/kmer_hash_amd.h"
#include "kh_gen.hpp"
#include "kh_internal.hpp"

struct kh_gen_dev {
    int device = -1;
    uint32_t* len = nullptr;
    uint64_t* off = nullptr;
    uint32_t* salt = nullptr;
    uint64_t* nb = nullptr;
};

namespace {

constexpr int GB = 256;

__global__ __launch_bounds__(GB) void k_gen_records(kh::GenView v, uint64_t pb, uint64_t n, uint8_t* out) {
    const uint32_t R = (uint32_t)v.kp.R;
    for (uint64_t q = (uint64_t)blockIdx.x * GB + threadIdx.x; q < n; q += (uint64_t)gridDim.x * GB) {
        uint8_t rec[2 * ((kh::KMAX + 3) / 4) + 2];
        v.record(pb + q, rec);
        uint8_t* o = out + q * R;
        for (uint32_t b = 0; b < R; ++b) o[b] = rec[b];
    }
}

template <class T>
hipError_t upload(T** d, const T* h, uint64_t n) {
    hipError_t e = hipMalloc((void**)d, (n ? n : 1) * sizeof(T));
    if (e != hipSuccess) return e;
    return n ? hipMemcpy(*d, h, n * sizeof(T), hipMemcpyHostToDevice) : hipSuccess;
}

}  // namespace

void kh_gen_dev_free(kh_gen_dev* d) {
    if (!d) return;
    for (void* p : {(void*)d->len, (void*)d->off, (void*)d->salt, (void*)d->nb})
        if (p) (void)hipFree(p);
    delete d;
}

int kh_gen_dev_records(const kh::GenView& v, kh_gen_dev** dev, uint64_t pb, uint64_t pe, uint8_t* out,
                       void* stream) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || cur < 0 || cur >= KH_GEN_MAX_DEVICES) return KH_ERR_HIP;
    dev += cur;
    if (!*dev) {
        kh_gen_dev* d = new kh_gen_dev();
        d->device = cur;
        hipError_t e = upload(&d->len, v.len, v.C);
        if (e == hipSuccess) e = upload(&d->off, v.off, v.C + 1);
        if (e == hipSuccess) e = upload(&d->salt, v.salt, v.C);
        if (e == hipSuccess && v.nb) e = upload(&d->nb, v.nb, v.C);
        if (e != hipSuccess) {
            kh_gen_dev_free(d);
            kh_set_error_internal(hipGetErrorString(e));
            return KH_ERR_HIP;
        }
        *dev = d;
    }
    kh::GenView dv = v;
    dv.len = (*dev)->len;
    dv.off = (*dev)->off;
    dv.salt = (*dev)->salt;
    dv.nb = (*dev)->nb;
    const uint64_t n = pe - pb;
    const unsigned grid = (unsigned)((n + GB - 1) / GB < 65536 ? (n + GB - 1) / GB : 65536);
    hipLaunchKernelGGL(k_gen_records, dim3(grid), dim3(GB), 0, (hipStream_t)stream, dv, pb, n, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        kh_set_error_internal(hipGetErrorString(e));
        return KH_ERR_HIP;
    }
    return KH_OK;
}
