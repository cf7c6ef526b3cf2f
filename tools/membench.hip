// membench.hip — random-access ceilings of the MI355X memory system for the k-mer table's access
// shapes (measurement tool; not part of the library). Prints one JSON object per case:
//   gather16   independent random 16-B loads (a table probe without the dependency)
//   chase16    dependent random 16-B loads, one chain per lane (the contig walk's shape)
//   cas8       random 64-bit atomicCAS that always fails (a probe of an occupied slot)
//   cas8w      random 64-bit atomicCAS that succeeds (claiming an empty slot)
//   store8sc1  random 8-B write-through stores
// over table sizes from 256 MiB to 16 GiB. Build: hipcc --offload-arch=gfx950 -O3 membench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                         \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t h) {
    h ^= h >> 33;
    h *= 0xff51afd7ed558ccdull;
    h ^= h >> 33;
    h *= 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 33;
    return h;
}

__global__ void k_init(uint64_t* t, uint64_t words) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < words; i += gridDim.x * 256ull) t[i] = mix(i + 1);
}

__global__ void k_gather16(const uint64_t* t, uint64_t nslots, int iters, uint64_t* sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        const uint64_t s = __umul64hi(mix(tid * 1000003ull + i), nslots);
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(t + 2 * s);
        acc ^= v.x + v.y;
    }
    if (acc == 42) sink[0] = acc;
}

__global__ void k_chase16(const uint64_t* t, uint64_t nslots, int iters, uint64_t* sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t x = mix(tid + 7);
    for (int i = 0; i < iters; ++i) {
        const uint64_t s = __umul64hi(mix(x), nslots);
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(t + 2 * s);
        x = v.x ^ v.y ^ i;
    }
    if (x == 42) sink[0] = x;
}

__global__ void k_cas8(uint64_t* t, uint64_t nslots, int iters, int succeed, uint64_t* sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        const uint64_t s = __umul64hi(mix(tid * 1000003ull + i), nslots);
        unsigned long long* p = reinterpret_cast<unsigned long long*>(t + 2 * s);
        // succeed: compare with the current value; fail: with a value never stored
        const unsigned long long cmp = succeed ? *p : 1ull;
        acc ^= atomicCAS(p, cmp, cmp + 2);
    }
    if (acc == 42) sink[0] = acc;
}

__global__ void k_store8(uint64_t* t, uint64_t nslots, int iters) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        const uint64_t s = __umul64hi(mix(tid * 1000003ull + i), nslots);
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(t + 2 * s + 1), (unsigned long long)tid,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}


// dependent random loads of a G*16-B aligned block, G lanes per chain (lane q of the group loads
// bytes 16q..16q+15): the cooperative-probe shape of a walk that fetches a whole bucket per step
template <int G>
__global__ void k_chaseg(const uint64_t* t, uint64_t nblocks, int iters, uint64_t* sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint32_t q = threadIdx.x & (G - 1);
    uint64_t x = mix(tid / G + 7);
    for (int i = 0; i < iters; ++i) {
        const uint64_t s = __umul64hi(mix(x), nblocks);
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(t + 2 * (s * G + q));
        uint64_t y = v.x ^ v.y;
#pragma unroll
        for (int o = 1; o < G; o <<= 1) y ^= __shfl_xor(y, o, G);
        x = y ^ i;
    }
    if (x == 42) sink[0] = x;
}

int main(int argc, char** argv) {
    // "calib": one pass over a 6.4 GB table per case, for PMC calibration of random access widths
    const bool calib = argc > 1 && !strcmp(argv[1], "calib");
    const double gib_all[] = {0.25, 1, 2, 4, 6.4, 16};
    const double gib_cal[] = {6.4};
    const double* gib_p = calib ? gib_cal : gib_all;
    const int ngib = calib ? 1 : 6;
    const uint64_t maxw = (uint64_t)(16.0 * (1ull << 30) / 8);
    uint64_t *t, *sink;
    CK(hipMalloc(&t, maxw * 8));
    CK(hipMalloc(&sink, 64));
    k_init<<<8192, 256>>>(t, maxw);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int threads = 256;
    for (int gi = 0; gi < ngib; ++gi) {
        const double g = gib_p[gi];
        const uint64_t nslots = (uint64_t)(g * (1ull << 30) / 16);
        struct Case { const char* name; int grid; int iters; } cases[] = {
            {"gather16", 16384, 64}, {"chase16", 2048, 256}, {"cas8", 16384, 16},
            {"cas8w", 16384, 16}, {"store8sc1", 16384, 16},
            {"chase32p", 4096, 256}, {"chase64q", 8192, 256}, {"chase128o", 16384, 256},
            {"chase16w", 8192, 256}};
        for (auto& c : cases) {
            float best = 1e30f;
            for (int rep = 0; rep < (calib ? 1 : 3); ++rep) {
                CK(hipEventRecord(a));
                if (c.name[0] == 'g') k_gather16<<<c.grid, threads>>>(t, nslots, c.iters, sink);
                else if (!strcmp(c.name, "chase32p")) k_chaseg<2><<<c.grid, threads>>>(t, nslots / 2, c.iters, sink);
                else if (!strcmp(c.name, "chase64q")) k_chaseg<4><<<c.grid, threads>>>(t, nslots / 4, c.iters, sink);
                else if (!strcmp(c.name, "chase128o")) k_chaseg<8><<<c.grid, threads>>>(t, nslots / 8, c.iters, sink);
                else if (c.name[1] == 'h') k_chase16<<<c.grid, threads>>>(t, nslots, c.iters, sink);
                else if (c.name[0] == 'c') k_cas8<<<c.grid, threads>>>(t, nslots, c.iters, c.name[4] == 'w', sink);
                else k_store8<<<c.grid, threads>>>(t, nslots, c.iters);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            int grp = !strcmp(c.name, "chase32p") ? 2 : !strcmp(c.name, "chase64q") ? 4
                    : !strcmp(c.name, "chase128o") ? 8 : 1;
            const double ops = (double)c.grid * threads / grp * c.iters;
            printf("{\"case\": \"%s\", \"table_gib\": %.2f, \"lanes\": %d, \"ops\": %.0f, \"ms\": %.3f, "
                   "\"gops\": %.3f}\n", c.name, g, c.grid * threads, ops, best, ops / best / 1e6);
            fflush(stdout);
        }
    }
    return 0;
}
