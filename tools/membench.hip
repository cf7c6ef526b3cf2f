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

int main(int argc, char** argv) {
    const double gib[] = {0.25, 1, 2, 4, 6.4, 16};
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
    for (double g : gib) {
        const uint64_t nslots = (uint64_t)(g * (1ull << 30) / 16);
        struct Case { const char* name; int grid; int iters; } cases[] = {
            {"gather16", 16384, 64}, {"chase16", 2048, 256}, {"cas8", 16384, 16},
            {"cas8w", 16384, 16}, {"store8sc1", 16384, 16}};
        for (auto& c : cases) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipEventRecord(a));
                if (c.name[0] == 'g') k_gather16<<<c.grid, threads>>>(t, nslots, c.iters, sink);
                else if (c.name[1] == 'h') k_chase16<<<c.grid, threads>>>(t, nslots, c.iters, sink);
                else if (c.name[0] == 'c') k_cas8<<<c.grid, threads>>>(t, nslots, c.iters, c.name[4] == 'w', sink);
                else k_store8<<<c.grid, threads>>>(t, nslots, c.iters);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            const double ops = (double)c.grid * threads * c.iters;
            printf("{\"case\": \"%s\", \"table_gib\": %.2f, \"lanes\": %d, \"ops\": %.0f, \"ms\": %.3f, "
                   "\"gops\": %.3f}\n", c.name, g, c.grid * threads, ops, best, ops / best / 1e6);
            fflush(stdout);
        }
    }
    return 0;
}
