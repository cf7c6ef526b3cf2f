// Microbenchmark: cost of per-block device-scope atomics vs grid size (same address, spread over
// 8 lines), and of a byte-state scan, on one GPU. hipcc --offload-arch=gfx950 -O3 -o /tmp/ap atomic_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_empty(unsigned long long* a) {}
__global__ void k_same(unsigned long long* a) {
    if (threadIdx.x == 0) atomicAdd(a, 1ull);
}
__global__ void k_spread(unsigned long long* a) {
    if (threadIdx.x == 0) atomicAdd(a + (blockIdx.x % 8) * 16, 1ull);
}
__global__ void k_same_ret(unsigned long long* a, unsigned long long* o) {
    if (threadIdx.x == 0) o[blockIdx.x] = atomicAdd(a, 1ull);
}
__global__ void k_scan8(uint8_t* st, uint64_t n, unsigned long long* a) {
    uint64_t c = 0;
    for (int j = 0; j < 8; ++j) {
        uint64_t i = (uint64_t)blockIdx.x * 2048 + j * 256 + threadIdx.x;
        if (i < n) { uint8_t s = st[i]; c += s != 6; st[i] = s; }
    }
    __syncthreads();
    if (threadIdx.x == 0 && c) atomicAdd(a, c);
}
__global__ void k_scan8_nowrite(const uint8_t* st, uint64_t n, unsigned long long* a) {
    uint64_t c = 0;
    for (int j = 0; j < 8; ++j) {
        uint64_t i = (uint64_t)blockIdx.x * 2048 + j * 256 + threadIdx.x;
        if (i < n) c += st[i] != 6;
    }
    if (c) atomicAdd(a, c);
}

int main() {
    unsigned long long *a, *o;
    uint8_t* st;
    const uint64_t n = 2000000;
    hipMalloc(&a, 1 << 16);
    hipMalloc(&o, 1 << 20);
    hipMalloc(&st, n);
    hipMemset(a, 0, 1 << 16);
    hipMemset(st, 6, n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        hipEventRecord(e0);
        for (int i = 0; i < 20; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %8.2f us\n", name, ms * 1e3 / 20);
    };
    for (unsigned g : {256u, 977u, 4096u}) {
        printf("grid %u\n", g);
        timeit("  empty", [&] { k_empty<<<g, 256>>>(a); });
        timeit("  same-address atomic", [&] { k_same<<<g, 256>>>(a); });
        timeit("  same-address atomic ret", [&] { k_same_ret<<<g, 256>>>(a, o); });
        timeit("  8-line spread atomic", [&] { k_spread<<<g, 256>>>(a); });
    }
    timeit("scan8 2M bytes r+w (977 blk)", [&] { k_scan8<<<977, 256>>>(st, n, a); });
    timeit("scan8 2M bytes r (977 blk)", [&] { k_scan8_nowrite<<<977, 256>>>(st, n, a); });
    return 0;
}
