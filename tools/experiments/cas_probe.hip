// Random 8-B atomicCAS throughput vs target footprint (is a small, L2-resident region faster than
// the HBM-wide table?), and plain random 16-B store throughput for comparison.
// hipcc --offload-arch=gfx950 -O3 -o /tmp/cp tools/cas_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}
// every block works in region (blockIdx % nreg); each lane does `per` CAS at random slots of it
__global__ void k_cas(unsigned long long* t, uint64_t region_slots, uint64_t nreg, int per) {
    const uint64_t r = blockIdx.x % nreg;
    unsigned long long* base = t + r * region_slots;
    uint64_t x = mix(blockIdx.x * 1024 + threadIdx.x + 1);
    for (int i = 0; i < per; ++i) {
        x = mix(x + i);
        const uint64_t s = (x >> 16) % region_slots;
        atomicCAS(base + s, ~0ull, x);
    }
}
__global__ void k_st(unsigned long long* t, uint64_t region_slots, uint64_t nreg, int per) {
    const uint64_t r = blockIdx.x % nreg;
    unsigned long long* base = t + r * region_slots;
    uint64_t x = mix(blockIdx.x * 1024 + threadIdx.x + 1);
    for (int i = 0; i < per; ++i) {
        x = mix(x + i);
        const uint64_t s = (x >> 16) % region_slots;
        base[s] = x;
    }
}
int main() {
    const uint64_t total = 800ull << 20;  // 800M slots = 6.4 GB
    unsigned long long* t;
    if (hipMalloc(&t, total * 8) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int per = 64;
    const unsigned grid = 8192, blk = 256;
    const double ops = (double)grid * blk * per;
    for (uint64_t reg_bytes : {256ull << 10, 1ull << 20, 2ull << 20, 4ull << 20, 16ull << 20, 256ull << 20, (unsigned long long)(total * 8)}) {
        const uint64_t rs = reg_bytes / 8;
        uint64_t nreg = total / rs;
        if (nreg > grid) nreg = grid;
        for (int kind = 0; kind < 2; ++kind) {
            (void)hipMemset(t, 0xff, total * 8);
            auto go = [&] {
                if (kind == 0) k_cas<<<grid, blk>>>(t, rs, nreg, per);
                else k_st<<<grid, blk>>>(t, rs, nreg, per);
            };
            go();
            hipEventRecord(e0);
            go();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("region %8llu KB x %5llu regions  %s  %.1f G/s\n", (unsigned long long)(reg_bytes >> 10),
                   (unsigned long long)nreg, kind == 0 ? "CAS  " : "store", ops / ms / 1e6);
        }
    }
    return 0;
}
