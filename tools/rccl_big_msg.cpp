// rccl_big_msg.cpp — one-rank reproducer for large per-peer RCCL messages.
//
// The sharded insert splits every per-peer message at 512 MiB (rccl_comm.hpp, dist.py) because a
// one-rank self-exchange of the whole C3 word array (3.2 GB) came back corrupted. This program pins
// which layer does it: a grouped ncclSend/ncclRecv to self (the pattern RcclComm::all_to_all and
// torch's all_to_all use) of 1 GiB .. 3.2 GiB, sent as u64 elements and as bytes, each checked word
// by word on the device. tools/rccl_big_msg.py runs the same sizes through torch.distributed.
//
//   hipcc --offload-arch=gfx950 -O2 rccl_big_msg.cpp -lrccl -o rccl_big_msg && ./rccl_big_msg
// Prints one JSON line per (size, element type): {"bytes":..,"dtype":..,"bad_words":..,"ms":..}.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define HIPCHK(x)                                                                    \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)
#define NCCLCHK(x)                                                                   \
    do {                                                                             \
        ncclResult_t r_ = (x);                                                       \
        if (r_ != ncclSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, ncclGetErrorString(r_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__device__ __forceinline__ uint64_t pattern(uint64_t i) { return (i + 1) * 0x9E3779B97F4A7C15ull; }

__global__ void k_fill(uint64_t* x, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        x[i] = pattern(i);
}

// mismatching words, and the first and last mismatching index
__global__ void k_check(const uint64_t* x, uint64_t n, unsigned long long* out) {
    unsigned long long bad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (x[i] != pattern(i)) {
            ++bad;
            atomicMin(&out[1], (unsigned long long)i);
            atomicMax(&out[2], (unsigned long long)i);
        }
    if (bad) atomicAdd(&out[0], bad);
}

int main(int argc, char** argv) {
    std::vector<double> gib = {1.0, 2.0 - 8.0 / (1ull << 30), 2.0, 2.0 + 8.0 / (1ull << 30), 3.2};
    if (argc > 1) {
        gib.clear();
        for (int i = 1; i < argc; ++i) gib.push_back(atof(argv[i]));
    }
    int dev = 0;
    HIPCHK(hipSetDevice(dev));
    ncclComm_t comm;
    NCCLCHK(ncclCommInitAll(&comm, 1, &dev));
    int ver = 0;
    NCCLCHK(ncclGetVersion(&ver));
    hipStream_t s;
    HIPCHK(hipStreamCreate(&s));
    uint64_t maxb = 0;
    for (double g : gib) {
        const uint64_t b = ((uint64_t)(g * (double)(1ull << 30)) + 7) & ~7ull;
        if (b > maxb) maxb = b;
    }
    uint64_t *src = nullptr, *dst = nullptr;
    unsigned long long* res = nullptr;
    HIPCHK(hipMalloc(&src, maxb));
    HIPCHK(hipMalloc(&dst, maxb));
    HIPCHK(hipMalloc(&res, 24));
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    for (double g : gib) {
        const uint64_t bytes = ((uint64_t)(g * (double)(1ull << 30)) + 7) & ~7ull;
        const uint64_t words = bytes / 8;
        for (int as_bytes = 0; as_bytes < 2; ++as_bytes) {
            k_fill<<<4096, 256, 0, s>>>(src, words);
            HIPCHK(hipMemsetAsync(dst, 0, bytes, s));
            const unsigned long long init[3] = {0, ~0ull, 0};
            HIPCHK(hipMemcpyAsync(res, init, 24, hipMemcpyHostToDevice, s));
            HIPCHK(hipEventRecord(e0, s));
            const size_t count = as_bytes ? bytes : words;
            const ncclDataType_t ty = as_bytes ? ncclUint8 : ncclUint64;
            NCCLCHK(ncclGroupStart());
            NCCLCHK(ncclSend(src, count, ty, 0, comm, s));
            NCCLCHK(ncclRecv(dst, count, ty, 0, comm, s));
            NCCLCHK(ncclGroupEnd());
            HIPCHK(hipEventRecord(e1, s));
            k_check<<<4096, 256, 0, s>>>(dst, words, res);
            unsigned long long out[3];
            HIPCHK(hipMemcpyAsync(out, res, 24, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"layer\": \"rccl grouped send/recv to self\", \"rccl_version\": %d, \"bytes\": %llu, "
                   "\"gib\": %.6f, \"dtype\": \"%s\", \"count\": %llu, \"bad_words\": %llu, \"first_bad\": %lld, "
                   "\"last_bad\": %lld, \"ms\": %.3f}\n",
                   ver, (unsigned long long)bytes, (double)bytes / (1ull << 30), as_bytes ? "uint8" : "uint64",
                   (unsigned long long)count, out[0], out[0] ? (long long)out[1] : -1LL,
                   out[0] ? (long long)out[2] : -1LL, ms);
            fflush(stdout);
        }
    }
    HIPCHK(hipFree(src));
    HIPCHK(hipFree(dst));
    HIPCHK(hipFree(res));
    ncclCommDestroy(comm);
    return 0;
}
