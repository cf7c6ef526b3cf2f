// rccl_comm.hpp — RCCL transport for the sharded DistributedHashMap (link with -lrccl).
//
// One rank per GPU over xGMI. The all-to-all is a group of ncclSend/ncclRecv pairs (RCCL runs
// them as point-to-point transfers on the xGMI links); count all-gathers go through a small
// device buffer. Per-peer messages are split at 512 MiB: single messages of >= 2 GiB per peer
// came back corrupted from RCCL 2.26 (found by the bench's ground-truth check).
//
//   auto comms = kh::RcclComm::init_all({0, 1, ..., P-1});   // one process, thread r uses comms[r]
//   kh::RcclComm c(rank, world, id, device);                 // one process per GPU (id from
//                                                            //  kh::RcclComm::unique_id() on rank 0)
#pragma once
#include <rccl/rccl.h>

#include <memory>
#include <vector>

#include "comm.hpp"

namespace kh {

class RcclComm : public Comm {
public:
    static constexpr uint64_t MAX_MSG_WORDS = (512ull << 20) / 8;

    static ncclUniqueId unique_id() {
        ncclUniqueId id;
        check(ncclGetUniqueId(&id), "ncclGetUniqueId");
        return id;
    }
    // P ranks in this process, rank r on devices[r] (hand comms[r] to the thread driving rank r)
    static std::vector<std::unique_ptr<RcclComm>> init_all(const std::vector<int>& devices) {
        std::vector<ncclComm_t> raw(devices.size());
        check(ncclCommInitAll(raw.data(), (int)devices.size(), devices.data()), "ncclCommInitAll");
        std::vector<std::unique_ptr<RcclComm>> out;
        for (size_t r = 0; r < devices.size(); ++r)
            out.emplace_back(new RcclComm(raw[r], (int)r, (int)devices.size(), devices[r]));
        return out;
    }
    RcclComm(int rank, int world, const ncclUniqueId& id, int device) : rank_(rank), world_(world), dev_(device) {
        hip_check(hipSetDevice(device), "hipSetDevice");
        check(ncclCommInitRank(&comm_, world, id, rank), "ncclCommInitRank");
        init_scratch();
    }
    ~RcclComm() override {
        if (scratch_) (void)hipFree(scratch_);
        if (stream_) (void)hipStreamDestroy(stream_);
        if (comm_) (void)ncclCommDestroy(comm_);
    }

    int rank() const override { return rank_; }
    int size() const override { return world_; }

    // on the caller's stream: every operation of this communicator is issued in one stream order
    void allgather(const uint64_t* mine, size_t n, uint64_t* all, hipStream_t stream) override {
        hip_check(hipSetDevice(dev_), "hipSetDevice");
        ensure_scratch(n * (world_ + 1));
        hip_check(hipMemcpyAsync(scratch_, mine, n * 8, hipMemcpyHostToDevice, stream), "hipMemcpyAsync");
        check(ncclAllGather(scratch_, scratch_ + n, n, ncclUint64, comm_, stream), "ncclAllGather");
        hip_check(hipMemcpyAsync(all, scratch_ + n, n * world_ * 8, hipMemcpyDeviceToHost, stream),
                  "hipMemcpyAsync");
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    }

    void alltoallv(const int64_t* send, const uint64_t* scount, const uint64_t* sdispl, int64_t* recv,
                   const uint64_t* rcount, const uint64_t* rdispl, uint64_t max_pair, hipStream_t stream) override {
        const uint64_t steps = max_pair ? (max_pair + MAX_MSG_WORDS - 1) / MAX_MSG_WORDS : 1;
        for (uint64_t s = 0; s < steps; ++s) {
            const uint64_t lo = s * MAX_MSG_WORDS;
            check(ncclGroupStart(), "ncclGroupStart");
            for (int q = 0; q < world_; ++q) {
                if (scount[q] > lo) {
                    const uint64_t c = scount[q] - lo < MAX_MSG_WORDS ? scount[q] - lo : MAX_MSG_WORDS;
                    check(ncclSend(send + sdispl[q] + lo, c, ncclInt64, q, comm_, stream), "ncclSend");
                }
                if (rcount[q] > lo) {
                    const uint64_t c = rcount[q] - lo < MAX_MSG_WORDS ? rcount[q] - lo : MAX_MSG_WORDS;
                    check(ncclRecv(recv + rdispl[q] + lo, c, ncclInt64, q, comm_, stream), "ncclRecv");
                }
            }
            check(ncclGroupEnd(), "ncclGroupEnd");
        }
    }

    void allgather_dev(const int64_t* dev_in, size_t n, int64_t* dev_out, hipStream_t stream) override {
        hip_check(hipSetDevice(dev_), "hipSetDevice");
        check(ncclAllGather(dev_in, dev_out, n, ncclInt64, comm_, stream), "ncclAllGather");
    }

    void barrier() override {
        uint64_t x = 0;
        std::vector<uint64_t> all(world_);
        allgather(&x, 1, all.data(), stream_);
    }

private:
    RcclComm(ncclComm_t c, int rank, int world, int device) : comm_(c), rank_(rank), world_(world), dev_(device) {
        hip_check(hipSetDevice(device), "hipSetDevice");
        init_scratch();
    }
    static void check(ncclResult_t r, const char* what) {
        if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
    }
    void init_scratch() {
        hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
        ensure_scratch(1024);
    }
    void ensure_scratch(size_t words) {
        if (words <= cap_) return;
        if (scratch_) {
            hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");  // no op still reads it
            hip_check(hipFree(scratch_), "hipFree");
        }
        hip_check(hipMalloc(reinterpret_cast<void**>(&scratch_), words * 8), "hipMalloc");
        cap_ = words;
    }
    ncclComm_t comm_ = nullptr;
    int rank_, world_, dev_;
    hipStream_t stream_ = nullptr;
    uint64_t* scratch_ = nullptr;
    size_t cap_ = 0;
};

}  // namespace kh
