// comm.hpp — the exchange layer under the sharded DistributedHashMap (dist_hash_map.hpp).
//
// The reference moves k-mers and lookups with UPC++ RPCs (hash_map.hpp:38-46 batched inserts,
// hash_map.hpp:94-100 remote finds). Here every exchange is a bulk all-to-all of 64-bit words
// between the ranks' device buffers plus a small host all-gather of counts, so a transport needs
// only three collectives:
//
//   ThreadComm  P ranks as P threads of one process (any mix of GPUs, several ranks per GPU
//               allowed): device-to-device copies through a shared slot table. Tests run P logical
//               ranks on one GPU with it.
//   RcclComm    rccl_comm.hpp: RCCL over xGMI (ncclSend/ncclRecv groups), one rank per GPU; built
//               either for P threads of one process (ncclCommInitAll) or one process per GPU
//               (ncclCommInitRank with a shared ncclUniqueId).
#pragma once
#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace kh {

inline void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

class Comm {
public:
    virtual ~Comm() = default;
    virtual int rank() const = 0;
    virtual int size() const = 0;
    // Every rank contributes n host words; all receives size() * n words, rank-major. Blocking;
    // device transports order it after the work already queued on `stream`.
    virtual void allgather(const uint64_t* mine, size_t n, uint64_t* all, hipStream_t stream) = 0;
    // Device all-to-all of int64 words: send + sdispl[q] holds scount[q] words for rank q, rank q's
    // words for this rank land at recv + rdispl[q] (rcount[q] words). max_pair = the largest
    // single (sender, receiver) count over ALL ranks (identical on every rank: transports that
    // split large messages run the same number of steps everywhere). Work is ordered on `stream`;
    // the recv buffer is complete when work queued on `stream` afterwards runs.
    virtual void alltoallv(const int64_t* send, const uint64_t* scount, const uint64_t* sdispl, int64_t* recv,
                           const uint64_t* rcount, const uint64_t* rdispl, uint64_t max_pair,
                           hipStream_t stream) = 0;
    virtual void barrier() = 0;
    // Device all-gather: every rank's n words at dev_in land at dev_out + q * n (rank q's), ordered
    // on `stream` (no host wait: the caller reads the result with its own copy).
    virtual void allgather_dev(const int64_t* dev_in, size_t n, int64_t* dev_out, hipStream_t stream) = 0;
};

// ---------------------------------------------------------------------------------------------
// P ranks as threads of one process. Create one group, hand comm(r) to thread r.
class ThreadComm : public Comm {
public:
    class Group {
    public:
        explicit Group(int world) : world_(world), slots_(world) {
            for (int r = 0; r < world; ++r) comms_.emplace_back(new ThreadComm(this, r));
        }
        ThreadComm* comm(int r) { return comms_.at(r).get(); }
        int world() const { return world_; }
        // a failing rank calls abort(): every rank blocked (or arriving later) in a collective
        // throws instead of waiting forever
        void abort() {
            std::lock_guard<std::mutex> g(m_);
            aborted_ = true;
            cv_.notify_all();
        }

    private:
        friend class ThreadComm;
        struct Slot {
            const void* p = nullptr;
            const uint64_t* count = nullptr;
            const uint64_t* displ = nullptr;
            int device = 0;
            hipEvent_t ready = nullptr;
        };
        void wait_all() {  // reusable barrier
            std::unique_lock<std::mutex> g(m_);
            if (aborted_) throw std::runtime_error("ThreadComm: another rank failed");
            const uint64_t gen = gen_;
            if (++arrived_ == world_) {
                arrived_ = 0;
                ++gen_;
                cv_.notify_all();
                return;
            }
            cv_.wait(g, [&] { return gen_ != gen || aborted_; });
            if (aborted_) throw std::runtime_error("ThreadComm: another rank failed");
        }
        int world_;
        std::vector<Slot> slots_;
        std::vector<std::unique_ptr<ThreadComm>> comms_;
        std::mutex m_;
        std::condition_variable cv_;
        int arrived_ = 0;
        uint64_t gen_ = 0;
        bool aborted_ = false;
    };

    int rank() const override { return rank_; }
    int size() const override { return g_->world_; }
    Group* group() { return g_; }

    void allgather(const uint64_t* mine, size_t n, uint64_t* all, hipStream_t) override {
        auto& s = g_->slots_[rank_];
        s.p = mine;
        g_->wait_all();
        for (int q = 0; q < g_->world_; ++q) {
            const uint64_t* src = static_cast<const uint64_t*>(g_->slots_[q].p);
            for (size_t i = 0; i < n; ++i) all[(size_t)q * n + i] = src[i];
        }
        g_->wait_all();
    }

    void alltoallv(const int64_t* send, const uint64_t* scount, const uint64_t* sdispl, int64_t* recv,
                   const uint64_t* rcount, const uint64_t* rdispl, uint64_t, hipStream_t stream) override {
        (void)scount;
        int dev = 0;
        hip_check(hipGetDevice(&dev), "hipGetDevice");
        if (!ev_) hip_check(hipEventCreateWithFlags(&ev_, hipEventDisableTiming), "hipEventCreate");
        hip_check(hipEventRecord(ev_, stream), "hipEventRecord");  // send buffer written
        auto& s = g_->slots_[rank_];
        s.p = send;
        s.count = scount;
        s.displ = sdispl;
        s.device = dev;
        s.ready = ev_;
        g_->wait_all();
        for (int q = 0; q < g_->world_; ++q) {
            const auto& o = g_->slots_[q];
            if (!rcount[q]) continue;
            hip_check(hipStreamWaitEvent(stream, o.ready, 0), "hipStreamWaitEvent");
            const int64_t* src = static_cast<const int64_t*>(o.p) + o.displ[rank_];
            if (o.device == dev)
                hip_check(hipMemcpyAsync(recv + rdispl[q], src, rcount[q] * 8, hipMemcpyDeviceToDevice, stream),
                          "hipMemcpyAsync");
            else
                hip_check(hipMemcpyPeerAsync(recv + rdispl[q], dev, src, o.device, rcount[q] * 8, stream),
                          "hipMemcpyPeerAsync");
        }
        // the senders' buffers must outlive every reader's copy
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
        g_->wait_all();
    }

    void barrier() override { g_->wait_all(); }

    void allgather_dev(const int64_t* dev_in, size_t n, int64_t* dev_out, hipStream_t stream) override {
        std::vector<uint64_t> cnt(g_->world_, n), dsp(g_->world_, 0), rd(g_->world_);
        for (int q = 0; q < g_->world_; ++q) rd[q] = (uint64_t)q * n;
        alltoallv(dev_in, cnt.data(), dsp.data(), dev_out, cnt.data(), rd.data(), n, stream);
    }

    ~ThreadComm() override {
        if (ev_) (void)hipEventDestroy(ev_);
    }

private:
    ThreadComm(Group* g, int r) : g_(g), rank_(r) {}
    Group* g_;
    int rank_;
    hipEvent_t ev_ = nullptr;
};

}  // namespace kh
