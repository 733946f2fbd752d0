// shard.hip — the row-sharded multi-GPU kNN build behind one C entry
// (SURVEY.md §8(b) `mn_knn_sharded_f32`, §8(e)): one process (or thread) per
// GPU, each holding its row shard, on a caller-owned RCCL communicator.
//
// ONE driver (sharded_drive) runs the build for the ranks a call drives over a
// Transport that carries its collectives:
//   * RcclTransport — one rank, the caller's communicator over xGMI; every
//     collective is waited for by polling the stream and ncclCommGetAsyncError
//     against a deadline (mn_rccl_set_timeout), so a peer that dies inside a
//     collective ends the call with MN_ECOMM (communicator aborted) instead of
//     hanging every other rank;
//   * LoopbackTransport — all R ranks of a simulated node on ONE device, each
//     on its own stream, device copies standing in for the collectives
//     (mn_knn_sharded_sim_f32: tests and single-GPU measurement of a share).
// The buffer layout, the exchange offsets, the in-place all-gathers and the
// status agreement are therefore the same code under both.
//
// Symmetric form (self kNN, L2^2, the bf16x1 generator applies, world > 1):
//   1. all-gather of the shards -> X_all resident on every rank;
//   2. stage A: tau0 of the rank's rows against the global phase-1 sample;
//      in-place all-gathers of tau0 and the row norms;
//   3. stage B: every rank builds the same Tf order and fp16 copy of all N
//      rows and sweeps ITS share of the symmetric block table (every
//      unordered pair of tiles once over the whole node), then re-ranks every
//      row in partial mode -> part lists of all rows [N][k];
//   4. exchange: each row's owner receives the R part lists of its rows
//      ([R][n_local][k], part p = the lists rank p computed);
//   5. stage C: merge + certify (the certificate of the single-GPU sweep:
//      the union of the parts' admitted candidates is the same set), exact
//      split scan of the rare uncertified rows against X_all.
// Per-shard form (other metrics / generators, or when the symmetric form
// does not apply — decided collectively):
//   exact per-shard top-k of all N queries against the rank's shard
//   (mn_knn_f32_qc, query chunks), the exchange, mn_knn_merge_f32.
// Both are exact: bit-identical to a single-GPU mn_knn_f32 of X.
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "common.hpp"
#include "gram_sweep2.hpp"
#include "shard_sym.hpp"

#define MN_NCCL_TRY(expr)                                                          \
    do {                                                                           \
        ncclResult_t _r = (expr);                                                  \
        if (_r != ncclSuccess) {                                                   \
            mn::set_error("%s failed: %s", #expr, ncclGetErrorString(_r));         \
            return MN_EHIP;                                                        \
        }                                                                          \
    } while (0)

namespace {

using mn::set_error;

// process-wide deadline of one collective (mn_rccl_set_timeout)
std::atomic<double> g_timeout_s{600.0};

// communicators this library aborted after a failed / timed-out collective:
// ncclCommAbort frees them, so mn_rccl_comm_destroy must not touch them again
std::mutex g_abort_mu;
std::set<void *> g_aborted;

bool comm_aborted(void *c) {
    std::lock_guard<std::mutex> g(g_abort_mu);
    return g_aborted.count(c) != 0;
}

}  // namespace

extern "C" {

int mn_rccl_unique_id(void *out_128_bytes) {
    mn::clear_error();
    MN_REQUIRE(out_128_bytes, MN_EINVAL, "mn_rccl_unique_id: NULL");
    ncclUniqueId id;
    MN_NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(out_128_bytes, &id, sizeof(id));
    return MN_OK;
}

int mn_rccl_comm_init(const void *unique_id_128_bytes, int32_t world, int32_t rank,
                      void **comm_out) {
    mn::clear_error();
    MN_REQUIRE(unique_id_128_bytes && comm_out && world >= 1 && rank >= 0 && rank < world,
               MN_EINVAL, "mn_rccl_comm_init: bad arguments");
    ncclUniqueId id;
    std::memcpy(&id, unique_id_128_bytes, sizeof(id));
    ncclComm_t c = nullptr;
    MN_NCCL_TRY(ncclCommInitRank(&c, world, id, rank));
    {
        // a new communicator may reuse the address of an aborted one
        std::lock_guard<std::mutex> g(g_abort_mu);
        g_aborted.erase((void *)c);
    }
    *comm_out = (void *)c;
    return MN_OK;
}

int mn_rccl_comm_destroy(void *comm) {
    mn::clear_error();
    if (!comm) return MN_OK;
    {
        std::lock_guard<std::mutex> g(g_abort_mu);
        if (g_aborted.erase(comm)) return MN_OK;  // already released by ncclCommAbort
    }
    MN_NCCL_TRY(ncclCommDestroy((ncclComm_t)comm));
    return MN_OK;
}

int mn_rccl_set_timeout(double seconds) {
    mn::clear_error();
    MN_REQUIRE(seconds > 0.0, MN_EINVAL, "mn_rccl_set_timeout: seconds must be > 0");
    g_timeout_s.store(seconds);
    return MN_OK;
}

}  // extern "C"

namespace {

// Release of a failed call's resources off the caller's thread.  Once a
// collective has failed, the caller's stream may still hold queued work that
// targets the call's buffers: a stalled kernel, or RCCL kernels that exit
// only when they see the abort.  hipFree / hipHostFree wait for the device
// to drain, so a failed call hands its buffers to a detached reaper thread
// that aborts the communicator and then frees them; the call returns
// MN_ECOMM at its deadline, not when the stream drains
// (mn_shard_quiesce waits for the reapers).
struct Graveyard {
    std::mutex mu;
    std::condition_variable cv;
    bool active = false;  // the call failed: buffers go to the reaper
    bool sealed = false;  // every buffer of the call has been handed over
    std::vector<void *> dev, host;
};

std::mutex g_reap_mu;
std::condition_variable g_reap_cv;
int g_reapers = 0;

struct DevBufs {
    std::vector<void *> v;
    std::shared_ptr<Graveyard> gy;  // may be null (the loopback transports)
    void *get(size_t bytes) {
        void *p = nullptr;
        if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
        v.push_back(p);
        return p;
    }
    ~DevBufs() {
        if (gy) {
            std::lock_guard<std::mutex> g(gy->mu);
            if (gy->active) {
                gy->dev.insert(gy->dev.end(), v.begin(), v.end());
                return;
            }
        }
        for (void *p : v) (void)hipFree(p);
    }
};

bool sym_applies(const mn::ShardPlan &pl, const mn_knn_opts *o) {
    return pl.ok && o->metric == MN_L2SQ && o->exclude_self &&
           (o->algo == MN_KNN_AUTO || o->algo == MN_KNN_BF16X1);
}

// ---- transports -------------------------------------------------------------

// The collectives of the sharded build for the ranks one call drives ("local
// ranks" l = 0 .. nlocal-1, global rank rank(l)).  Buffers are per local rank;
// sizes in bytes.  Every call returns with its data in place (or an error).
class Transport {
  public:
    virtual ~Transport() = default;
    virtual int world() const = 0;
    virtual int nlocal() const = 0;
    virtual int rank(int l) const = 0;
    virtual hipStream_t stream(int l) const = 0;
    // local rank l's stage work has been issued on stream(l)
    virtual int stage_done(int l) = 0;
    // recv[l] [world][bytes] <- every rank's send; in place when send[l] ==
    // recv[l] + rank(l) * bytes
    virtual int all_gather(const void *const *send, void *const *recv, size_t bytes,
                           const char *what) = 0;
    // for each of `na` arrays: block p of send[l] (bytes at p * bytes) goes to
    // rank p, which receives it as block rank(l) of its recv
    virtual int all_to_all(int na, const void *const *const *send, void *const *const *recv,
                           size_t bytes, const char *what) = 0;
    // *out = max over every rank of mine[l] (0 ok, 1 per-shard form, 2 error)
    virtual int agree(const int *mine, int *out) = 0;
    // where the driver's buffers go if a collective fails (null: freed in place)
    virtual std::shared_ptr<Graveyard> graveyard() { return nullptr; }
    // the tuning build's collective-order fault injection (MN_SHARD_REORDER=<rank>)
    virtual bool reorder_gathers() const { return false; }
};

#ifdef MN_TUNING
__global__ void k_stall(uint64_t ticks) {  // fault injection (tuning build only)
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
#endif

class RcclTransport final : public Transport {
  public:
    RcclTransport(ncclComm_t c, hipStream_t s)
        : c_(c), s_(s), timeout_(g_timeout_s.load()), gy_(std::make_shared<Graveyard>()) {}
    ~RcclTransport() override {
        {
            std::lock_guard<std::mutex> g(gy_->mu);
            if (gy_->active) {  // the reaper frees them once the stream drained
                if (pin_) gy_->host.push_back(pin_);
                if (dflag_) gy_->dev.push_back(dflag_);
                gy_->sealed = true;
                gy_->cv.notify_all();
                return;
            }
        }
        if (dflag_) (void)hipFree(dflag_);
        if (pin_) (void)hipHostFree(pin_);
    }
    int init() {
        MN_NCCL_TRY(ncclCommCount(c_, &world_));
        MN_NCCL_TRY(ncclCommUserRank(c_, &rank_));
        MN_HIP_TRY(hipGetDevice(&dev_));
        MN_HIP_TRY(hipHostMalloc((void **)&pin_, 64, hipHostMallocDefault));
        if (hipMalloc((void **)&dflag_, 64) != hipSuccess) {
            dflag_ = nullptr;
            set_error("mn_knn_sharded_f32: device allocation failed");
            return MN_ENOMEM;
        }
        // tuning build: stall the stream before the first collective (tests of
        // the deadline: the call must end with MN_ECOMM, not hang)
#ifdef MN_TUNING
        const int stall_ms = mn::knob_int("MN_SHARD_STALL_MS", 0);
        if (stall_ms > 0) {
            int khz = 0;
            MN_HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_));
            hipLaunchKernelGGL(k_stall, dim3(1), dim3(64), 0, s_, (uint64_t)stall_ms * (uint64_t)khz);
            MN_HIP_TRY(hipGetLastError());
        }
#endif
        return MN_OK;
    }
    int world() const override { return world_; }
    int nlocal() const override { return 1; }
    int rank(int) const override { return rank_; }
    hipStream_t stream(int) const override { return s_; }
    int stage_done(int) override { return MN_OK; }
    std::shared_ptr<Graveyard> graveyard() override { return gy_; }
    bool reorder_gathers() const override {
        const char *e = mn::knob("MN_SHARD_REORDER");
        return e && *e && atoi(e) == rank_;
    }

    int all_gather(const void *const *send, void *const *recv, size_t bytes,
                   const char *what) override {
        const ncclResult_t r = ncclAllGather(send[0], recv[0], bytes, ncclChar, c_, s_);
        if (r != ncclSuccess) return fail(what, ncclGetErrorString(r));
        return wait(what);
    }
    int all_to_all(int na, const void *const *const *send, void *const *const *recv, size_t bytes,
                   const char *what) override {
        ncclResult_t r = ncclGroupStart();
        for (int a = 0; a < na && r == ncclSuccess; ++a)
            for (int p = 0; p < world_ && r == ncclSuccess; ++p) {
                r = ncclSend((const char *)send[a][0] + (size_t)p * bytes, bytes, ncclChar, p, c_, s_);
                if (r == ncclSuccess)
                    r = ncclRecv((char *)recv[a][0] + (size_t)p * bytes, bytes, ncclChar, p, c_, s_);
            }
        const ncclResult_t r2 = ncclGroupEnd();
        if (r != ncclSuccess || r2 != ncclSuccess)
            return fail(what, ncclGetErrorString(r != ncclSuccess ? r : r2));
        return wait(what);
    }
    // pinned host flag: every copy is asynchronous, so the only blocking
    // point is the polled wait
    int agree(const int *mine, int *out) override {
        static const char *what = "the shard status all-reduce";
        pin_[0] = mine[0];
        hipError_t e = hipMemcpyAsync(dflag_, pin_, 4, hipMemcpyHostToDevice, s_);
        if (e != hipSuccess) return fail(what, hipGetErrorString(e));
        const ncclResult_t r = ncclAllReduce(dflag_, dflag_, 1, ncclInt32, ncclMax, c_, s_);
        if (r != ncclSuccess) return fail(what, ncclGetErrorString(r));
        e = hipMemcpyAsync(pin_ + 1, dflag_, 4, hipMemcpyDeviceToHost, s_);
        if (e != hipSuccess) return fail(what, hipGetErrorString(e));
        const int rc = wait(what);
        if (rc != MN_OK) return rc;
        *out = pin_[1];
        return MN_OK;
    }

  private:
    // the stream drained, or the communicator aborted: a stream error, an
    // RCCL async error, or no completion before the deadline (a peer died or
    // stalled)
    int wait(const char *what) {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        int nap_us = 20;
        for (;;) {
            const hipError_t e = hipStreamQuery(s_);
            if (e == hipSuccess) return MN_OK;
            if (e != hipErrorNotReady) {
                char why[160];
                snprintf(why, sizeof(why), "stream error %s", hipGetErrorString(e));
                return fail(what, why);
            }
            ncclResult_t ae = ncclSuccess;
            const ncclResult_t q = ncclCommGetAsyncError(c_, &ae);
            if (q != ncclSuccess) return fail(what, ncclGetErrorString(q));
            if (ae != ncclSuccess && ae != ncclInProgress) return fail(what, ncclGetErrorString(ae));
            const double el = std::chrono::duration<double>(clk::now() - t0).count();
            if (el > timeout_) {
                char why[160];
                snprintf(why, sizeof(why), "no completion within %.3g s (a peer rank failed or stalled)",
                         timeout_);
                return fail(what, why);
            }
            std::this_thread::sleep_for(std::chrono::microseconds(nap_us));
            nap_us = std::min(nap_us * 2, 1000);
        }
    }
    // Abort the communicator and hand the call's buffers to a reaper thread:
    // ncclCommAbort sets the abort flag the RCCL kernels poll, then releases
    // the communicator's memory, which (like our hipFree) waits for the
    // device; neither may hold up the return.
    int fail(const char *what, const char *why) {
        bool first = false;
        {
            std::lock_guard<std::mutex> g(gy_->mu);
            first = !gy_->active;
            gy_->active = true;
        }
        if (first) {
            {
                std::lock_guard<std::mutex> g(g_abort_mu);
                g_aborted.insert((void *)c_);
            }
            std::shared_ptr<Graveyard> gy = gy_;
            const ncclComm_t c = c_;
            const int dev = dev_;
            {
                std::lock_guard<std::mutex> g(g_reap_mu);
                ++g_reapers;
            }
            auto reap = [c, gy, dev]() {
                (void)hipSetDevice(dev);
                (void)ncclCommAbort(c);
                std::unique_lock<std::mutex> lk(gy->mu);
                gy->cv.wait(lk, [&] { return gy->sealed; });
                for (void *p : gy->dev) (void)hipFree(p);
                for (void *p : gy->host) (void)hipHostFree(p);
                gy->dev.clear();
                gy->host.clear();
                lk.unlock();
                {
                    std::lock_guard<std::mutex> g(g_reap_mu);
                    --g_reapers;
                }
                g_reap_cv.notify_all();
            };
            try {
                std::thread(reap).detach();
            } catch (...) {
                // no thread: abort here (the buffers are released when the
                // transport is destroyed, i.e. once the stream drained)
                (void)ncclCommAbort(c);
                std::lock_guard<std::mutex> g(gy_->mu);
                gy_->active = false;
                std::lock_guard<std::mutex> g2(g_reap_mu);
                --g_reapers;
            }
        }
        set_error("mn_knn_sharded_f32: %s: %s; the RCCL communicator was aborted "
                  "(mn_rccl_comm_destroy on it is a no-op)", what, why);
        return MN_ECOMM;
    }

    ncclComm_t c_;
    hipStream_t s_;
    double timeout_;
    std::shared_ptr<Graveyard> gy_;
    int world_ = 1, rank_ = 0, dev_ = 0;
    int *pin_ = nullptr, *dflag_ = nullptr;
};

// R ranks on one device: rank l on stream l (rank 0 on the caller's stream),
// stages one rank at a time (they share the calling thread's scratch), the
// collectives as device copies between full drains.
class LoopbackTransport final : public Transport {
  public:
    LoopbackTransport(int world, hipStream_t s0) : s_((size_t)world, nullptr) { s_[0] = s0; }
    ~LoopbackTransport() override {
        for (size_t l = 1; l < s_.size(); ++l)  // only the streams this object created
            if (s_[l]) (void)hipStreamDestroy(s_[l]);
    }
    int init() {
        for (size_t l = 1; l < s_.size(); ++l)
            MN_HIP_TRY(hipStreamCreateWithFlags(&s_[l], hipStreamNonBlocking));
        return MN_OK;
    }
    int world() const override { return (int)s_.size(); }
    int nlocal() const override { return (int)s_.size(); }
    int rank(int l) const override { return l; }
    hipStream_t stream(int l) const override { return s_[(size_t)l]; }
    int stage_done(int l) override {
        MN_HIP_TRY(hipStreamSynchronize(s_[(size_t)l]));
        return MN_OK;
    }
    int all_gather(const void *const *send, void *const *recv, size_t bytes, const char *) override {
        const int R = world();
        MN_HIP_TRY(drain());
        std::set<const void *> done;  // a receive buffer shared by ranks takes each block once
        for (int l = 0; l < R; ++l)
            for (int r = 0; r < R; ++r) {
                char *dst = (char *)recv[l] + (size_t)r * bytes;
                if (dst == (const char *)send[r] || !done.insert(dst).second) continue;  // in place
                MN_HIP_TRY(hipMemcpyAsync(dst, send[r], bytes, hipMemcpyDeviceToDevice, s_[(size_t)l]));
            }
        MN_HIP_TRY(drain());
        return MN_OK;
    }
    int all_to_all(int na, const void *const *const *send, void *const *const *recv, size_t bytes,
                   const char *) override {
        const int R = world();
        MN_HIP_TRY(drain());
        for (int a = 0; a < na; ++a)
            for (int l = 0; l < R; ++l)
                for (int p = 0; p < R; ++p)
                    MN_HIP_TRY(hipMemcpyAsync((char *)recv[a][l] + (size_t)p * bytes,
                                              (const char *)send[a][p] + (size_t)l * bytes, bytes,
                                              hipMemcpyDeviceToDevice, s_[(size_t)l]));
        MN_HIP_TRY(drain());
        return MN_OK;
    }
    int agree(const int *mine, int *out) override {
        int m = 0;
        for (int l = 0; l < world(); ++l) m = std::max(m, mine[l]);
        *out = m;
        return MN_OK;
    }

  private:
    hipError_t drain() {
        for (hipStream_t s : s_) {
            const hipError_t e = hipStreamSynchronize(s);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    std::vector<hipStream_t> s_;
};

// R ranks on one device, ONE HOST THREAD EACH (mn_knn_sharded_threads_f32):
// the ranks run concurrently, as the processes of a node do, each through
// the driver with nlocal() == 1 exactly as over RCCL.  Every collective is a
// rendezvous that first checks that all ranks issued the same collective —
// kind, sequence number, name and byte size.  A divergence in the collective
// order (one rank in the status agreement while another is in an
// all-gather), or a rank that left the driver while others wait in a
// collective, is reported on every rank as MN_ECOMM where RCCL would hang.
class Rendezvous {
  public:
    enum Kind { kAllGather = 1, kAllToAll, kAgree };
    struct Post {
        int kind = 0;
        int64_t seq = -1;
        size_t bytes = 0;
        const char *what = "";
        int na = 0;
        const void *send[2] = {nullptr, nullptr};
        void *recv[2] = {nullptr, nullptr};
        int val = 0;
    };
    Rendezvous(int R, double timeout_s) : R_(R), timeout_(timeout_s), post_((size_t)R), left_((size_t)R, 0) {}

    // post, wait for every rank, check that they all posted the same collective
    int enter(int r, const Post &p, std::vector<Post> *all) {
        {
            std::lock_guard<std::mutex> g(mu_);
            post_[(size_t)r] = p;
        }
        const int rc = barrier(r, p);
        if (rc != MN_OK) return rc;
        std::lock_guard<std::mutex> g(mu_);
        for (int q = 0; q < R_; ++q) {
            const Post &o = post_[(size_t)q];
            if (o.kind != p.kind || o.seq != p.seq || o.bytes != p.bytes || strcmp(o.what, p.what) != 0) {
                if (!broken_) {
                    char b[512];
                    snprintf(b, sizeof(b),
                             "collective order diverged at collective #%lld: rank %d issued %s "
                             "(kind %d, %zu bytes) while rank %d issued %s (kind %d, %zu bytes)",
                             (long long)p.seq, r, p.what, p.kind, p.bytes, q, o.what, o.kind, o.bytes);
                    why_ = b;
                    broken_ = true;
                    cv_.notify_all();
                }
                set_error("mn_knn_sharded_threads_f32: %s", why_.c_str());
                return MN_ECOMM;
            }
        }
        *all = post_;
        return MN_OK;
    }
    // every rank done with the others' buffers of this collective
    int leave_collective(int r, const Post &p) { return barrier(r, p); }
    // rank r left the driver (after its last collective, or early on an error)
    void depart(int r) {
        std::lock_guard<std::mutex> g(mu_);
        left_[(size_t)r] = 1;
        cv_.notify_all();
    }
    void abort(const char *why) {
        std::lock_guard<std::mutex> g(mu_);
        if (!broken_) why_ = why;
        broken_ = true;
        cv_.notify_all();
    }

  private:
    int barrier(int r, const Post &p) {
        using clk = std::chrono::steady_clock;
        std::unique_lock<std::mutex> lk(mu_);
        if (broken_) {
            set_error("mn_knn_sharded_threads_f32: %s", why_.c_str());
            return MN_ECOMM;
        }
        const uint64_t g = gen_;
        if (++arrived_ == R_) {
            arrived_ = 0;
            ++gen_;
            cv_.notify_all();
            return MN_OK;
        }
        const auto dl = clk::now() + std::chrono::duration_cast<clk::duration>(
                                         std::chrono::duration<double>(timeout_));
        while (gen_ == g && !broken_) {
            for (int q = 0; q < R_; ++q)
                if (left_[(size_t)q] && !broken_) {
                    char b[384];
                    snprintf(b, sizeof(b),
                             "rank %d left the driver while rank %d waits in %s (collective #%lld)", q,
                             r, p.what, (long long)p.seq);
                    why_ = b;
                    broken_ = true;
                }
            if (broken_) break;
            if (cv_.wait_until(lk, dl) == std::cv_status::timeout && gen_ == g && !broken_) {
                char b[384];
                snprintf(b, sizeof(b), "no completion of %s (collective #%lld) within %.3g s: a rank "
                         "never arrived", p.what, (long long)p.seq, timeout_);
                why_ = b;
                broken_ = true;
            }
        }
        if (gen_ != g) return MN_OK;
        cv_.notify_all();
        set_error("mn_knn_sharded_threads_f32: %s", why_.c_str());
        return MN_ECOMM;
    }

    const int R_;
    const double timeout_;
    std::mutex mu_;
    std::condition_variable cv_;
    uint64_t gen_ = 0;
    int arrived_ = 0;
    bool broken_ = false;
    std::string why_;
    std::vector<Post> post_;
    std::vector<char> left_;
};

class ThreadedTransport final : public Transport {
  public:
    ThreadedTransport(Rendezvous &h, int world, int rank, hipStream_t s)
        : h_(h), world_(world), rank_(rank), s_(s) {}
    int world() const override { return world_; }
    int nlocal() const override { return 1; }
    int rank(int) const override { return rank_; }
    hipStream_t stream(int) const override { return s_; }
    int stage_done(int) override { return MN_OK; }
    bool reorder_gathers() const override {
        const char *e = mn::knob("MN_SHARD_REORDER");
        return e && *e && atoi(e) == rank_;
    }
    int all_gather(const void *const *send, void *const *recv, size_t bytes,
                   const char *what) override {
        Rendezvous::Post p = post(Rendezvous::kAllGather, what, bytes);
        p.na = 1;
        p.send[0] = send[0];
        p.recv[0] = recv[0];
        std::vector<Rendezvous::Post> all;
        int rc = h_.enter(rank_, p, &all);
        if (rc != MN_OK) return rc;
        for (int q = 0; q < world_; ++q) {
            char *dst = (char *)recv[0] + (size_t)q * bytes;
            if (dst == (const char *)all[(size_t)q].send[0]) continue;  // in place (a shared X_all)
            rc = copy(dst, all[(size_t)q].send[0], bytes);
            if (rc != MN_OK) break;
        }
        if (rc == MN_OK) rc = sync();
        const int lrc = h_.leave_collective(rank_, p);
        return rc != MN_OK ? rc : lrc;
    }
    int all_to_all(int na, const void *const *const *send, void *const *const *recv, size_t bytes,
                   const char *what) override {
        Rendezvous::Post p = post(Rendezvous::kAllToAll, what, bytes);
        p.na = na;
        for (int a = 0; a < na && a < 2; ++a) {
            p.send[a] = send[a][0];
            p.recv[a] = recv[a][0];
        }
        std::vector<Rendezvous::Post> all;
        int rc = h_.enter(rank_, p, &all);
        if (rc != MN_OK) return rc;
        for (int a = 0; a < na && a < 2 && rc == MN_OK; ++a)
            for (int q = 0; q < world_ && rc == MN_OK; ++q)
                rc = copy((char *)recv[a][0] + (size_t)q * bytes,
                          (const char *)all[(size_t)q].send[a] + (size_t)rank_ * bytes, bytes);
        if (rc == MN_OK) rc = sync();
        const int lrc = h_.leave_collective(rank_, p);
        return rc != MN_OK ? rc : lrc;
    }
    int agree(const int *mine, int *out) override {
        Rendezvous::Post p = post(Rendezvous::kAgree, "the shard status agreement", 4);
        p.val = mine[0];
        std::vector<Rendezvous::Post> all;
        const int rc = h_.enter(rank_, p, &all);
        if (rc != MN_OK) return rc;
        int m = 0;
        for (const auto &o : all) m = std::max(m, o.val);
        *out = m;
        return h_.leave_collective(rank_, p);
    }

  private:
    // the rank's stage work is complete before its buffers are shared
    Rendezvous::Post post(int kind, const char *what, size_t bytes) {
        Rendezvous::Post p;
        p.kind = kind;
        p.seq = seq_++;
        p.bytes = bytes;
        p.what = what;
        const hipError_t e = hipStreamSynchronize(s_);
        if (e != hipSuccess) h_.abort("a rank's stream failed before a collective");
        return p;
    }
    int copy(void *dst, const void *src, size_t bytes) {
        MN_HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s_));
        return MN_OK;
    }
    int sync() {
        MN_HIP_TRY(hipStreamSynchronize(s_));
        return MN_OK;
    }
    Rendezvous &h_;
    int world_, rank_;
    hipStream_t s_;
    int64_t seq_ = 0;
};

// ---- the driver ---------------------------------------------------------------

// tuning build: MN_SHARD_FAIL=<stage><rank> fails that rank's stage A or B
// after it ran (tests of the status agreement)
int injected(char stage, int rank) {
    const char *e = mn::knob("MN_SHARD_FAIL");
    if (!e || e[0] != stage || atoi(e + 1) != rank) return MN_OK;
    set_error("mn_knn_sharded_f32: injected failure of stage %c on rank %d", stage, rank);
    return MN_EINVAL;
}

// per local rank: events at fixed slots, so the stage times have the same
// meaning in both forms (a slot not reached is recorded with the next one)
enum Slot { kStart, kGathered, kStageA, kGathered2, kStageB, kExchanged, kEnd, kSlots };

struct RankTimer {
    bool on = false;
    hipStream_t s = nullptr;
    hipEvent_t ev[kSlots] = {};
    int next = 0;
    int start(bool enable, hipStream_t stream) {
        on = enable;
        s = stream;
        if (!on) return MN_OK;
        for (auto &e : ev) MN_HIP_TRY(hipEventCreate(&e));
        upto(kStart);
        return MN_OK;
    }
    void upto(int slot) {
        if (!on) return;
        for (; next <= slot; ++next) (void)hipEventRecord(ev[next], s);
    }
    float ms(int a, int b) const {
        if (!on || a >= next || b >= next) return 0.f;
        (void)hipEventSynchronize(ev[b]);
        float t = 0.f;
        (void)hipEventElapsedTime(&t, ev[a], ev[b]);
        return t;
    }
    ~RankTimer() {
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
    }
};

struct RankIO {
    const float *x_shard;  // [n_local][d]
    int32_t *out_idx;      // [n_local][k]
    float *out_dist;
};

struct DriveOut {
    std::vector<float> rank_ms;  // [nlocal][3]: stage A, stage B, stage C
    mn_knn_stats st{};
};

// The build for T's local ranks.  xall_given (may be NULL): the all-gathered
// shards already resident (the loopback's X_all: the gather is in place).
// allow_sym1: the symmetric form also on one rank (tuning build).
int sharded_drive(Transport &T, const RankIO *io, int64_t nl, int d, const mn_knn_opts *opts,
                  int64_t query_chunk, const float *xall_given, bool allow_sym1, bool timing,
                  DriveOut *res) {
    using namespace mn;
    const int R = T.world(), NL = T.nlocal(), k = opts->k;
    const int64_t N = nl * R;
    MN_REQUIRE(N <= INT32_MAX, MN_EINVAL, "mn_knn_sharded_f32: ids must fit int32");
    MN_REQUIRE(R <= kMaxShardRanks, MN_ENOTSUP, "mn_knn_sharded_f32: at most %d ranks (merge width)",
               kMaxShardRanks);
    const size_t lb = 4 * (size_t)nl * k;  // bytes of one rank's block of a [*][k] list
    // per local rank: X_all, part lists of all rows li/ld [N][k], received
    // parts pi/pd [R][n_local][k], per-row tau0 / norms / Tc [3][N]
    DevBufs B;
    B.gy = T.graveyard();  // a failed collective leaves the frees to the reaper
    std::vector<float *> xall(NL);
    std::vector<int32_t *> li(NL), pi(NL);
    std::vector<float *> ld(NL), pd(NL), rowv(NL);
    for (int l = 0; l < NL; ++l) {
        xall[l] = xall_given ? (float *)xall_given : (float *)B.get(sizeof(float) * (size_t)N * d);
        li[l] = (int32_t *)B.get(lb * R);
        ld[l] = (float *)B.get(lb * R);
        pi[l] = (int32_t *)B.get(lb * R);
        pd[l] = (float *)B.get(lb * R);
        rowv[l] = (float *)B.get(4 * (size_t)N * 3 + 64);
        if (!xall[l] || !li[l] || !ld[l] || !pi[l] || !pd[l] || !rowv[l]) {
            set_error("mn_knn_sharded_f32: device allocation failed");
            return MN_ENOMEM;
        }
    }
    auto tau0 = [&](int l) { return rowv[l]; };
    auto qn = [&](int l) { return rowv[l] + N; };
    auto tc = [&](int l) { return rowv[l] + 2 * N; };
    std::vector<RankTimer> tm(NL);
    for (int l = 0; l < NL; ++l) {
        const int trc = tm[l].start(timing, T.stream(l));
        if (trc != MN_OK) return trc;
    }
    std::vector<int> rc(NL, MN_OK), st_of(NL, 0);
    int agreed = 0;
    // after an agreement: 0 continue; else the code this rank returns (never
    // the internal status 1; a healthy rank whose peer failed says so)
    auto settle = [&]() -> int {
        if (agreed != 2) return MN_OK;
        for (int l = 0; l < NL; ++l)
            if (rc[l] < 0) return rc[l];
        set_error("mn_knn_sharded_f32: another rank failed");
        return MN_EHIP;
    };
    auto status = [](int r) { return r == MN_OK ? 0 : r == 1 ? 1 : 2; };

    // 1. the shards everywhere
    {
        std::vector<const void *> snd(NL);
        std::vector<void *> rcv(NL);
        for (int l = 0; l < NL; ++l) {
            snd[l] = io[l].x_shard;
            rcv[l] = xall[l];
        }
        const int grc = T.all_gather(snd.data(), rcv.data(), sizeof(float) * (size_t)nl * d,
                                     "the all-gather of the shards");
        if (grc != MN_OK) return grc;
    }
    const ShardPlan pl = shard_plan(N, d, k, R);
    bool sym = (R > 1 || allow_sym1) && sym_applies(pl, opts);
    int64_t ncand = 0;
    int nfb = 0;
    if (sym) {
        // 2. stage A, then every rank's tau0 / norms everywhere (in place)
        for (int l = 0; l < NL; ++l) {
            tm[l].upto(kGathered);  // per rank: the loopback runs the ranks' stages in turn
            const int64_t row0 = (int64_t)T.rank(l) * nl;
            rc[l] = shard_phase1(xall[l], pl, row0, nl, T.stream(l), tau0(l) + row0, qn(l) + row0);
            if (rc[l] == MN_OK) rc[l] = injected('A', T.rank(l));
            tm[l].upto(kStageA);
            const int drc = T.stage_done(l);
            if (drc != MN_OK && rc[l] >= 0) rc[l] = drc;
            st_of[l] = status(rc[l]);
        }
        const int arc = T.agree(st_of.data(), &agreed);
        if (arc != MN_OK) return arc;
        if (const int e = settle()) return e;
        sym = agreed == 0;
    }
    if (sym) {
        const size_t rb = sizeof(float) * (size_t)nl;
        // in-place all-gather of one per-row array (0 tau0, 1 the norms)
        auto gather_rows = [&](int which) -> int {
            std::vector<const void *> snd(NL);
            std::vector<void *> rcv(NL);
            for (int l = 0; l < NL; ++l) {
                float *base = which == 0 ? tau0(l) : qn(l);
                snd[l] = base + (int64_t)T.rank(l) * nl;
                rcv[l] = base;
            }
            return T.all_gather(snd.data(), rcv.data(), rb,
                                which == 0 ? "the all-gather of the thresholds"
                                           : "the all-gather of the row norms");
        };
        // (tuning build: one rank issues the two in the other order — the
        // threaded loopback must report it, RCCL would hang or mix the data)
        const int first = T.reorder_gathers() ? 1 : 0;
        int grc = gather_rows(first);
        if (grc != MN_OK) return grc;
        grc = gather_rows(1 - first);
        if (grc != MN_OK) return grc;
        // 3. stage B: this rank's share, part lists of all rows
        for (int l = 0; l < NL; ++l) {
            tm[l].upto(kGathered2);
            int64_t nc1 = 0;
            rc[l] = shard_share(xall[l], pl, tau0(l), qn(l), T.rank(l), R, T.stream(l), li[l], ld[l],
                                tc(l), timing ? &nc1 : nullptr);
            if (rc[l] == MN_OK) rc[l] = injected('B', T.rank(l));
            tm[l].upto(kStageB);
            const int drc = T.stage_done(l);
            if (drc != MN_OK && rc[l] >= 0) rc[l] = drc;
            st_of[l] = status(rc[l]);
            ncand += nc1;
        }
        const int arc = T.agree(st_of.data(), &agreed);
        if (arc != MN_OK) return arc;
        if (const int e = settle()) return e;
        sym = agreed == 0;  // 1: a non-finite threshold anywhere (the same verdict everywhere)
    }
    if (sym) {
        // 4. the exchange, 5. stage C
        const void *const *snd[2] = {(const void *const *)li.data(), (const void *const *)ld.data()};
        void *const *rcv[2] = {(void *const *)pi.data(), (void *const *)pd.data()};
        const int xrc = T.all_to_all(2, snd, rcv, lb, "the exchange of the part lists");
        if (xrc != MN_OK) return xrc;
        for (int l = 0; l < NL; ++l) {
            tm[l].upto(kExchanged);
            int nf = 0;
            const int frc = shard_finish(xall[l], pl, (int64_t)T.rank(l) * nl, nl, R, (int64_t)nl * k,
                                         pi[l], pd[l], tc(l), T.stream(l), io[l].out_idx,
                                         io[l].out_dist, &nf);
            if (frc != MN_OK) return frc;  // nothing collective follows
            tm[l].upto(kEnd);
            const int drc = T.stage_done(l);
            if (drc != MN_OK) return drc;
            nfb += nf;
        }
    } else {
        // the per-shard form: exact per-shard top-k of every query against
        // the rank's shard, the exchange, the merge
        const int64_t qc = query_chunk > 0 ? query_chunk : ((int64_t)1 << 21);
        for (int l = 0; l < NL; ++l) {
            tm[l].upto(kGathered2);
            mn_knn_opts o = *opts;
            o.stream = T.stream(l);
            o.timing = 0;
            int r = MN_OK;
            for (int64_t a = 0; a < N && r == MN_OK; a += qc) {
                const int64_t b = std::min(N, a + qc);
                r = mn_knn_f32_qc(xall[l] + a * d, b - a, io[l].x_shard, nl, d, a,
                                  (int64_t)T.rank(l) * nl, &o, li[l] + a * k, ld[l] + a * k);
            }
            rc[l] = r;
            tm[l].upto(kStageB);
            const int drc = T.stage_done(l);
            if (drc != MN_OK && rc[l] >= 0) rc[l] = drc;
            st_of[l] = rc[l] == MN_OK ? 0 : 2;
        }
        // a failed rank must not leave the others waiting in the exchange
        const int arc = T.agree(st_of.data(), &agreed);
        if (arc != MN_OK) return arc;
        if (const int e = settle()) return e;
        const void *const *snd[2] = {(const void *const *)li.data(), (const void *const *)ld.data()};
        void *const *rcv[2] = {(void *const *)pi.data(), (void *const *)pd.data()};
        const int xrc = T.all_to_all(2, snd, rcv, lb, "the exchange of the per-shard lists");
        if (xrc != MN_OK) return xrc;
        for (int l = 0; l < NL; ++l) {
            tm[l].upto(kExchanged);
            const int mrc = mn_knn_merge_f32(pi[l], pd[l], R, nl, k, io[l].out_idx, io[l].out_dist,
                                             T.stream(l));
            if (mrc != MN_OK) return mrc;
            tm[l].upto(kEnd);
            const int drc = T.stage_done(l);
            if (drc != MN_OK) return drc;
        }
    }
    for (int l = 0; l < NL; ++l) MN_HIP_TRY(hipStreamSynchronize(T.stream(l)));
    mn_knn_stats &st = res->st;
    st = mn_knn_stats{};
    st.n_queries = nl * NL;
    st.algo = sym ? MN_KNN_BF16X1 : MN_KNN_AUTO;
    st.sweep_slices = sym ? -1 : 0;
    st.sample_rows = sym ? pl.m0 : 0;
    st.n_uncertified = nfb;
    st.n_candidates = ncand;
    res->rank_ms.assign((size_t)NL * 3, 0.f);
    for (int l = 0; l < NL; ++l) {
        const RankTimer &t = tm[l];
        const float a = t.ms(kGathered, kStageA), b = t.ms(kGathered2, kStageB),
                    c = t.ms(kExchanged, kEnd);
        res->rank_ms[(size_t)l * 3] = a;
        res->rank_ms[(size_t)l * 3 + 1] = b;
        res->rank_ms[(size_t)l * 3 + 2] = c;
        // max over the local ranks (the share that bounds the node)
        st.ms_norms = std::max(st.ms_norms, t.ms(kStart, kGathered) + t.ms(kStageA, kGathered2));
        st.ms_sample = std::max(st.ms_sample, a);
        st.ms_sweep = std::max(st.ms_sweep, b);
        st.ms_rerank = std::max(st.ms_rerank, t.ms(kStageB, kExchanged));
        st.ms_fallback = std::max(st.ms_fallback, c);
        st.ms_total = std::max(st.ms_total, t.ms(kStart, kEnd));
    }
    st.ms_gram = st.ms_sample + st.ms_sweep;
    return MN_OK;
}

}  // namespace

extern "C" {

int mn_knn_sharded_f32(const float *X_shard, int64_t n_local, int32_t d, void *comm,
                       const mn_knn_opts *opts, int64_t query_chunk, int32_t *out_idx,
                       float *out_dist) {
    using namespace mn;
    clear_error();
    MN_REQUIRE(X_shard && comm && opts && out_idx && out_dist, MN_EINVAL,
               "mn_knn_sharded_f32: NULL argument");
    MN_REQUIRE(n_local >= 1 && d >= 1 && opts->k >= 1, MN_EINVAL,
               "mn_knn_sharded_f32: bad shape");
    MN_REQUIRE(!comm_aborted(comm), MN_EINVAL,
               "mn_knn_sharded_f32: the communicator was aborted by an earlier call");
    RcclTransport T((ncclComm_t)comm, (hipStream_t)opts->stream);
    const int irc = T.init();
    if (irc != MN_OK) return irc;
    const RankIO io{X_shard, out_idx, out_dist};
    DriveOut res;
    const bool sym1 = knob_int("MN_SHARD_SYM1", 0) != 0;  // tuning build: world-1 symmetric form
    const int rc = sharded_drive(T, &io, n_local, d, opts, query_chunk, nullptr, sym1,
                                 opts->timing != 0, &res);
    if (rc != MN_OK) return rc;
    knn_stats_ref() = res.st;
    return MN_OK;
}

// Host only: rank `rank`'s share of the node-wide symmetric tile table over
// nbk 256-row blocks (ksw2::sym_block_table_share; entries (I, Jfirst, tiles,
// stride), the empty XCD padding included).  out4 [cap][4] may be NULL to
// query the count; *n_out = entries.  MN_ECAP when cap is too small.
int mn_sym_share_table(int32_t nbk, int32_t rank, int32_t world, int32_t *out4, int64_t cap,
                       int64_t *n_out) {
    using namespace mn;
    clear_error();
    MN_REQUIRE(nbk >= 1 && world >= 1 && rank >= 0 && rank < world && n_out, MN_EINVAL,
               "mn_sym_share_table: bad arguments");
    const std::vector<int4> tab = ksw2::sym_block_table_share(nbk, 256, rank, world, ksw2::kShareGR);
    *n_out = (int64_t)tab.size();
    if (!out4) return MN_OK;
    MN_REQUIRE((int64_t)tab.size() <= cap, MN_ECAP, "mn_sym_share_table: cap < %zu", tab.size());
    for (size_t i = 0; i < tab.size(); ++i) {
        out4[4 * i] = tab[i].x;
        out4[4 * i + 1] = tab[i].y;
        out4[4 * i + 2] = tab[i].z;
        out4[4 * i + 3] = tab[i].w;
    }
    return MN_OK;
}

// The sharded build of `world` ranks on ONE device through the loopback
// transport: X_all [n_tot][d] (device) holds the shards (rank r's at r *
// n_tot / world, so the all-gather is in place); the same driver as
// mn_knn_sharded_f32 runs every rank's stages in turn and the collectives as
// device copies.  out [n_tot][k]: the global graph (bit-identical to
// mn_knn_f32).  rank_ms [world][3] (host, may be NULL): per rank the stage A,
// stage B and stage C milliseconds (device events) — a rank's share of the
// real build.
int mn_knn_sharded_sim_f32(const float *X_all, int64_t n_tot, int32_t d, int32_t world,
                           const mn_knn_opts *opts, int32_t *out_idx, float *out_dist,
                           float *rank_ms) {
    using namespace mn;
    clear_error();
    MN_REQUIRE(X_all && opts && out_idx && out_dist, MN_EINVAL, "mn_knn_sharded_sim_f32: NULL argument");
    MN_REQUIRE(world >= 1 && world <= kMaxShardRanks && n_tot >= world && n_tot % world == 0 &&
                   d >= 1 && opts->k >= 1 && n_tot <= INT32_MAX,
               MN_EINVAL, "mn_knn_sharded_sim_f32: bad shape (n_tot a multiple of world <= 16)");
    const int64_t nl = n_tot / world;
    LoopbackTransport T(world, (hipStream_t)opts->stream);
    const int irc = T.init();
    if (irc != MN_OK) return irc;
    std::vector<RankIO> io((size_t)world);
    for (int r = 0; r < world; ++r)
        io[(size_t)r] = RankIO{X_all + (size_t)r * nl * d, out_idx + (size_t)r * nl * opts->k,
                               out_dist + (size_t)r * nl * opts->k};
    DriveOut res;
    const int rc = sharded_drive(T, io.data(), nl, d, opts, 0, X_all, false,
                                 opts->timing != 0 || rank_ms != nullptr, &res);
    if (rc != MN_OK) return rc;
    knn_stats_ref() = res.st;
    if (rank_ms) std::memcpy(rank_ms, res.rank_ms.data(), sizeof(float) * res.rank_ms.size());
    return MN_OK;
}

// The sharded build of `world` ranks on ONE device with one host thread per
// rank (ThreadedTransport): the ranks' stages and collectives run
// concurrently, each rank through the driver exactly as one RCCL process
// does, and every collective checks that all ranks issued the same one.
// Arguments as mn_knn_sharded_sim_f32; the collective deadline is
// mn_rccl_set_timeout's.
int mn_knn_sharded_threads_f32(const float *X_all, int64_t n_tot, int32_t d, int32_t world,
                               const mn_knn_opts *opts, int32_t *out_idx, float *out_dist,
                               float *rank_ms) {
    using namespace mn;
    clear_error();
    MN_REQUIRE(X_all && opts && out_idx && out_dist, MN_EINVAL,
               "mn_knn_sharded_threads_f32: NULL argument");
    MN_REQUIRE(world >= 1 && world <= kMaxShardRanks && n_tot >= world && n_tot % world == 0 &&
                   d >= 1 && opts->k >= 1 && n_tot <= INT32_MAX,
               MN_EINVAL, "mn_knn_sharded_threads_f32: bad shape (n_tot a multiple of world <= 16)");
    const int64_t nl = n_tot / world;
    int dev = 0;
    MN_HIP_TRY(hipGetDevice(&dev));
    MN_HIP_TRY(hipStreamSynchronize((hipStream_t)opts->stream));  // X_all is complete
    const bool timing = opts->timing != 0 || rank_ms != nullptr;
    Rendezvous hub(world, g_timeout_s.load());
    std::vector<int> rc((size_t)world, MN_OK);
    std::vector<std::string> err((size_t)world);
    std::vector<DriveOut> res((size_t)world);
    auto run_rank = [&](int r) {
        int code = MN_OK;
        hipStream_t s = nullptr;
        if (hipSetDevice(dev) != hipSuccess ||
            hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
            set_error("mn_knn_sharded_threads_f32: rank %d could not get a stream", r);
            code = MN_EHIP;
        } else {
            mn_knn_opts o = *opts;
            o.stream = s;
            ThreadedTransport T(hub, world, r, s);
            const RankIO io{X_all + (size_t)r * nl * d, out_idx + (size_t)r * nl * opts->k,
                            out_dist + (size_t)r * nl * opts->k};
            code = sharded_drive(T, &io, nl, d, &o, 0, X_all, false, timing, &res[(size_t)r]);
        }
        hub.depart(r);
        if (code != MN_OK) err[(size_t)r] = mn_last_error();
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
        rc[(size_t)r] = code;
    };
    std::vector<std::thread> th;
    th.reserve((size_t)world);
    for (int r = 0; r < world; ++r) {
        try {
            th.emplace_back(run_rank, r);
        } catch (...) {
            hub.abort("a rank's host thread could not be started");
            for (int q = r; q < world; ++q) {
                rc[(size_t)q] = MN_EHIP;
                err[(size_t)q] = "mn_knn_sharded_threads_f32: could not start a host thread";
            }
            break;
        }
    }
    for (auto &t : th) t.join();
    // the error to report: the first rank whose own stage or collective
    // failed (the others only say that another rank failed)
    int bad = -1;
    for (int r = 0; r < world; ++r)
        if (rc[(size_t)r] != MN_OK &&
            (bad < 0 || (err[(size_t)bad].find("another rank failed") != std::string::npos &&
                         err[(size_t)r].find("another rank failed") == std::string::npos)))
            bad = r;
    if (bad >= 0) {
        set_error("rank %d: %s", bad, err[(size_t)bad].c_str());
        return rc[(size_t)bad];
    }
    mn_knn_stats st = res[0].st;
    for (int r = 1; r < world; ++r) {
        const mn_knn_stats &o = res[(size_t)r].st;
        st.n_queries += o.n_queries;
        st.n_uncertified += o.n_uncertified;
        st.n_candidates += o.n_candidates;
        st.ms_norms = std::max(st.ms_norms, o.ms_norms);
        st.ms_sample = std::max(st.ms_sample, o.ms_sample);
        st.ms_sweep = std::max(st.ms_sweep, o.ms_sweep);
        st.ms_rerank = std::max(st.ms_rerank, o.ms_rerank);
        st.ms_fallback = std::max(st.ms_fallback, o.ms_fallback);
        st.ms_total = std::max(st.ms_total, o.ms_total);
        st.ms_gram = std::max(st.ms_gram, o.ms_gram);
    }
    knn_stats_ref() = st;
    if (rank_ms)
        for (int r = 0; r < world; ++r)
            for (int c = 0; c < 3; ++c)
                rank_ms[3 * r + c] = res[(size_t)r].rank_ms.size() == 3 ? res[(size_t)r].rank_ms[(size_t)c] : 0.f;
    return MN_OK;
}

// Wait (up to timeout_s) for the reaper threads of failed sharded calls to
// abort their communicators and free those calls' buffers.
int mn_shard_quiesce(double timeout_s) {
    mn::clear_error();
    std::unique_lock<std::mutex> lk(g_reap_mu);
    const bool done = g_reap_cv.wait_for(lk, std::chrono::duration<double>(timeout_s > 0 ? timeout_s : 0),
                                         [] { return g_reapers == 0; });
    if (!done) {
        mn::set_error("mn_shard_quiesce: %d failed call(s) still releasing after %.3g s", g_reapers,
                      timeout_s);
        return MN_ECOMM;
    }
    return MN_OK;
}

}  // extern "C"
