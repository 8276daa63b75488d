// Collective transports (collective.hpp): RCCL across processes, and the
// in-process group of contexts driven by threads.
#include "collective.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <vector>

#include <unistd.h>

namespace wfsa {
namespace {

// ---- RCCL ----------------------------------------------------------------

// A non-blocking communicator's call that returned ncclInProgress: poll its
// state until it settles; ncclInProgress after limit_s = timed out
ncclResult_t rccl_settle(ncclComm_t c, double limit_s) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        ncclResult_t st = ncclInProgress;
        if (ncclCommGetAsyncError(c, &st) != ncclSuccess) return ncclInternalError;
        if (st != ncclInProgress) return st;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) return ncclInProgress;
        usleep(20);
    }
}


class RcclCollective final : public Collective {
public:
    RcclCollective(ncclComm_t c, int n, int r) : comm_(c), timeout_s_(comm_timeout_s()) {
        n_ = n;
        r_ = r;
    }
    // the communicator's asynchronous error, or a host wait past the limit:
    // abort it (its pending kernels on this rank end) and report
    int watchdog(double waited_s) override {
        if (check()) return 1;
        std::string why;
        ncclResult_t st = ncclSuccess;
        if (comm_ && ncclCommGetAsyncError(comm_, &st) == ncclSuccess && st != ncclSuccess && st != ncclInProgress)
            why = std::string("RCCL asynchronous error: ") + ncclGetErrorString(st);
        else if (waited_s > timeout_s_)
            why = "no progress within WFSA_COMM_TIMEOUT_S (a member failed or stalled)";
        if (why.empty()) return 0;
        abort(why.c_str());
        err_ = why;
        return 1;
    }
    ~RcclCollective() override {
        if (comm_) (void)ncclCommDestroy(comm_);
    }
    const char* kind() const override { return "rccl"; }
    bool peer_default() const override { return true; }
    void abort_transport(const std::string&) override {   // the other members' pending RCCL calls see a broken ring
        if (comm_) (void)ncclCommAbort(comm_);
        comm_ = nullptr;
    }
    int transport_allreduce(void* buf, size_t n, RedOp op, hipStream_t s) override {
        if (n == 0) return 0;
        if (!comm_) {
            err_ = "the RCCL communicator was aborted";
            return 1;
        }
        ncclDataType_t t = op == RedOp::MaxU8 ? ncclUint8 : ncclDouble;
        ncclRedOp_t o = op == RedOp::SumF64 ? ncclSum : op == RedOp::MinF64 ? ncclMin : ncclMax;
        ncclResult_t r = ncclAllReduce(buf, buf, n, t, o, comm_, s);
        if (r == ncclInProgress) r = rccl_settle(comm_, timeout_s_);   // (enqueued once it settles)
        if (r != ncclSuccess) {
            err_ = r == ncclInProgress ? std::string("ncclAllReduce did not settle within WFSA_COMM_TIMEOUT_S")
                                       : std::string("ncclAllReduce failed: ") + ncclGetErrorString(r);
            return 1;
        }
        return 0;
    }

private:
    ncclComm_t comm_;
    double timeout_s_;
};

// ---- in-process group ----------------------------------------------------

constexpr char kLocalMagic[8] = {'w', 'f', 's', 'a', 'L', 'O', 'C', 'L'};

struct LocalGroup {
    int n = 0;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    int joined = 0;
    void* ptrs[kLocalMaxRanks] = {};
    size_t count[kLocalMaxRanks] = {};
    int op[kLocalMaxRanks] = {};
    int dev[kLocalMaxRanks] = {};

    bool poisoned = false;   // a member timed out or failed: the group is out of step for good
    std::string why;         // (under m) what poisoned it
    int limit_s = 120;       // WFSA_GROUP_TIMEOUT_S when the group was made

    // false on a timeout (a member that never arrives: a bug upstream, or a
    // member that failed without aborting) or once the group is poisoned.  A
    // timeout poisons the group -- the late member's arrival would otherwise
    // release a later barrier at the wrong count and combine buffers from
    // different calls -- so every later call fails at once.  A member that
    // fails anywhere poisons it too (Collective::abort), which wakes every
    // waiting member now.  WFSA_GROUP_TIMEOUT_S sets the limit (default 120 s,
    // inside a test's limit; a healthy rank's host work between collectives,
    // e.g. a sparse factorisation, is replicated on every rank, so members
    // arrive together).
    bool barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (poisoned) return false;
        const uint64_t g0 = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        if (cv.wait_for(lk, std::chrono::seconds(limit_s), [&] { return gen != g0 || poisoned; }) && !poisoned)
            return true;
        if (!poisoned) why = "a member did not arrive within WFSA_GROUP_TIMEOUT_S";
        poisoned = true;
        cv.notify_all();
        return false;
    }
    void poison(const std::string& w) {
        std::lock_guard<std::mutex> lk(m);
        if (!poisoned) why = w;
        poisoned = true;
        cv.notify_all();
    }
    std::string reason() {
        std::lock_guard<std::mutex> lk(m);
        return why;
    }
};

std::mutex g_reg_m;
std::map<uint64_t, std::shared_ptr<LocalGroup>> g_reg;
std::atomic<uint64_t> g_serial{1};

struct Ptrs {
    const void* p[kLocalMaxRanks];
};

template <int OP>
__global__ void __launch_bounds__(256) rank_reduce_kernel(Ptrs src, int k, size_t n, void* dst) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    for (size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        if constexpr (OP == int(RedOp::MaxU8)) {
            uint8_t v = static_cast<const uint8_t*>(src.p[0])[i];
            for (int r = 1; r < k; ++r) v = max(v, static_cast<const uint8_t*>(src.p[r])[i]);
            static_cast<uint8_t*>(dst)[i] = v;
        } else {
            double v = static_cast<const double*>(src.p[0])[i];
            for (int r = 1; r < k; ++r) {   // rank order: deterministic
                const double x = static_cast<const double*>(src.p[r])[i];
                v = OP == int(RedOp::SumF64) ? v + x : fmin(v, x);
            }
            static_cast<double*>(dst)[i] = v;
        }
    }
}

class LocalCollective final : public Collective {
public:
    LocalCollective(std::shared_ptr<LocalGroup> g, int r, int device) : g_(std::move(g)), device_(device) {
        n_ = g_->n;
        r_ = r;
    }
    ~LocalCollective() override {
        if (tmp_) (void)hipFree(tmp_);
    }
    const char* kind() const override { return "local"; }
    bool same_process() const override { return true; }
    int device() const override { return device_; }
    void abort_transport(const std::string& why) override { g_->poison("member " + std::to_string(r_) + " aborted: " + why); }
    int transport_allreduce(void* buf, size_t n, RedOp op, hipStream_t s) override {
        const size_t esz = op == RedOp::MaxU8 ? 1 : 8;
        if (n * esz > tmp_bytes_) {
            if (tmp_) (void)hipFree(tmp_);
            tmp_ = nullptr;
            tmp_bytes_ = 0;
            if (hipMalloc(&tmp_, n * esz) != hipSuccess) return fail("hipMalloc of the group scratch failed");
            tmp_bytes_ = n * esz;
        }
        if (hipStreamSynchronize(s) != hipSuccess) return fail("hipStreamSynchronize failed");
        g_->ptrs[r_] = buf;
        g_->count[r_] = n;
        g_->op[r_] = int(op);
        g_->dev[r_] = device_;
        if (!g_->barrier()) return fail_group();
        Ptrs src{};
        for (int r = 0; r < n_; ++r) {
            if (g_->count[r] != n || g_->op[r] != int(op))   // every member must make the same call
                return fail("in-process group: members called all-reduce with different counts or operations");
            src.p[r] = g_->ptrs[r];
            if (g_->dev[r] != device_ && !(peer_ & (1u << r))) {   // read a peer device's buffer over the fabric
                const hipError_t e = hipDeviceEnablePeerAccess(g_->dev[r], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return fail("in-process group: peer access between the members' devices is unavailable");
                (void)hipGetLastError();
                peer_ |= 1u << r;
            }
        }
        if (n > 0) {
            const int grid = int(std::min<size_t>((n + 255) / 256, 1024));
            switch (op) {
                case RedOp::SumF64: rank_reduce_kernel<int(RedOp::SumF64)><<<grid, 256, 0, s>>>(src, n_, n, tmp_); break;
                case RedOp::MinF64: rank_reduce_kernel<int(RedOp::MinF64)><<<grid, 256, 0, s>>>(src, n_, n, tmp_); break;
                case RedOp::MaxU8: rank_reduce_kernel<int(RedOp::MaxU8)><<<grid, 256, 0, s>>>(src, n_, n, tmp_); break;
            }
            if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
                return fail("rank reduction kernel failed");
        }
        if (!g_->barrier()) return fail_group();
        if (n > 0 && hipMemcpyAsync(buf, tmp_, n * esz, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return fail("copy of the reduced values failed");
        return 0;
    }

private:
    int fail(const char* m) {   // the members are out of step now: poison the group
        err_ = m;
        g_->poison(std::string("member ") + std::to_string(r_) + ": " + m);
        return 1;
    }
    int fail_group() {
        err_ = "in-process group failed: " + g_->reason();
        return 1;
    }
    std::shared_ptr<LocalGroup> g_;
    int device_;
    unsigned peer_ = 0;
    void* tmp_ = nullptr;
    size_t tmp_bytes_ = 0;
};

}  // namespace

void local_group_id(int nranks, uint8_t id[kCommIdBytes]) {
    std::memset(id, 0, kCommIdBytes);
    std::memcpy(id, kLocalMagic, 8);
    const uint64_t serial = g_serial.fetch_add(1);
    std::memcpy(id + 8, &serial, 8);
    const int32_t n = nranks;
    std::memcpy(id + 16, &n, 4);
}

bool is_local_group_id(const uint8_t id[kCommIdBytes]) { return std::memcmp(id, kLocalMagic, 8) == 0; }

std::unique_ptr<Collective> make_rccl_collective(int nranks, int rank, const uint8_t id[kCommIdBytes],
                                                 std::string& err) {
    static_assert(sizeof(ncclUniqueId) == kCommIdBytes, "ncclUniqueId size");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    void* agree = Collective::reserve_agreement(err);   // before joining: a failure here leaves no member short
    if (!agree) return nullptr;
    ncclComm_t c = nullptr;
    // non-blocking: a member that never joins ends the set-up after
    // WFSA_COMM_TIMEOUT_S instead of blocking this thread for good
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&c, nranks, uid, rank, &cfg);
    if (c && (r == ncclInProgress || (r == ncclSuccess && !cfg.blocking))) r = rccl_settle(c, comm_timeout_s());
    if (r != ncclSuccess) {
        err = r == ncclInProgress ? std::string("ncclCommInitRankConfig: the members did not all join within WFSA_COMM_TIMEOUT_S")
                                  : std::string("ncclCommInitRankConfig failed: ") + ncclGetErrorString(r);
        if (c) (void)ncclCommAbort(c);
        (void)hipFree(agree);
        return nullptr;
    }
    auto col = std::make_unique<RcclCollective>(c, nranks, rank);
    col->adopt_agreement(agree);
    return col;
}

std::unique_ptr<Collective> make_local_collective(int nranks, int rank, const uint8_t id[kCommIdBytes],
                                                  int device, std::string& err) {
    int32_t n = 0;
    uint64_t serial = 0;
    std::memcpy(&serial, id + 8, 8);
    std::memcpy(&n, id + 16, 4);
    if (n != nranks || n < 1 || n > kLocalMaxRanks) {
        err = "in-process group: size does not match its id (at most 16 members)";
        return nullptr;
    }
    void* agree = Collective::reserve_agreement(err);   // before joining the group (see collective.hpp)
    if (!agree) return nullptr;
    std::shared_ptr<LocalGroup> g;
    {
        std::lock_guard<std::mutex> lk(g_reg_m);
        auto& slot = g_reg[serial];
        if (!slot) {
            slot = std::make_shared<LocalGroup>();
            slot->n = n;
            const char* e = std::getenv("WFSA_GROUP_TIMEOUT_S");
            const int v = e ? std::atoi(e) : 0;
            if (v > 0) slot->limit_s = v;
        }
        g = slot;
        if (++g->joined == n) g_reg.erase(serial);   // every member holds the group now
    }
    auto col = std::make_unique<LocalCollective>(g, rank, device);
    col->adopt_agreement(agree);
    return col;
}

int rccl_unique_id(uint8_t id[kCommIdBytes], std::string& err) {
    ncclUniqueId uid;
    ncclResult_t r = ncclGetUniqueId(&uid);
    if (r != ncclSuccess) {
        err = std::string("ncclGetUniqueId failed: ") + ncclGetErrorString(r);
        return 1;
    }
    std::memcpy(id, &uid, sizeof uid);
    return 0;
}


// ---- host-callback transport ---------------------------------------------

namespace {

// Every all-reduce is two callback calls: a fixed 8-byte header (max of
// bytes; byte 0 = poisoned), then the payload.  abort() on a member standing
// between collectives sends the header alone with the poison byte set: the
// other members are waiting in (or will enter) a header exchange of the same
// size whatever collective they are in, so theirs completes with the poison
// and fails at once -- the abort reaches every rank through the transport
// itself.  The aborting call returns once every member has entered a
// collective (or the transport reports a closed peer).  A member that dies
// without aborting leaves the others to the callback transport's own timeout.
class HostCollective final : public Collective {
public:
    HostCollective(int n, int r, HostAllreduceFn fn, void* user) : fn_(fn), user_(user) {
        n_ = n;
        r_ = r;
        // fault injection (tests/test_gpu_multiprocess.py): payload number k
        // (from 1) of this member finds its device-to-host copy failed
        if (const char* e = std::getenv("WFSA_FAULT_HOST_D2H")) fault_at_ = std::atoi(e);
    }
    const char* kind() const override { return "host"; }
    void abort_transport(const std::string&) override {
        if (phase_ != 0 || broken_) return;   // (inside a callback: the exchange is out of step already)
        uint8_t hdr[8] = {1, 0, 0, 0, 0, 0, 0, 0};
        broken_ = true;
        (void)fn_(user_, hdr, 8, 2);
    }
    int transport_allreduce(void* buf, size_t n, RedOp op, hipStream_t s) override {
        if (n == 0) return 0;
        if (broken_) {
            err_ = "host transport: the group was aborted";
            return 1;
        }
        uint8_t hdr[8] = {};
        phase_ = 1;
        const int hr = fn_(user_, hdr, 8, 2);
        phase_ = 0;
        if (hr != 0 || hdr[0] != 0) {
            broken_ = true;
            err_ = hr != 0 ? "host transport: the all-reduce callback failed"
                           : "host transport: another member aborted the group";
            return 1;
        }
        const size_t bytes = n * (op == RedOp::MaxU8 ? 1 : 8);
        if (host_.size() < bytes) host_.resize(bytes);
        // After the header the members are committed to this payload
        // exchange: a local copy failure still joins it (so no member is left
        // in an exchange of n elements while this one sends an 8-byte abort
        // header), with a poisoned buffer -- all bits set: NaN doubles, which
        // make the members' sums and minima non-finite, 0xff bytes -- and
        // then leaves the transport broken: this member makes no further
        // calls, so the others fail at their next header exchange (the
        // callback's own wait limit) at the latest
        bool local_bad = (++payloads_ == fault_at_ ||
                          hipMemcpyAsync(host_.data(), buf, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
                          hipStreamSynchronize(s) != hipSuccess);
        if (local_bad) {
            (void)hipGetLastError();
            std::memset(host_.data(), 0xff, bytes);
        }
        const int32_t code = op == RedOp::SumF64 ? 0 : op == RedOp::MinF64 ? 1 : 2;
        phase_ = 2;
        const int pr = fn_(user_, host_.data(), int64_t(n), code);
        phase_ = 0;
        if (local_bad) {
            broken_ = true;
            err_ = "host transport: device to host copy failed";
            return 1;
        }
        if (pr != 0) {
            broken_ = true;
            err_ = "host transport: the all-reduce callback failed";
            return 1;
        }
        if (hipMemcpyAsync(buf, host_.data(), bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            err_ = "host transport: host to device copy failed";
            return 1;
        }
        return 0;
    }

private:
    HostAllreduceFn fn_;
    void* user_;
    std::vector<uint8_t> host_;
    int phase_ = 0;         // 1 / 2: inside the header / payload callback
    int payloads_ = 0, fault_at_ = 0;   // (fault injection)
    bool broken_ = false;   // aborted, poisoned or a failed callback: the exchange is out of step
};

}  // namespace

std::unique_ptr<Collective> make_host_collective(int nranks, int rank, HostAllreduceFn fn, void* user,
                                                 std::string& err) {
    if (!fn || nranks < 1 || rank < 0 || rank >= nranks) {
        err = "host transport: bad arguments";
        return nullptr;
    }
    void* agree = Collective::reserve_agreement(err);
    if (!agree) return nullptr;
    auto col = std::make_unique<HostCollective>(nranks, rank, fn, user);
    col->adopt_agreement(agree);
    return col;
}

// ---- one-shot peer all-reduce (collective.hpp) ----------------------------

namespace {

struct PeerArgs {
    double* area[kLocalMaxRanks];   // rank r's area as mapped in this process
    const double* src;
    double* dst;
    int64_t n;
    int nranks, me;
    uint64_t seq;
    uint64_t timeout;   // s_memrealtime ticks (100 MHz)
    unsigned* status;   // host-mapped: set to 1 when the call failed
};

__device__ __forceinline__ bool poisoned(double* area, int nranks) {
    return __hip_atomic_load(peer_poison(area, nranks), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

__global__ __launch_bounds__(256) void peer_sum_kernel(PeerArgs a) {
    const int c = int(blockIdx.x);
    const int64_t b = int64_t(c) * kPeerChunk, e = min(a.n, b + kPeerChunk);
    const int par = int(a.seq & 1);
    const size_t my_slot = (size_t(par) * a.nranks + a.me) * kPeerCap;
    __shared__ int late;
    if (threadIdx.x == 0) late = poisoned(a.area[a.me], a.nranks) ? 1 : 0;   // a member failed before: no wait
    __syncthreads();
    if (!late) {
        // this rank's chunk into its slot of every member's area
        for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) {
            const double v = a.src[i];
            for (int r = 0; r < a.nranks; ++r) a.area[r][my_slot + i] = v;
        }
        __threadfence_system();   // the slots before the flags, on every member
        __syncthreads();
        const size_t fl = (size_t(par) * a.nranks + a.me) * kPeerFlags + c;
        if (int(threadIdx.x) < a.nranks)
            __hip_atomic_store(peer_flags(a.area[threadIdx.x], a.nranks) + fl, a.seq, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        // every member's chunk c in this rank's area; a poisoned area ends the wait
        if (int(threadIdx.x) < a.nranks) {
            const uint64_t* f = peer_flags(a.area[a.me], a.nranks) + (size_t(par) * a.nranks + threadIdx.x) * kPeerFlags + c;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.seq) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout || poisoned(a.area[a.me], a.nranks)) {
                    atomicOr(&late, 1);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __threadfence_system();
        __syncthreads();
    }
    if (late) {   // every member's next call fails at entry; the host sees the status
        if (int(threadIdx.x) < a.nranks)
            __hip_atomic_store(peer_poison(a.area[threadIdx.x], a.nranks), uint64_t(1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        if (threadIdx.x == 0) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const double* mine = a.area[a.me] + size_t(par) * a.nranks * kPeerCap;
    for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) {
        double t = 0.0;
        if (!late)
            for (int r = 0; r < a.nranks; ++r) t += mine[size_t(r) * kPeerCap + i];   // rank order: deterministic
        a.dst[i] = late ? __builtin_nan("") : t;
    }
}

// the poison word of every area (Collective::abort)
__global__ void peer_poison_kernel(PeerArgs a) {
    if (int(threadIdx.x) < a.nranks)
        __hip_atomic_store(peer_poison(a.area[threadIdx.x], a.nranks), uint64_t(1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

struct PeerBlob {   // what a rank publishes at set-up
    uint8_t handle[64];
    uint64_t ptr;
    int32_t pid, pad;
};
static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");

// Uncached areas are kept for the life of the process and reused by later
// groups, never handed back to HIP: freed, their pages went on (still mapped
// uncached) to ordinary allocations of later contexts, where the evaluation
// kernels' fp64 atomic adds were lost -- a context made after an in-process
// peer group summed gradients short (round 3; tests/test_gpu_multiprocess.py,
// test_context_after_peer_selftest_is_exact).
std::mutex g_uncached_mu;
std::multimap<size_t, void*> g_uncached_free;

void* uncached_get(size_t bytes) {
    {
        std::lock_guard<std::mutex> lk(g_uncached_mu);
        auto it = g_uncached_free.find(bytes);
        if (it != g_uncached_free.end()) {
            void* p = it->second;
            g_uncached_free.erase(it);
            return p;
        }
    }
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return p;
}

void uncached_put(void* p, size_t bytes) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_uncached_mu);
    g_uncached_free.emplace(bytes, p);
}

double peer_timeout_s() {
    const char* e = std::getenv("WFSA_PEER_TIMEOUT_S");   // (read per set-up: tests shorten it)
    const double v = e ? std::atof(e) : 0.0;
    return v > 0 ? v : 120.0;
}

}  // namespace

class PeerSum {
public:
    ~PeerSum() {
        for (int r = 0; r < n_; ++r)
            if (opened_[r]) (void)hipIpcCloseMemHandle(args_.area[r]);
        if (own_) {   // (no kernel of this group is in flight: its users synchronised first)
            (void)hipDeviceSynchronize();
            uncached_put(own_, own_bytes_);
        }
        if (status_h_) (void)hipHostFree(status_h_);
        if (aux_) (void)hipStreamDestroy(aux_);
        if (area_tbl_) (void)hipFree(area_tbl_);
    }

    // this rank's area and status word (false: err says why).  Always safe to
    // follow with exchange(): a failed set-up still takes part in it.
    bool alloc(int nranks, int me, hipStream_t s, std::string& err) {
        n_ = nranks;
        me_ = me;
        own_bytes_ = peer_area_bytes(n_);
        own_ = static_cast<double*>(uncached_get(own_bytes_));
        bool ok = own_ != nullptr && hipMemsetAsync(own_, 0, own_bytes_, s) == hipSuccess &&
                  hipHostMalloc(reinterpret_cast<void**>(&status_h_), sizeof(unsigned),
                                hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) == hipSuccess &&
                  hipHostGetDevicePointer(reinterpret_cast<void**>(&status_d_), status_h_, 0) == hipSuccess &&
                  hipStreamCreateWithFlags(&aux_, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess;
        if (!ok) {
            (void)hipGetLastError();
            err = "peer set-up: allocation of the receive area failed";
        } else {
            *status_h_ = 0;
        }
        args_.nranks = n_;
        args_.me = me_;
        args_.status = status_d_;
        args_.timeout = uint64_t(peer_timeout_s() * 1e8);
        return ok;
    }

    // maps every member's area; xfer carries the exchange (a byte max-
    // reduction over the transport, dbuf its device buffer).  Every member
    // makes the same calls whatever happened before (ok in/out).
    bool exchange(bool ok, bool same_process, hipStream_t s, void* dbuf,
                  const std::function<int(void*, size_t, RedOp)>& xfer, std::string& err) {
        std::vector<PeerBlob> blobs(static_cast<size_t>(n_));
        std::memset(blobs.data(), 0, blobs.size() * sizeof(PeerBlob));
        PeerBlob& mine = blobs[size_t(me_)];
        if (ok && !same_process) {
            hipIpcMemHandle_t h;
            ok = hipIpcGetMemHandle(&h, own_) == hipSuccess;
            if (ok) std::memcpy(mine.handle, &h, sizeof h);
            else (void)hipGetLastError();
            if (!ok) err = "peer set-up: hipIpcGetMemHandle failed";
        }
        mine.ptr = reinterpret_cast<uint64_t>(own_);
        mine.pid = int32_t(getpid());
        mine.pad = ok ? 0 : 1;   // (a member whose area is unusable says so)
        const size_t bb = blobs.size() * sizeof(PeerBlob);
        if (hipMemcpyAsync(dbuf, blobs.data(), bb, hipMemcpyHostToDevice, s) != hipSuccess ||
            xfer(dbuf, bb, RedOp::MaxU8) != 0 ||
            hipMemcpyAsync(blobs.data(), dbuf, bb, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            err = "peer set-up: exchange failed";
            return false;   // (the transport itself failed: the caller reports it)
        }
        for (int r = 0; r < n_ && ok; ++r) {
            if (blobs[size_t(r)].pad) {
                ok = false;
                err = "peer set-up: another member's area is unusable";
            } else if (r == me_) {
                args_.area[r] = own_;
            } else if (same_process) {
                args_.area[r] = reinterpret_cast<double*>(blobs[size_t(r)].ptr);
            } else {
                hipIpcMemHandle_t h;
                std::memcpy(&h, blobs[size_t(r)].handle, sizeof h);
                void* p = nullptr;
                ok = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess;
                if (ok) {
                    args_.area[r] = static_cast<double*>(p);
                    opened_[r] = true;
                } else {
                    (void)hipGetLastError();
                    err = "peer set-up: a member's area could not be mapped";
                }
            }
        }
        mapped_ = ok;
        return true;
    }
    bool mapped() const { return mapped_; }

    int run(double* buf, size_t n, hipStream_t s) {
        PeerArgs a = args_;
        a.src = buf;
        a.dst = buf;
        a.n = int64_t(n);
        a.seq = ++seq_;
        const int blocks = int((n + kPeerChunk - 1) / kPeerChunk);
        if (blocks == 0) return 0;
        hipLaunchKernelGGL(peer_sum_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, a);
        return hipGetLastError() == hipSuccess ? 0 : 1;
    }

    // a call failed (this rank's wait gave up, or it found its area poisoned)
    bool failed() const { return __atomic_load_n(status_h_, __ATOMIC_ACQUIRE) != 0; }

    // poison every member's area from the host side (on a stream of its own,
    // not waited for: the member's own stream may hold a waiting kernel)
    void poison_all() {
        if (!mapped_) return;
        hipLaunchKernelGGL(peer_poison_kernel, dim3(1), dim3(64), 0, aux_, args_);
        (void)hipGetLastError();
    }

    // an in-kernel exchange's view, with the next sequence number
    bool exchange_view(PeerX& x) {
        if (!area_tbl_) {   // the areas' pointers as a device table (once)
            if (hipMalloc(reinterpret_cast<void**>(&area_tbl_), sizeof(args_.area)) != hipSuccess ||
                hipMemcpy(area_tbl_, args_.area, sizeof(args_.area), hipMemcpyHostToDevice) != hipSuccess) {
                (void)hipGetLastError();
                if (area_tbl_) (void)hipFree(area_tbl_);
                area_tbl_ = nullptr;
                return false;
            }
        }
        x.area = area_tbl_;
        x.on = 1;
        x.nranks = n_;
        x.me = me_;
        x.seq = ++seq_;
        x.timeout = args_.timeout;
        x.status = status_d_;
        return true;
    }

    // selftest access
    PeerArgs& args() { return args_; }
    double* own() const { return own_; }
    unsigned* status_host() const { return status_h_; }
    uint64_t seq() const { return seq_; }

private:
    int n_ = 0, me_ = 0;
    double* own_ = nullptr;
    size_t own_bytes_ = 0;
    unsigned* status_h_ = nullptr;
    unsigned* status_d_ = nullptr;
    hipStream_t aux_ = nullptr;
    bool opened_[kLocalMaxRanks] = {};
    bool mapped_ = false;
    uint64_t seq_ = 0;
    PeerArgs args_{};
    double** area_tbl_ = nullptr;   // args_.area on the device (exchange_view)
};

double comm_timeout_s() {
    const char* e = std::getenv("WFSA_COMM_TIMEOUT_S");   // (read per communicator: tests shorten it)
    const double v = e ? std::atof(e) : 0.0;
    return v > 0 ? v : 300.0;
}

constexpr size_t kAgreeBytes = std::max(size_t(3000) * sizeof(double), size_t(kLocalMaxRanks) * 88);

void* Collective::reserve_agreement(std::string& err) {
    void* b = nullptr;
    if (hipMalloc(&b, kAgreeBytes) != hipSuccess) {
        (void)hipGetLastError();
        err = "communicator set-up: no device memory for the peer path's agreement";
        return nullptr;
    }
    return b;
}

Collective::~Collective() {
    if (agree_buf_) (void)hipFree(agree_buf_);
}

const char* Collective::peer_state() const {
    return peer_st_ == 1 ? "on" : peer_st_ == -1 ? "off" : peer_st_ == -2 ? "failed" : "untried";
}

// Decides once, on the first sum that fits, whether the peer path is used.
// Every member makes the same transport calls whatever fails locally (a
// local failure is carried as its "bad" byte), so no member is left waiting:
// (1) the members' devices (the path is refused when two share a device in
// one process, see collective.hpp), (2) the areas' set-up and exchange, (3) a
// check sum (rank r contributes (r + 1)(i + 1)) through the path, (4) the
// ranks agree -- any failure anywhere and every rank stays on the transport.
int Collective::try_peer(hipStream_t s) {
    const char* pe = std::getenv("WFSA_PEER");   // (read per communicator: tests switch it)
    const int want = pe && pe[0] ? (pe[0] == '0' ? 0 : 1) : -1;
    const bool on = want < 0 ? peer_default() : want == 1;
    if (!on || n_ < 2 || n_ > kLocalMaxRanks) {
        peer_st_ = -1;
        peer_why_ = !on ? "not requested (WFSA_PEER)" : "group size";
        return 0;
    }
    constexpr size_t kCheck = 3000;   // spans three chunks
    static_assert(kCheck * sizeof(double) <= kAgreeBytes && kLocalMaxRanks * sizeof(PeerBlob) <= kAgreeBytes,
                  "the agreement buffer holds the check sum and the set-up blobs");
    // the agreement's buffer, reserved with the communicator: no allocation
    // here can fail, so every member takes part in every exchange below and a
    // local failure travels as its "bad" byte
    uint8_t* d = static_cast<uint8_t*>(agree_buf_);
    if (!d) {   // (never: the communicator is not made without it)
        err_ = "peer set-up: no agreement buffer";
        return 1;
    }
    auto xfer = [&](void* b, size_t n, RedOp op) { return transport_allreduce(b, n, op, s); };
    auto agree = [&](bool mine_ok, bool& all_ok) {   // a byte per rank, max-reduced
        std::vector<uint8_t> bad(size_t(n_), 0);
        bad[size_t(r_)] = mine_ok ? 0 : 1;
        if (hipMemcpyAsync(d, bad.data(), bad.size(), hipMemcpyHostToDevice, s) != hipSuccess) return 1;
        if (transport_allreduce(d, bad.size(), RedOp::MaxU8, s)) return 1;
        if (hipMemcpyAsync(bad.data(), d, bad.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return 1;
        all_ok = true;
        for (uint8_t b : bad) all_ok &= b == 0;
        return 0;
    };
    auto done = [&](int rc) { return rc; };
    std::string why;
    // (1) devices: a byte per rank holding its device + 1
    {
        std::vector<uint8_t> dv(size_t(n_), 0);
        dv[size_t(r_)] = uint8_t(std::max(0, device()) + 1);
        if (hipMemcpyAsync(d, dv.data(), dv.size(), hipMemcpyHostToDevice, s) != hipSuccess ||
            transport_allreduce(d, dv.size(), RedOp::MaxU8, s) != 0 ||
            hipMemcpyAsync(dv.data(), d, dv.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return done(1);
        if (same_process())
            for (int a = 0; a < n_; ++a)
                for (int b = a + 1; b < n_; ++b)
                    if (dv[size_t(a)] == dv[size_t(b)]) {
                        peer_st_ = -1;
                        peer_why_ = "members share a device in one process (their kernels need not run concurrently)";
                        if (std::getenv("WFSA_VERBOSE"))
                            std::fprintf(stderr, "[wfsa] rank %d: peer all-reduce off: %s\n", r_, peer_why_.c_str());
                        return done(0);
                    }
    }
    // (2) areas
    auto p = std::make_unique<PeerSum>();
    bool ok = p->alloc(n_, r_, s, why);
    if (!p->exchange(ok, same_process(), s, d, xfer, why)) return done(1);
    ok = p->mapped();
    // (3) the check sum
    if (ok) {
        std::vector<double> h(kCheck);
        for (size_t i = 0; i < kCheck; ++i) h[i] = double(r_ + 1) * double(i + 1);
        double* dd = reinterpret_cast<double*>(d);
        ok = hipMemcpyAsync(dd, h.data(), kCheck * sizeof(double), hipMemcpyHostToDevice, s) == hipSuccess &&
             p->run(dd, kCheck, s) == 0 &&
             hipMemcpyAsync(h.data(), dd, kCheck * sizeof(double), hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess && !p->failed();
        const double tri = double(n_) * double(n_ + 1) / 2.0;
        for (size_t i = 0; i < kCheck && ok; ++i) ok = h[i] == tri * double(i + 1);
        if (!ok && why.empty()) why = "the check sum through the peer path was wrong or timed out";
    }
    // (4) agree
    bool all = false;
    if (agree(ok, all)) return done(1);
    if (std::getenv("WFSA_VERBOSE"))
        std::fprintf(stderr, "[wfsa] rank %d: peer all-reduce %s%s%s\n", r_, all ? "on" : "failed",
                     why.empty() ? "" : ": ", why.c_str());
    if (all) {
        peer_ = std::move(p);
        peer_st_ = 1;
        peer_why_.clear();
    } else {
        peer_st_ = -2;
        peer_why_ = why.empty() ? "another member's set-up or check failed" : why;
    }
    return done(0);
}

bool Collective::peer_exchange(PeerX& x) {
    x = PeerX{};
    if (peer_st_ != 1 || !peer_ || aborted_) return false;
    return peer_->exchange_view(x);
}

int Collective::check() {
    if (aborted_) {
        err_ = "communicator aborted: " + abort_why_;
        return 1;
    }
    if (peer_ && peer_->failed()) {
        err_ = "peer all-reduce: a member did not arrive within WFSA_PEER_TIMEOUT_S, or failed";
        return 1;
    }
    return 0;
}

void Collective::abort(const char* why) {
    if (aborted_) return;
    aborted_ = true;
    abort_why_ = why ? why : "";
    if (peer_) peer_->poison_all();
    abort_transport(abort_why_);
}

int Collective::allreduce(void* buf, size_t n, RedOp op, hipStream_t s) {
    if (check()) return 1;
    if (op == RedOp::SumF64 && n > 0 && n <= kPeerCap) {
        if (peer_st_ == 0 && try_peer(s)) {
            if (err_.empty()) err_ = "peer all-reduce set-up failed";
            return 1;
        }
        if (peer_st_ == 1) {
            if (peer_->run(static_cast<double*>(buf), n, s)) {
                err_ = "peer all-reduce launch failed";
                return 1;
            }
            return 0;
        }
    }
    return transport_allreduce(buf, n, op, s);
}

// ---- the peer kernel on one device (collective.hpp: peer_selftest) --------

namespace {

__global__ void selftest_fill_kernel(PeerArgs a, int rank, uint64_t seq, int with_flags) {
    // what member `rank` would have stored into this rank's area: its slot
    // (value (rank + 1) * (i + 1) + i * 1e-3) and the flags of every chunk
    const int par = int(seq & 1);
    double* area = a.area[a.me];
    const size_t slot = (size_t(par) * a.nranks + rank) * kPeerCap;
    for (int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < a.n; i += int64_t(gridDim.x) * blockDim.x)
        area[slot + size_t(i)] = double(rank + 1) * double(i + 1) + double(i) * 1e-3;
    if (with_flags && blockIdx.x == 0) {
        const int chunks = int((a.n + kPeerChunk - 1) / kPeerChunk);
        for (int c = int(threadIdx.x); c < chunks; c += int(blockDim.x))
            __hip_atomic_store(peer_flags(area, a.nranks) + (size_t(par) * a.nranks + rank) * kPeerFlags + c, seq,
                               __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

int peer_selftest(int nranks, int64_t n, double timeout_s, int mode, double out[4], std::string& err) {
    if (nranks < 2 || nranks > kLocalMaxRanks || n < 1 || n > int64_t(kPeerCap) || mode < 0 || mode > 2 ||
        !(timeout_s > 0)) {
        err = "peer selftest: bad arguments";
        return 1;
    }
    hipStream_t s = nullptr;
    if (hipStreamCreate(&s) != hipSuccess) {
        err = "peer selftest: no stream";
        return 1;
    }
    // rank 0's PeerSum; the other members' areas are plain local areas of the
    // same layout (only their poison words and rank 0's stores land there)
    PeerSum p;
    std::vector<void*> others;
    auto cleanup = [&](int rc) {
        (void)hipStreamSynchronize(s);
        for (void* o : others) uncached_put(o, peer_area_bytes(nranks));
        (void)hipStreamDestroy(s);
        return rc;
    };
    if (!p.alloc(nranks, 0, s, err)) return cleanup(1);
    PeerArgs& a = p.args();
    a.area[0] = p.own();
    for (int r = 1; r < nranks; ++r) {
        void* o = uncached_get(peer_area_bytes(nranks));
        if (!o || hipMemsetAsync(o, 0, peer_area_bytes(nranks), s) != hipSuccess) {
            err = "peer selftest: allocation failed";
            return cleanup(1);
        }
        others.push_back(o);
        a.area[r] = static_cast<double*>(o);
    }
    a.timeout = uint64_t(timeout_s * 1e8);
    double* buf = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&buf), size_t(n) * sizeof(double)) != hipSuccess) {
        err = "peer selftest: allocation failed";
        return cleanup(1);
    }
    std::vector<double> h(static_cast<size_t>(n));
    for (int64_t i = 0; i < n; ++i) h[size_t(i)] = double(i + 1) + double(i) * 1e-3;   // rank 0's own values
    const uint64_t seq = p.seq() + 1;
    PeerArgs fa = a;
    fa.n = n;
    bool ok = hipMemcpyAsync(buf, h.data(), size_t(n) * sizeof(double), hipMemcpyHostToDevice, s) == hipSuccess;
    for (int r = 1; r < nranks && ok; ++r) {
        const int flags = mode == 1 && r == nranks - 1 ? 0 : 1;   // mode 1: the last member never arrives
        hipLaunchKernelGGL(selftest_fill_kernel, dim3(64), dim3(256), 0, s, fa, r, seq, flags);
        ok = hipGetLastError() == hipSuccess;
    }
    if (ok && mode == 2) {   // another member failed before this call
        hipLaunchKernelGGL(peer_poison_kernel, dim3(1), dim3(64), 0, s, a);
        ok = hipGetLastError() == hipSuccess;
    }
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    const auto t0 = std::chrono::steady_clock::now();
    ok = ok && p.run(buf, size_t(n), s) == 0 && hipStreamSynchronize(s) == hipSuccess;
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::vector<double> got(static_cast<size_t>(n));
    ok = ok && hipMemcpy(got.data(), buf, size_t(n) * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
    int poisoned_areas = 0;
    for (int r = 0; r < nranks && ok; ++r) {
        uint64_t w = 0;
        const uint8_t* base = reinterpret_cast<const uint8_t*>(a.area[r]) + peer_area_bytes(nranks) - 16;
        ok = hipMemcpy(&w, base, sizeof w, hipMemcpyDeviceToHost) == hipSuccess;
        poisoned_areas += w != 0;
    }
    (void)hipFree(buf);
    if (!ok) {
        err = "peer selftest: a HIP call failed";
        return cleanup(1);
    }
    double metric = 0.0;
    if (mode == 0) {
        for (int64_t i = 0; i < n; ++i) {
            double want = 0.0;   // rank order, as the kernel sums
            for (int r = 0; r < nranks; ++r) want += double(r + 1) * double(i + 1) + double(i) * 1e-3;
            metric = std::max(metric, std::fabs(got[size_t(i)] - want));
        }
    } else {
        for (double v : got) metric += std::isnan(v) ? 1.0 : 0.0;
    }
    out[0] = metric;
    out[1] = double(*p.status_host());
    out[2] = double(poisoned_areas);
    out[3] = el;
    return cleanup(0);
}

}  // namespace wfsa
