// Collective transports (collective.hpp): RCCL across processes, and the
// in-process group of contexts driven by threads.
#include "collective.hpp"

#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
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

class RcclCollective final : public Collective {
public:
    RcclCollective(ncclComm_t c, int n, int r) : comm_(c) {
        n_ = n;
        r_ = r;
    }
    ~RcclCollective() override { (void)ncclCommDestroy(comm_); }
    const char* kind() const override { return "rccl"; }
    bool peer_default() const override { return true; }
    int transport_allreduce(void* buf, size_t n, RedOp op, hipStream_t s) override {
        if (n == 0) return 0;
        ncclDataType_t t = op == RedOp::MaxU8 ? ncclUint8 : ncclDouble;
        ncclRedOp_t o = op == RedOp::SumF64 ? ncclSum : op == RedOp::MinF64 ? ncclMin : ncclMax;
        ncclResult_t r = ncclAllReduce(buf, buf, n, t, o, comm_, s);
        if (r != ncclSuccess) {
            err_ = std::string("ncclAllReduce failed: ") + ncclGetErrorString(r);
            return 1;
        }
        return 0;
    }

private:
    ncclComm_t comm_;
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

    bool poisoned = false;   // a member timed out: the group is out of step for good

    // false on a timeout (a member that never arrives: a bug upstream,
    // reported instead of hanging the process) or once the group is poisoned.
    // A timeout poisons the group -- the late member's arrival would
    // otherwise release a later barrier at the wrong count and combine
    // buffers from different calls -- so every later call fails at once.
    // WFSA_GROUP_TIMEOUT_S sets the limit (default 600 s: a healthy rank may
    // do long host work, e.g. a sparse factorisation, between collectives).
    bool barrier() {
        static const int limit_s = [] {
            const char* e = std::getenv("WFSA_GROUP_TIMEOUT_S");
            const int v = e ? std::atoi(e) : 0;
            return v > 0 ? v : 600;
        }();
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
        poisoned = true;
        cv.notify_all();
        return false;
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
        if (!g_->barrier()) return fail("in-process group: a member did not arrive in time (WFSA_GROUP_TIMEOUT_S), or the group failed before");
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
        if (!g_->barrier()) return fail("in-process group: a member did not arrive in time (WFSA_GROUP_TIMEOUT_S), or the group failed before");
        if (n > 0 && hipMemcpyAsync(buf, tmp_, n * esz, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return fail("copy of the reduced values failed");
        return 0;
    }

private:
    int fail(const char* m) {
        err_ = m;
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
    ncclComm_t c = nullptr;
    ncclResult_t r = ncclCommInitRank(&c, nranks, uid, rank);
    if (r != ncclSuccess) {
        err = std::string("ncclCommInitRank failed: ") + ncclGetErrorString(r);
        return nullptr;
    }
    return std::make_unique<RcclCollective>(c, nranks, rank);
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
    std::shared_ptr<LocalGroup> g;
    {
        std::lock_guard<std::mutex> lk(g_reg_m);
        auto& slot = g_reg[serial];
        if (!slot) {
            slot = std::make_shared<LocalGroup>();
            slot->n = n;
        }
        g = slot;
        if (++g->joined == n) g_reg.erase(serial);   // every member holds the group now
    }
    return std::make_unique<LocalCollective>(g, rank, device);
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

class HostCollective final : public Collective {
public:
    HostCollective(int n, int r, HostAllreduceFn fn, void* user) : fn_(fn), user_(user) {
        n_ = n;
        r_ = r;
    }
    const char* kind() const override { return "host"; }
    int transport_allreduce(void* buf, size_t n, RedOp op, hipStream_t s) override {
        if (n == 0) return 0;
        const size_t bytes = n * (op == RedOp::MaxU8 ? 1 : 8);
        if (host_.size() < bytes) host_.resize(bytes);
        if (hipMemcpyAsync(host_.data(), buf, bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            err_ = "host transport: device to host copy failed";
            return 1;
        }
        const int32_t code = op == RedOp::SumF64 ? 0 : op == RedOp::MinF64 ? 1 : 2;
        if (fn_(user_, host_.data(), int64_t(n), code) != 0) {
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
};

}  // namespace

std::unique_ptr<Collective> make_host_collective(int nranks, int rank, HostAllreduceFn fn, void* user,
                                                 std::string& err) {
    if (!fn || nranks < 1 || rank < 0 || rank >= nranks) {
        err = "host transport: bad arguments";
        return nullptr;
    }
    return std::make_unique<HostCollective>(nranks, rank, fn, user);
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
    unsigned* status;   // set to 1 on a timeout
};

__device__ __forceinline__ uint64_t* peer_flags(double* area, int nranks) {
    return reinterpret_cast<uint64_t*>(area + 2 * size_t(nranks) * kPeerCap);
}

__global__ __launch_bounds__(256) void peer_sum_kernel(PeerArgs a) {
    const int c = int(blockIdx.x);
    const int64_t b = int64_t(c) * kPeerChunk, e = min(a.n, b + kPeerChunk);
    const int par = int(a.seq & 1);
    const size_t my_slot = (size_t(par) * a.nranks + a.me) * kPeerCap;
    // this rank's chunk into its slot of every member's area
    for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) {
        const double v = a.src[i];
        for (int r = 0; r < a.nranks; ++r) a.area[r][my_slot + i] = v;
    }
    __threadfence_system();   // the slots before the flags, on every member
    __syncthreads();
    const size_t fl = (size_t(par) * a.nranks + a.me) * kPeerMaxChunks + c;
    if (int(threadIdx.x) < a.nranks)
        __hip_atomic_store(peer_flags(a.area[threadIdx.x], a.nranks) + fl, a.seq, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    // every member's chunk c in this rank's area
    __shared__ int late;
    if (threadIdx.x == 0) late = 0;
    __syncthreads();
    if (int(threadIdx.x) < a.nranks) {
        const uint64_t* f = peer_flags(a.area[a.me], a.nranks) + (size_t(par) * a.nranks + threadIdx.x) * kPeerMaxChunks + c;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < a.seq) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout) {
                atomicOr(&late, 1);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __threadfence_system();
    __syncthreads();
    if (late && threadIdx.x == 0) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const double* mine = a.area[a.me] + size_t(par) * a.nranks * kPeerCap;
    for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) {
        double t = 0.0;
        for (int r = 0; r < a.nranks; ++r) t += mine[size_t(r) * kPeerCap + i];   // rank order: deterministic
        a.dst[i] = late ? __builtin_nan("") : t;
    }
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
// peer group summed gradients short (tests/test_gpu_multiprocess.py,
// test_context_after_peer_group_is_exact).
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
        if (status_) (void)hipFree(status_);
    }

    // maps every member's area; the transport carries the exchange.  Every
    // member makes the same calls (false: err says why; the caller agrees
    // with the others before using the path)
    bool setup(Collective& c, bool same_process, hipStream_t s,
               const std::function<int(void*, size_t, RedOp)>& xfer, std::string& err) {
        n_ = c.nranks();
        me_ = c.rank();
        const size_t bytes = 2 * size_t(n_) * kPeerCap * sizeof(double) +
                             2 * size_t(n_) * kPeerMaxChunks * sizeof(uint64_t);
        own_ = static_cast<double*>(uncached_get(bytes));
        own_bytes_ = bytes;
        bool ok = own_ != nullptr && hipMemsetAsync(own_, 0, bytes, s) == hipSuccess &&
                  hipMalloc(reinterpret_cast<void**>(&status_), sizeof(unsigned)) == hipSuccess &&
                  hipMemsetAsync(status_, 0, sizeof(unsigned), s) == hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess;
        if (!ok) (void)hipGetLastError();
        std::vector<PeerBlob> blobs(static_cast<size_t>(n_));
        std::memset(blobs.data(), 0, blobs.size() * sizeof(PeerBlob));
        PeerBlob& mine = blobs[size_t(me_)];
        if (ok && !same_process) {
            hipIpcMemHandle_t h;
            ok = hipIpcGetMemHandle(&h, own_) == hipSuccess;
            if (ok) std::memcpy(mine.handle, &h, sizeof h);
            else (void)hipGetLastError();
        }
        mine.ptr = reinterpret_cast<uint64_t>(own_);
        mine.pid = int32_t(getpid());
        // exchange: every rank's blob in its own slot, the rest zero, max-reduced
        void* dbuf = nullptr;
        const size_t bb = blobs.size() * sizeof(PeerBlob);
        if (hipMalloc(&dbuf, bb) != hipSuccess) {
            err = "peer set-up: allocation failed";
            return false;
        }
        if (hipMemcpyAsync(dbuf, blobs.data(), bb, hipMemcpyHostToDevice, s) != hipSuccess ||
            xfer(dbuf, bb, RedOp::MaxU8) != 0 ||
            hipMemcpyAsync(blobs.data(), dbuf, bb, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            (void)hipFree(dbuf);
            err = "peer set-up: exchange failed";
            return false;
        }
        (void)hipFree(dbuf);
        for (int r = 0; r < n_ && ok; ++r) {
            if (r == me_) {
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
                }
            }
        }
        if (!ok) err = "peer set-up: a member's area could not be mapped";
        static const double limit_s = [] {
            const char* e = std::getenv("WFSA_PEER_TIMEOUT_S");
            const double v = e ? std::atof(e) : 0.0;
            return v > 0 ? v : 10.0;
        }();
        args_.nranks = n_;
        args_.me = me_;
        args_.status = status_;
        args_.timeout = uint64_t(limit_s * 1e8);
        return ok;
    }

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

    // a wait that gave up since the set-up (reads the status word)
    bool timed_out(hipStream_t s) {
        unsigned h = 0;
        if (hipMemcpyAsync(&h, status_, sizeof h, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return true;
        return h != 0;
    }

private:
    int n_ = 0, me_ = 0;
    double* own_ = nullptr;
    size_t own_bytes_ = 0;
    unsigned* status_ = nullptr;
    bool opened_[kLocalMaxRanks] = {};
    uint64_t seq_ = 0;
    PeerArgs args_{};
};

Collective::~Collective() = default;

const char* Collective::peer_state() const {
    return peer_st_ == 1 ? "on" : peer_st_ == -1 ? "off" : peer_st_ == -2 ? "failed" : "untried";
}

// Decides once, on the first sum that fits, whether the peer path is used:
// the set-up on every rank, then a check sum (rank r contributes (r + 1)(i + 1))
// through it, then the ranks agree over the transport -- any failure anywhere
// and every rank stays on the transport.
int Collective::try_peer(hipStream_t s) {
    const char* pe = std::getenv("WFSA_PEER");   // (read per communicator: tests switch it)
    const int want = pe && pe[0] ? (pe[0] == '0' ? 0 : 1) : -1;
    const bool on = want < 0 ? peer_default() : want == 1;
    if (!on || n_ < 2 || n_ > kLocalMaxRanks) {
        peer_st_ = -1;
        return 0;
    }
    auto xfer = [&](void* b, size_t n, RedOp op) { return transport_allreduce(b, n, op, s); };
    auto p = std::make_unique<PeerSum>();
    std::string why;
    bool ok = p->setup(*this, same_process(), s, xfer, why);
    constexpr size_t kCheck = 3000;   // spans three chunks
    std::vector<double> h(kCheck);
    double* d = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&d), kCheck * sizeof(double)) != hipSuccess) return 1;
    if (ok) {
        for (size_t i = 0; i < kCheck; ++i) h[i] = double(r_ + 1) * double(i + 1);
        ok = hipMemcpyAsync(d, h.data(), kCheck * sizeof(double), hipMemcpyHostToDevice, s) == hipSuccess &&
             p->run(d, kCheck, s) == 0 &&
             hipMemcpyAsync(h.data(), d, kCheck * sizeof(double), hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess && !p->timed_out(s);
        const double tri = double(n_) * double(n_ + 1) / 2.0;
        for (size_t i = 0; i < kCheck && ok; ++i) ok = h[i] == tri * double(i + 1);
    }
    // agree: a byte per rank, max-reduced over the transport
    std::vector<uint8_t> bad(size_t(n_), 0);
    bad[size_t(r_)] = ok ? 0 : 1;
    int rc = hipMemcpyAsync(d, bad.data(), bad.size(), hipMemcpyHostToDevice, s) == hipSuccess ? 0 : 1;
    if (!rc) rc = transport_allreduce(d, bad.size(), RedOp::MaxU8, s);
    if (!rc)
        rc = (hipMemcpyAsync(bad.data(), d, bad.size(), hipMemcpyDeviceToHost, s) == hipSuccess &&
              hipStreamSynchronize(s) == hipSuccess) ? 0 : 1;
    (void)hipFree(d);
    if (rc) return 1;
    bool all = true;
    for (uint8_t b : bad) all &= b == 0;
    if (std::getenv("WFSA_VERBOSE"))
        std::fprintf(stderr, "[wfsa] rank %d: peer all-reduce %s%s%s\n", r_, all ? "on" : "failed",
                     why.empty() ? "" : ": ", why.c_str());
    if (all) {
        peer_ = std::move(p);
        peer_st_ = 1;
    } else {
        peer_st_ = -2;
    }
    return 0;
}

int Collective::allreduce(void* buf, size_t n, RedOp op, hipStream_t s) {
    if (op == RedOp::SumF64 && n > 0 && n <= kPeerCap) {
        if (peer_st_ == 0 && try_peer(s)) {
            err_ = "peer all-reduce set-up failed";
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

}  // namespace wfsa
