// Collective transports (collective.hpp): RCCL across processes, and the
// in-process group of contexts driven by threads.
#include "collective.hpp"

#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>

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
    int allreduce(void* buf, size_t n, RedOp op, hipStream_t s) override {
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

    // false on a 120 s timeout (a member that never arrives: a bug upstream,
    // reported instead of hanging the process)
    bool barrier() {
        std::unique_lock<std::mutex> lk(m);
        const uint64_t g0 = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        return cv.wait_for(lk, std::chrono::seconds(120), [&] { return gen != g0; });
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
    int allreduce(void* buf, size_t n, RedOp op, hipStream_t s) override {
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
        if (!g_->barrier()) return fail("in-process group: a member did not arrive within 120 s");
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
        if (!g_->barrier()) return fail("in-process group: a member did not arrive within 120 s");
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

}  // namespace wfsa
