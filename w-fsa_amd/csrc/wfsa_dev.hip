// Implementation of the C-ABI device boundary declared in include/wfsa_dev.h.
//
// A context owns one HIP stream on one gfx950 device, the compiled trellis
// automaton, the packed corpus, per-wave scratch and (optionally) an RCCL
// communicator.  Per iteration the host sends w_full (n_params doubles) and
// receives [loglik, grad_full] (n_params+1 doubles); everything else stays in
// HBM.
#include "wfsa_dev.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "fb_kernels.hpp"
#include "trellis_model.hpp"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) return fail(WFSA_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

#define RCCL_TRY(expr)                                                                                 \
    do {                                                                                               \
        ncclResult_t r_ = (expr);                                                                      \
        if (r_ != ncclSuccess) return fail(WFSA_ERR_RCCL, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)

// device buffer (RAII)
template <class T>
struct DevBuf {
    T* ptr = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        n = 0;
    }
    hipError_t alloc(size_t count) {
        if (count <= n && ptr) return hipSuccess;
        release();
        const size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&ptr), bytes);
        if (e == hipSuccess) n = std::max<size_t>(count, 1);
        return e;
    }
    hipError_t upload(const T* src, size_t count, hipStream_t s) {
        hipError_t e = alloc(count);
        if (e != hipSuccess || count == 0) return e;
        return hipMemcpyAsync(ptr, src, count * sizeof(T), hipMemcpyHostToDevice, s);
    }
};

constexpr int kLdsPerCu = 163840;
constexpr int kNumCu = 256;

}  // namespace

struct wfsa_dev {
    int device = 0;
    int n_cu = kNumCu;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;

    // model
    bool has_model = false;
    int32_t n_params = 0, n_nodes = 0, start = 0;
    int64_t n_edges = 0, n_end = 0;
    DevBuf<int32_t> o_ptr, o_dst, o_pptr, o_pidx, x_ptr, x_pptr, x_pidx;
    DevBuf<uint8_t> o_byte;
    DevBuf<double> o_w, x_w, node_end, node_end_count;

    // corpus
    bool has_corpus = false;
    int64_t n_strings = 0, total_sym = 0;
    int32_t max_len = 0;
    DevBuf<uint8_t> sym;
    DevBuf<int64_t> off;
    DevBuf<double> p;
    DevBuf<int32_t> list_all;

    // tiers: strings whose trellis fits the small slab / the large slab
    bool tiers_ready = false;
    wfsa::SlabConfig cfg[2];
    wfsa::SlabLayout lay[2];
    int grid[2] = {0, 0};
    int32_t n_list[2] = {0, 0};
    DevBuf<int32_t> list[2];
    DevBuf<uint8_t> overflow;

    // work buffers
    DevBuf<double> w_full, out, ll_part, logq, pcount;
    DevBuf<uint8_t> used, recog;
    DevBuf<unsigned long long> live;
    double* pinned = nullptr;   // n_params + 1 doubles
    size_t pinned_n = 0;

    // communicator
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;

    wfsa_dev_stats stats{};
};

namespace {

int check_ctx(wfsa_dev* ctx) {
    if (!ctx) return fail(WFSA_ERR_ARG, "null context");
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail(WFSA_ERR_HIP, "hipSetDevice: %s", hipGetErrorString(e));
    return WFSA_OK;
}

// Slab capacities for a per-wave LDS budget: fixed part (position arrays and
// the node->slot map) first, the rest split between frontier entries (20 B)
// and live edges (12 B) at 1 : 1.5.
bool make_slab(int32_t budget, int32_t max_len, int32_t n_nodes, int32_t waves_per_block,
               wfsa::SlabConfig& cfg, wfsa::SlabLayout& lay) {
    const int64_t fixed = 12 * int64_t(max_len + 2) + 4 * int64_t(n_nodes) + 16;
    const int64_t rem = int64_t(budget) - fixed;
    if (rem < 38 * 64) return false;
    int32_t cap_f = int32_t(rem / 38) & ~1;
    int32_t cap_e = int32_t((rem - 20 * int64_t(cap_f)) / 12);
    lay = wfsa::slab_layout(cap_f, cap_e, max_len, n_nodes);
    while (lay.total > budget && cap_e > 64) {
        cap_e -= 16;
        lay = wfsa::slab_layout(cap_f, cap_e, max_len, n_nodes);
    }
    if (lay.total > budget) return false;
    cfg.cap_f = cap_f;
    cfg.cap_e = cap_e;
    cfg.max_len = max_len;
    cfg.n_nodes = n_nodes;
    cfg.bytes = lay.total;
    cfg.waves_per_block = waves_per_block;
    return true;
}

int grid_for(const wfsa::SlabConfig& c, int n_cu, int32_t n_list) {
    const int block_lds = c.bytes * c.waves_per_block;
    int per_cu = std::max(1, std::min(kLdsPerCu / std::max(block_lds, 1), 32 / c.waves_per_block));
    per_cu = std::min(per_cu, 8);
    const int64_t want = (int64_t(n_list) + c.waves_per_block - 1) / c.waves_per_block;
    return int(std::max<int64_t>(1, std::min<int64_t>(want, int64_t(n_cu) * per_cu)));
}

wfsa::FBArgs base_args(wfsa_dev* ctx, int tier) {
    wfsa::FBArgs a{};
    a.m.o_ptr = ctx->o_ptr.ptr;
    a.m.o_byte = ctx->o_byte.ptr;
    a.m.o_dst = ctx->o_dst.ptr;
    a.m.o_pptr = ctx->o_pptr.ptr;
    a.m.o_pidx = ctx->o_pidx.ptr;
    a.m.o_w = ctx->o_w.ptr;
    a.m.x_ptr = ctx->x_ptr.ptr;
    a.m.x_pptr = ctx->x_pptr.ptr;
    a.m.x_pidx = ctx->x_pidx.ptr;
    a.m.x_w = ctx->x_w.ptr;
    a.m.node_end = ctx->node_end.ptr;
    a.m.node_end_count = ctx->node_end_count.ptr;
    a.m.n_nodes = ctx->n_nodes;
    a.m.start = ctx->start;
    a.sym = ctx->sym.ptr;
    a.off = ctx->off.ptr;
    a.p = ctx->p.ptr;
    a.slab = ctx->cfg[tier];
    a.lay = ctx->lay[tier];
    a.overflow = ctx->overflow.ptr;
    a.live_edges = ctx->live.ptr;
    return a;
}

// Counting pass over `list`; optional structural outputs.  Tier lists are
// (re)built from the overflow flags when build_tiers is set.
int counting_pass(wfsa_dev* ctx, bool want_outputs) {
    const int64_t S = ctx->n_strings;
    HIP_TRY(ctx->overflow.alloc(size_t(S)));
    HIP_TRY(hipMemsetAsync(ctx->overflow.ptr, 0, size_t(S), ctx->stream));
    if (want_outputs) {
        HIP_TRY(ctx->pcount.alloc(size_t(S)));
        HIP_TRY(ctx->recog.alloc(size_t(S)));
        HIP_TRY(ctx->used.alloc(size_t(ctx->n_params)));
        HIP_TRY(hipMemsetAsync(ctx->used.ptr, 0, size_t(std::max(ctx->n_params, 1)), ctx->stream));
    }
    HIP_TRY(hipMemsetAsync(ctx->live.ptr, 0, sizeof(unsigned long long), ctx->stream));
    // tier 0 over all strings
    wfsa::FBArgs a = base_args(ctx, 0);
    a.list = ctx->list_all.ptr;
    a.n_list = int32_t(S);
    if (want_outputs) {
        a.path_count = ctx->pcount.ptr;
        a.recognized = ctx->recog.ptr;
        a.used = ctx->used.ptr;
    }
    if (S > 0) HIP_TRY(wfsa::launch_fb(true, a, grid_for(ctx->cfg[0], ctx->n_cu, int32_t(S)), ctx->stream));
    std::vector<uint8_t> ovf(static_cast<size_t>(S));
    if (S > 0) HIP_TRY(hipMemcpyAsync(ovf.data(), ctx->overflow.ptr, size_t(S), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    std::vector<int32_t> l0, l1;
    l0.reserve(size_t(S));
    for (int64_t s = 0; s < S; ++s) (ovf[size_t(s)] ? l1 : l0).push_back(int32_t(s));
    if (!l1.empty()) {
        if (ctx->cfg[1].bytes == 0)
            return fail(WFSA_ERR_CAPACITY, "%zu strings exceed the per-wave trellis slab and the model is too "
                        "large for the single-wave tier", l1.size());
        HIP_TRY(ctx->list[1].upload(l1.data(), l1.size(), ctx->stream));
        wfsa::FBArgs b = base_args(ctx, 1);
        b.list = ctx->list[1].ptr;
        b.n_list = int32_t(l1.size());
        if (want_outputs) {
            b.path_count = ctx->pcount.ptr;
            b.recognized = ctx->recog.ptr;
            b.used = ctx->used.ptr;
        }
        HIP_TRY(hipMemsetAsync(ctx->overflow.ptr, 0, size_t(S), ctx->stream));
        HIP_TRY(wfsa::launch_fb(true, b, grid_for(ctx->cfg[1], ctx->n_cu, b.n_list), ctx->stream));
        HIP_TRY(hipMemcpyAsync(ovf.data(), ctx->overflow.ptr, size_t(S), hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(hipStreamSynchronize(ctx->stream));
        for (int32_t s : l1)
            if (ovf[size_t(s)])
                return fail(WFSA_ERR_CAPACITY, "string %d: trellis exceeds %d frontier nodes / %d live edges "
                            "(single-wave LDS tier)", s, ctx->cfg[1].cap_f, ctx->cfg[1].cap_e);
    }
    HIP_TRY(ctx->list[0].upload(l0.data(), l0.size(), ctx->stream));
    ctx->n_list[0] = int32_t(l0.size());
    ctx->n_list[1] = int32_t(l1.size());
    for (int t = 0; t < 2; ++t) ctx->grid[t] = ctx->n_list[t] ? grid_for(ctx->cfg[t], ctx->n_cu, ctx->n_list[t]) : 0;
    const size_t waves = size_t(ctx->grid[0]) * size_t(ctx->cfg[0].waves_per_block) +
                         size_t(ctx->grid[1]) * size_t(ctx->cfg[1].waves_per_block);
    HIP_TRY(ctx->ll_part.alloc(waves));
    ctx->stats.tier1_strings = ctx->n_list[1];
    ctx->stats.waves_per_block = ctx->cfg[0].waves_per_block;
    ctx->tiers_ready = true;
    return WFSA_OK;
}

int configure_tiers(wfsa_dev* ctx) {
    // tier 0: 4 waves per block, ~20 KB per wave (8 waves per CU); grows
    // to fit large automata.  tier 1: one wave per block, the whole LDS.
    ctx->cfg[0] = wfsa::SlabConfig{};
    ctx->cfg[1] = wfsa::SlabConfig{};
    bool ok0 = false;
    for (int budget : {20480, 40960}) {
        if (make_slab(budget, ctx->max_len, ctx->n_nodes, 4, ctx->cfg[0], ctx->lay[0])) { ok0 = true; break; }
    }
    const bool ok1 = make_slab(kLdsPerCu - 1024, ctx->max_len, ctx->n_nodes, 1, ctx->cfg[1], ctx->lay[1]);
    if (!ok1) ctx->cfg[1] = wfsa::SlabConfig{};
    if (!ok0) {
        if (!ok1)
            return fail(WFSA_ERR_CAPACITY, "automaton too large for the LDS trellis slab (%d nodes, max length %d)",
                        ctx->n_nodes, ctx->max_len);
        ctx->cfg[0] = ctx->cfg[1];
        ctx->lay[0] = ctx->lay[1];
    }
    ctx->tiers_ready = false;
    return WFSA_OK;
}

}  // namespace

extern "C" {

const char* wfsa_dev_last_error(void) { return g_last_error.c_str(); }

int wfsa_dev_create(int device, wfsa_dev** out) {
    if (!out) return fail(WFSA_ERR_ARG, "null output pointer");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail(WFSA_ERR_NODEV, "no HIP device available (%s)", e == hipSuccess ? "count 0" : hipGetErrorString(e));
    if (device < 0 || device >= n) return fail(WFSA_ERR_ARG, "device %d out of range (%d devices)", device, n);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(WFSA_ERR_NODEV, "device %d is %s; this build targets gfx950 (MI355X) only", device, prop.gcnArchName);
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(wfsa::configure_fb_kernels(kLdsPerCu));
    std::unique_ptr<wfsa_dev> ctx(new wfsa_dev());
    ctx->device = device;
    ctx->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : kNumCu;
    HIP_TRY(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&ctx->ev0));
    HIP_TRY(hipEventCreate(&ctx->ev1));
    HIP_TRY(ctx->live.alloc(1));
    *out = ctx.release();
    return WFSA_OK;
}

void wfsa_dev_destroy(wfsa_dev* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int wfsa_dev_load_model(wfsa_dev* ctx, const wfsa_model_desc* model) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!model) return fail(WFSA_ERR_ARG, "null model");
    wfsa::TrellisModel tm;
    const std::string err = wfsa::compile_trellis_model(*model, tm);
    if (!err.empty()) return fail(WFSA_ERR_MODEL, "automaton rejected: %s", err.c_str());
    hipStream_t s = ctx->stream;
    HIP_TRY(ctx->o_ptr.upload(tm.o_ptr.data(), tm.o_ptr.size(), s));
    HIP_TRY(ctx->o_byte.upload(tm.o_byte.data(), tm.o_byte.size(), s));
    HIP_TRY(ctx->o_dst.upload(tm.o_dst.data(), tm.o_dst.size(), s));
    HIP_TRY(ctx->o_pptr.upload(tm.o_pptr.data(), tm.o_pptr.size(), s));
    HIP_TRY(ctx->o_pidx.upload(tm.o_pidx.data(), tm.o_pidx.size(), s));
    HIP_TRY(ctx->x_ptr.upload(tm.x_ptr.data(), tm.x_ptr.size(), s));
    HIP_TRY(ctx->x_pptr.upload(tm.x_pptr.data(), tm.x_pptr.size(), s));
    HIP_TRY(ctx->x_pidx.upload(tm.x_pidx.data(), tm.x_pidx.size(), s));
    HIP_TRY(ctx->node_end_count.upload(tm.node_end_count.data(), tm.node_end_count.size(), s));
    ctx->n_edges = int64_t(tm.o_byte.size());
    ctx->n_end = int64_t(tm.x_pptr.size()) - 1;
    HIP_TRY(ctx->o_w.alloc(size_t(ctx->n_edges)));
    HIP_TRY(ctx->x_w.alloc(size_t(ctx->n_end)));
    HIP_TRY(ctx->node_end.alloc(size_t(tm.n_nodes)));
    ctx->n_params = tm.n_params;
    ctx->n_nodes = tm.n_nodes;
    ctx->start = tm.start;
    HIP_TRY(ctx->w_full.alloc(size_t(ctx->n_params)));
    HIP_TRY(ctx->out.alloc(size_t(ctx->n_params) + 1));
    HIP_TRY(ctx->used.alloc(size_t(ctx->n_params)));
    if (ctx->pinned_n < size_t(ctx->n_params) + 1) {
        if (ctx->pinned) (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->pinned), (size_t(ctx->n_params) + 1) * sizeof(double)));
        ctx->pinned_n = size_t(ctx->n_params) + 1;
    }
    HIP_TRY(hipStreamSynchronize(s));
    ctx->has_model = true;
    ctx->stats.n_nodes = ctx->n_nodes;
    ctx->stats.n_edges = ctx->n_edges;
    ctx->stats.n_end_edges = ctx->n_end;
    if (ctx->has_corpus) return configure_tiers(ctx);
    return WFSA_OK;
}

int wfsa_dev_load_corpus(wfsa_dev* ctx, const uint8_t* sym, const int64_t* off, const double* p, int64_t n_strings) {
    if (int rc = check_ctx(ctx)) return rc;
    if (n_strings < 0 || !off || (n_strings > 0 && !p)) return fail(WFSA_ERR_ARG, "bad corpus arguments");
    if (n_strings >= (int64_t(1) << 31) - 1) return fail(WFSA_ERR_ARG, "too many strings for one device (%lld)", (long long)n_strings);
    if (off[0] != 0) return fail(WFSA_ERR_ARG, "off[0] must be 0");
    int64_t max_len = 0;
    for (int64_t s = 0; s < n_strings; ++s) {
        const int64_t len = off[s + 1] - off[s];
        if (len < 0) return fail(WFSA_ERR_ARG, "string %lld has negative length", (long long)s);
        max_len = std::max(max_len, len);
    }
    if (max_len > 1000000) return fail(WFSA_ERR_CAPACITY, "string of length %lld too long", (long long)max_len);
    const int64_t total = off[n_strings];
    if (total > 0 && !sym) return fail(WFSA_ERR_ARG, "null symbol buffer");
    hipStream_t s = ctx->stream;
    HIP_TRY(ctx->sym.upload(sym, size_t(total), s));
    HIP_TRY(ctx->off.upload(off, size_t(n_strings) + 1, s));
    HIP_TRY(ctx->p.upload(p, size_t(n_strings), s));
    std::vector<int32_t> ids(static_cast<size_t>(n_strings));
    for (int64_t i = 0; i < n_strings; ++i) ids[size_t(i)] = int32_t(i);
    HIP_TRY(ctx->list_all.upload(ids.data(), ids.size(), s));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->n_strings = n_strings;
    ctx->total_sym = total;
    ctx->max_len = int32_t(max_len);
    ctx->has_corpus = true;
    ctx->stats.n_strings = n_strings;
    ctx->stats.total_symbols = total;
    ctx->stats.max_len = int32_t(max_len);
    if (ctx->has_model) return configure_tiers(ctx);
    return WFSA_OK;
}

int wfsa_dev_recognize(wfsa_dev* ctx, uint8_t* recognized, double* path_count, uint8_t* used_param) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->has_model || !ctx->has_corpus) return fail(WFSA_ERR_ARG, "load a model and a corpus first");
    if (int rc = counting_pass(ctx, true)) return rc;
    hipStream_t s = ctx->stream;
    const size_t S = size_t(ctx->n_strings);
    if (ctx->comm && ctx->n_params > 0)
        RCCL_TRY(ncclAllReduce(ctx->used.ptr, ctx->used.ptr, size_t(ctx->n_params), ncclUint8, ncclMax, ctx->comm, s));
    if (recognized && S) HIP_TRY(hipMemcpyAsync(recognized, ctx->recog.ptr, S, hipMemcpyDeviceToHost, s));
    if (path_count && S) HIP_TRY(hipMemcpyAsync(path_count, ctx->pcount.ptr, S * sizeof(double), hipMemcpyDeviceToHost, s));
    if (used_param && ctx->n_params)
        HIP_TRY(hipMemcpyAsync(used_param, ctx->used.ptr, size_t(ctx->n_params), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return WFSA_OK;
}

int wfsa_dev_objective_grad(wfsa_dev* ctx, const double* w_full, double* loglik, double* grad_full, double* logq) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->has_model || !ctx->has_corpus) return fail(WFSA_ERR_ARG, "load a model and a corpus first");
    if (!w_full && ctx->n_params > 0) return fail(WFSA_ERR_ARG, "null weights");
    if (!ctx->tiers_ready)
        if (int rc = counting_pass(ctx, false)) return rc;
    hipStream_t s = ctx->stream;
    const int32_t np = ctx->n_params;
    HIP_TRY(hipEventRecord(ctx->ev0, s));   // whole call, device side
    if (np > 0) {
        std::memcpy(ctx->pinned, w_full, size_t(np) * sizeof(double));
        HIP_TRY(hipMemcpyAsync(ctx->w_full.ptr, ctx->pinned, size_t(np) * sizeof(double), hipMemcpyHostToDevice, s));
    }
    HIP_TRY(wfsa::launch_edge_weights(ctx->w_full.ptr, ctx->o_pptr.ptr, ctx->o_pidx.ptr, ctx->o_w.ptr, ctx->n_edges, s));
    HIP_TRY(wfsa::launch_edge_weights(ctx->w_full.ptr, ctx->x_pptr.ptr, ctx->x_pidx.ptr, ctx->x_w.ptr, ctx->n_end, s));
    HIP_TRY(wfsa::launch_node_end(ctx->x_ptr.ptr, ctx->x_w.ptr, ctx->node_end.ptr, ctx->n_nodes, s));
    HIP_TRY(hipMemsetAsync(ctx->out.ptr, 0, (size_t(np) + 1) * sizeof(double), s));
    HIP_TRY(hipMemsetAsync(ctx->live.ptr, 0, sizeof(unsigned long long), s));
    if (logq) HIP_TRY(ctx->logq.alloc(size_t(ctx->n_strings)));
    hipEvent_t k0, k1;
    HIP_TRY(hipEventCreate(&k0));
    HIP_TRY(hipEventCreate(&k1));
    HIP_TRY(hipEventRecord(k0, s));
    int32_t wave_off = 0;
    for (int t = 0; t < 2; ++t) {
        if (!ctx->n_list[t]) continue;
        wfsa::FBArgs a = base_args(ctx, t);
        a.list = ctx->list[t].ptr;
        a.n_list = ctx->n_list[t];
        a.grad = ctx->out.ptr + 1;
        a.ll_part = ctx->ll_part.ptr + wave_off;
        a.logq = logq ? ctx->logq.ptr : nullptr;
        HIP_TRY(wfsa::launch_fb(false, a, ctx->grid[t], s));
        wave_off += ctx->grid[t] * ctx->cfg[t].waves_per_block;
    }
    HIP_TRY(hipEventRecord(k1, s));
    HIP_TRY(wfsa::launch_finalize(ctx->ll_part.ptr, wave_off, ctx->out.ptr, s));
    if (ctx->comm) RCCL_TRY(ncclAllReduce(ctx->out.ptr, ctx->out.ptr, size_t(np) + 1, ncclDouble, ncclSum, ctx->comm, s));
    HIP_TRY(hipMemcpyAsync(ctx->pinned, ctx->out.ptr, (size_t(np) + 1) * sizeof(double), hipMemcpyDeviceToHost, s));
    if (logq && ctx->n_strings)
        HIP_TRY(hipMemcpyAsync(logq, ctx->logq.ptr, size_t(ctx->n_strings) * sizeof(double), hipMemcpyDeviceToHost, s));
    unsigned long long live = 0;
    HIP_TRY(hipMemcpyAsync(&live, ctx->live.ptr, sizeof live, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(ctx->ev1, s));
    HIP_TRY(hipStreamSynchronize(s));
    float kms = 0.f, cms = 0.f;
    HIP_TRY(hipEventElapsedTime(&kms, k0, k1));
    HIP_TRY(hipEventElapsedTime(&cms, ctx->ev0, ctx->ev1));
    (void)hipEventDestroy(k0);
    (void)hipEventDestroy(k1);
    if (loglik) *loglik = ctx->pinned[0];
    if (grad_full && np > 0) std::memcpy(grad_full, ctx->pinned + 1, size_t(np) * sizeof(double));
    ctx->stats.fb_launches += 1;
    ctx->stats.fb_kernel_ms += double(kms);
    ctx->stats.last_fb_kernel_ms = double(kms);
    ctx->stats.last_call_ms = double(cms);
    ctx->stats.last_live_edges = int64_t(live);
    return WFSA_OK;
}

int wfsa_dev_comm_unique_id(uint8_t id[WFSA_COMM_ID_BYTES]) {
    if (!id) return fail(WFSA_ERR_ARG, "null id");
    static_assert(sizeof(ncclUniqueId) == WFSA_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId uid;
    RCCL_TRY(ncclGetUniqueId(&uid));
    std::memcpy(id, &uid, sizeof uid);
    return WFSA_OK;
}

int wfsa_dev_comm_init(wfsa_dev* ctx, int nranks, int rank, const uint8_t id[WFSA_COMM_ID_BYTES]) {
    if (int rc = check_ctx(ctx)) return rc;
    if (nranks < 1 || rank < 0 || rank >= nranks || !id) return fail(WFSA_ERR_ARG, "bad communicator arguments");
    if (ctx->comm) {
        (void)ncclCommDestroy(ctx->comm);
        ctx->comm = nullptr;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    RCCL_TRY(ncclCommInitRank(&ctx->comm, nranks, uid, rank));
    ctx->nranks = nranks;
    ctx->rank = rank;
    return WFSA_OK;
}

int wfsa_dev_allreduce(wfsa_dev* ctx, double* host_buf, int64_t count) {
    if (int rc = check_ctx(ctx)) return rc;
    if (count <= 0) return WFSA_OK;
    if (!host_buf) return fail(WFSA_ERR_ARG, "null buffer");
    if (!ctx->comm) return WFSA_OK;   // single rank: the sum is the input
    DevBuf<double> tmp;
    HIP_TRY(tmp.upload(host_buf, size_t(count), ctx->stream));
    RCCL_TRY(ncclAllReduce(tmp.ptr, tmp.ptr, size_t(count), ncclDouble, ncclSum, ctx->comm, ctx->stream));
    HIP_TRY(hipMemcpyAsync(host_buf, tmp.ptr, size_t(count) * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return WFSA_OK;
}

int wfsa_dev_get_stats(wfsa_dev* ctx, wfsa_dev_stats* out) {
    if (!ctx || !out) return fail(WFSA_ERR_ARG, "null argument");
    *out = ctx->stats;
    return WFSA_OK;
}

}  // extern "C"
