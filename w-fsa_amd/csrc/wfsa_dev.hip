// Implementation of the C-ABI device boundary declared in include/wfsa_dev.h.
//
// A context owns one HIP stream on one gfx950 device, the compiled trellis
// automaton, the packed corpus, the compiled per-string streams, scratch and
// (optionally) an RCCL communicator.  Per iteration the host sends w_full
// (n_params doubles) and receives [loglik, grad_full] (n_params+1 doubles);
// everything else stays in HBM.
//
// Preparing a corpus (once per wfsa_dev_load_corpus):
//   1. trav_kernel<MODE_COUNT> over every string (small-slab tier, then the
//      single-wave tier for strings that overflow): recognition, path counts,
//      used parameters, and the size of each string's compiled stream;
//   2. host: strings sorted by stream length into groups of 64 (one
//      wavefront each), interleaved stream offsets, bubble offsets;
//   3. trav_kernel<MODE_EMIT> writes the streams.
// Strings whose trellis does not compile (a bubble over the limits) stay on
// the traversal kernel in weighted mode.
#include "wfsa_dev.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdlib>
#include <queue>
#include <cstdio>
#include <cstring>
#include <memory>
#include <limits>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "collective.hpp"
#include "dense_path.hpp"
#include "matrix_path.hpp"
#include "sym_solver.hpp"
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

// an all-reduce over the context's communicator (collective.hpp)
#define COMM_TRY(ctx, buf, n, op, s)                                                                      \
    do {                                                                                               \
        if ((ctx)->comm->allreduce((buf), (n), (op), (s)))                                             \
            return fail(WFSA_ERR_RCCL, "%s all-reduce: %s", (ctx)->comm->kind(), (ctx)->comm->last_error()); \
    } while (0)

// after a host sync: a peer all-reduce of this call that gave up (NaN
// results) is reported as the error it is
#define COMM_CHECK(ctx)                                                                               \
    do {                                                                                               \
        if ((ctx)->comm && (ctx)->comm->check())                                                       \
            return fail(WFSA_ERR_RCCL, "%s all-reduce: %s", (ctx)->comm->kind(), (ctx)->comm->last_error()); \
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
        const size_t c = std::max<size_t>(count, 1);
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&ptr), c * sizeof(T));
        if (e == hipSuccess) n = c;
        return e;
    }
    hipError_t upload(const T* src, size_t count, hipStream_t s) {
        hipError_t e = alloc(count);
        if (e != hipSuccess || count == 0) return e;
        return hipMemcpyAsync(ptr, src, count * sizeof(T), hipMemcpyHostToDevice, s);
    }
    hipError_t download(T* dst, size_t count, hipStream_t s) const {
        if (count == 0) return hipSuccess;
        return hipMemcpyAsync(dst, ptr, count * sizeof(T), hipMemcpyDeviceToHost, s);
    }
};

constexpr int kLdsPerCu = 163840;
constexpr int kNumCu = 256;
constexpr int kWave = 64;
constexpr int kGradBlock = 64;   // the preparation-time gradient pass: one wavefront per block
constexpr int kIterWavesPerCu = 16;   // per-iteration stream kernel
constexpr int kQnDepth = 8;   // device-resident QN steps in flight

// weights after the results in the host-mapped buffer, 16-byte aligned
inline size_t weights_off(int32_t np) { return (size_t(np) + 3) & ~size_t(1); }

}  // namespace

struct wfsa_dev {
    int device = 0;
    int n_cu = kNumCu;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // per in-flight step: before the stream kernel, after it, after the tail
    hipEvent_t k0[kQnDepth] = {}, kc[kQnDepth] = {}, k2[kQnDepth] = {};
    // nothing was enqueued between kc and the tail's end: k2 is kc (each
    // timing marker costs the step ~1 us, profiles/r02/v23_timing_ab.txt)
    bool k2_kc[kQnDepth] = {};
    // host-mapped QN state (x | lambda | grad) for set_state / get_state:
    // kernels move it, where pageable copies cost ~25 us each
    double* qst = nullptr;
    double* qst_dev = nullptr;
    size_t qst_n = 0;
    // QN runs time the kernels of every 16th step (WFSA_TIMING_STRIDE), steps
    // stride-1, 2*stride-1, ...: not the first, whose launch latency the
    // event markers would lengthen
    int timing_stride = 16;

    // model
    bool has_model = false;
    int32_t n_params = 0, n_nodes = 0, start = 0;
    int64_t n_edges = 0, n_end = 0;
    DevBuf<int32_t> o_ptr, o_dst, x_ptr, pptr, pidx;
    DevBuf<uint8_t> o_byte;
    DevBuf<double> lw, ew, node_end, node_end_count;
    DevBuf<int32_t> multi_of, multi_edge;   // multi-parameter combined edges
    int32_t n_multi = 0;
    DevBuf<wfsa::EdgeRec> erec;

    // corpus
    bool has_corpus = false;
    int64_t n_strings = 0, total_sym = 0;
    int32_t max_len = 0;
    DevBuf<uint8_t> sym;
    DevBuf<int64_t> off;
    DevBuf<double> p;
    DevBuf<int32_t> list_all;

    // traversal tiers: small LDS slab (several waves per block) / whole LDS
    wfsa::SlabConfig cfg[2];
    wfsa::SlabLayout lay[2];
    DevBuf<uint8_t> overflow;

    // preparation state (valid until the next load): 0 none, 1 counted,
    // 2 counted + streams compiled
    int prep_level = 0;
    DevBuf<double> pcount;
    DevBuf<uint8_t> recog, used;

    // compiled streams
    int32_t n_groups = 0;
    int64_t n_compiled = 0;
    DevBuf<uint4> stream_w;   // 16-byte chunks
    int wide = 0;             // 32-bit stream words
    DevBuf<int32_t> bub, g_len, l_str, l_len;
    DevBuf<int32_t> wave_first;   // [stream waves + 1] the per-iteration kernel's groups of each wave
    DevBuf<int64_t> g_base;
    // the per-iteration stream kernel's copy of the streams in the delta
    // format (fb_kernels.hpp): its own groups, dealing and layout; the 16-bit
    // streams above stay for the preparation-time gradient pass
    bool delta_on = false;
    double qw_mean_rows = 0.0;       // the delta deal's mean stream rows per wave (the in-kernel QN's cover rule)
    bool qw_cover = true;            // the stream covers the bubble tail: the one-launch step is the faster one
    bool qw_force = false;           // WFSA_QN_INKERNEL=1: the one-launch step whenever it is possible
    int32_t d_tab = 0;
    DevBuf<uint4> dstream;
    DevBuf<int64_t> d_g_base;
    DevBuf<int32_t> d_g_len, d_l_str, d_wave_first;
    int64_t d_stream_bytes = 0;
    int c_grid = 0, c_tables = 0;    // gradient pass (once, at preparation)
    int i_grid = 0, i_tables = 0;    // per-iteration pass (log-weights only)
    int i_block = 1024;
    size_t i_lds = 0;
    DevBuf<double> fixed_grad;       // [n_params] gradient of the trivial words (constant)
    DevBuf<double> fixed_t;          // [qn_n] the same in trimmed order (QN runs)
    bool fixed_t_on = false;
    int64_t fixed_t_key = -1;        // (prep_gen, qn setup) the gather above was made for
    int64_t qn_setup_gen = 0;
    bool qn_flags_clear = false;     // halted / halt_pending are 0 (the last run did not halt)
    bool eval_no_slice = false;      // this evaluation's stream kernel skips edge_weight_slice
    int32_t lead_grp_nch = 1;        // chunks of the largest constraint-led slot group
    int32_t qn_max_nm = 1;           // members of the largest constraint
    // bubbles
    int32_t n_bubbles = 0, n_small4 = 0, n_small = 0, n_big = 0, big_lds_edges = 2;
    int b_waves = 0;
    DevBuf<int4> sm4_tbl, sm_tbl;
    DevBuf<int32_t> big_off, big_edge_base, big_eslot_ptr, big_eslot;
    DevBuf<int32_t> bub_off;
    DevBuf<double> contrib;
    // contribution slots: parameter-major in a slot order (position pos_of[j]
    // of full parameter j; identity, or the trimmed order once the QN loop is
    // set up, so a constraint's members own one contiguous run); seg_ptr by
    // position, param_at its inverse, and the reduction's tiles
    std::vector<int32_t> h_bubbuf, h_sm4_list, h_sm_list, h_big_list;   // host copies (re-layout)
    std::vector<int32_t> slot_order;        // [n_params] pos_of used by the current layout
    std::vector<int32_t> h_seg_ptr;
    DevBuf<int32_t> seg_ptr, param_at, tile_ptr;   // tile_ptr: [n_tiles + 1] position range of each reduction group
    int32_t n_tiles = 0;
    DevBuf<int64_t> grp_base;            // [n_tiles + 1] physical slot base of each reduction group
    DevBuf<int32_t> grp_nch;             // [n_tiles] its chunk count
    DevBuf<int32_t> chunk_ptr;           // [n_params + 1] slot chunks by position (cumulative)
    std::vector<int32_t> slot_groups;     // leading reduction groups (positions): the QN constraints
    std::vector<int32_t> h_pptr, h_pidx;   // host copy of the combined parameter lists

    size_t c_lds = 0;

    // traversal fallback: per tier string lists (tier 2: wide_kernel)
    int32_t n_fall[3] = {0, 0, 0};
    std::vector<int8_t> h_tier;   // per string: -1 compiled, 0..2 traversal tier
    int fall_grid[3] = {0, 0, 0};
    DevBuf<int32_t> fall[3];
    // tier 2: byte-indexed in-edge lists and per-block scratch
    DevBuf<int32_t> w_cptr, w_dst, w_eptr, w_esrc, w_eg;
    DevBuf<double> w_scratch;
    int64_t w_stride = 0;
    int32_t tier2_strings = 0;
    bool force_tier2 = false;   // WFSA_TIER2=1: every string on tier 2 (tests)
    // tier 2 weighted pass, wave per string (wide2_kernel; WFSA_WIDE2=0: the
    // block-per-string wide_kernel): (node, byte) out-edge table, per-wave
    // scratch (alpha rows zero between strings), work counters
    bool use_wide2 = true;
    bool has_pairs = false;   // the byte-pair tables were built (size cap)
    int32_t pt_K = 0, pt_max_n = 0;
    int64_t pt_ne = 0;
    DevBuf<int32_t> pt_bidx, pt_n, pt_dlptr, pt_dlnode, pt_eptr;
    DevBuf<int4> pt_ent;
    DevBuf<int32_t> pt_sd;
    DevBuf<double> pt_w;   // [2 ne]: ew, lw per entry
    // the same pairs laid out for wave_pull_kernel (PullTables; WFSA_PULL=0: wide2_kernel)
    bool use_pull = true;
    bool has_pull = false;
    bool w2_pull = false;           // this preparation runs wave_pull_kernel
    int64_t pl_nf = 0, pl_nb = 0;   // forward / backward entries
    DevBuf<int4> pl_info, pl_fhdr, pl_bent;
    int32_t pl_items = 8;
    DevBuf<int32_t> pl_fcode, pl_g;   // pl_g: edge id per forward then per backward entry
    DevBuf<double> pl_w;              // [nf + nb + nf]: forward ew, backward ew, forward lw
    int w2_waves = 16;           // waves per block
    bool w2_lgrad = false;       // the gradient in LDS
    DevBuf<double> w2_scratch;
    int64_t w2_stride = 0;
    int w2_grid = 0;
    DevBuf<unsigned> w2_ctr;
    DevBuf<unsigned long long> w2_fix;   // the wave kernel's fixed-point sums (WideArgs::fix)
    int32_t w2_fix_frac = 52;
    bool w2_all = true;          // every traversal string on the wave kernel
    DevBuf<int32_t> w2_list;     // its strings, longest first
    int32_t w2_n = 0;

    // work buffers
    DevBuf<double> w_full, ewp, out, ll_part, logq;
    double* ll_cur = nullptr;      // this launch sequence's half of ll_part (QN steps alternate)
    size_t ll_stride = 0;
    DevBuf<unsigned long long> live;
    double* pinned = nullptr;   // [0, n_params+1): results; from weights_off(n_params): weights
    double* pinned_dev = nullptr;   // the same memory as the device addresses it
    size_t pinned_n = 0;
    // completion flag (host-mapped) and the device sequence counter
    unsigned* flag = nullptr;
    unsigned* flag_dev = nullptr;
    DevBuf<unsigned> counters;   // [0] sequence
    unsigned seq = 0;            // last sequence number the host expects
    bool timing_pending = false; // events of the last call not yet read
    bool kernel_timing = true;
    bool use_delta = true;       // WFSA_DELTA=0: the per-iteration pass reads the 16-bit streams

    DevBuf<double> gpart;        // per-block partial gradients of the compiled kernel

    // rmin info column: per-bubble / per-string logs, block partials, results
    // (two halves: a QN step's finish reads its own while the next step writes)
    DevBuf<double> rm_rs, rm_vb, rm_part, rm_res, rm_key;
    DevBuf<double> rm_sv;           // [n_bubbles] per-bubble rmin values at list positions (fused kernel)
    DevBuf<int32_t> rm_bpos;        // [n_bubbles] list position of each bubble
    bool rm_sv_used = false;        // the last evaluation stored per-bubble values into rm_sv
    double rm_base = 0.0;        // across ranks: global index of this rank's first loaded string
    DevBuf<int4> rm_amb;         // the ambiguous strings (path count > 1) with their bubble runs
    std::vector<int32_t> h_bfirst, h_nbub;   // per string: first bubble ordinal, bubbles (compiled strings)
    int max_bub_nodes = 1;                   // largest compiled bubble (nodes)
    int64_t rm_n_amb = 0;
    // the rmin column folded into the in-kernel QN step (fb_kernels.hpp RminFold)
    std::vector<int32_t> h_bpos;    // list position of each bubble (layout)
    DevBuf<int2> rm_bk;             // [positions] (bubbles of its ambiguous string, its run in rm_mpos)
    DevBuf<int32_t> rm_mpos;        // the positions of each multi-bubble string's bubbles, in bubble order
    DevBuf<unsigned> rm_cnt;        // [rm_mpos entries] arrivals per multi-bubble string, zero between launches
    DevBuf<int32_t> rm_trav;        // the ambiguous traversal strings
    int32_t rm_n_trav = 0;
    DevBuf<double> rm_bpart;        // [2][stream-kernel blocks][2] block minima, by step parity
    double* rm_bpart_cur = nullptr; // this step's half (set by enqueue_qn_step for enqueue_compiled)
    int rm_gen = -1;             // prep_gen the list was built for
    bool qn_rmin = false;        // the device QN loop fills the rmin columns
    bool rm_eval = false;        // the evaluation being enqueued also runs the traversal min forward
    std::unique_ptr<wfsa::MatrixPath> mpath;   // matrix-file mode (wfsa_dev_load_paths)
    std::unique_ptr<wfsa::SymSolver> ldlt;     // dense LDL^T of the HessianLearner's KKT system
    std::unique_ptr<wfsa::TrellisModel> h_tm;  // host copy of the trellis model (H_f set-up)

    // the per-iteration device sequence, captured once per prepared corpus
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    bool graph_failed = false;
    bool use_graph = false;    // WFSA_GRAPH=1: replay a captured graph (no per-kernel timing)
    bool in_flight = false;    // between objective_grad_begin and _end
    bool weights_staged = false;   // wfsa_dev_weights_staging handed out the staging area since the last _begin
    bool logq_ready = false;   // the call in flight computes log q

    // device-resident QuasiNewton (wfsa_dev_qn_*)
    bool qn_ready = false;
    int32_t qn_n = 0, qn_k = 0, qn_exp_lambda = 0;
    double qn_plogp = 0.0;
    DevBuf<int32_t> qn_trim, qn_full_of, qn_ccol, qn_cptr;
    int prep_gen = 0;
    DevBuf<double> qn_x, qn_lambda, qn_expx, qn_grad, qn_partial;
    // the QN finish of the last enqueued step, not yet enqueued (fin_pending),
    // and the one handed to the next stream kernel launch (fin_for_fbs)
    wfsa::QnFinish fin_next{}, fin_for_fbs{};
    DevBuf<double> ll_stash;   // [2] the all-reduced log-likelihood of a multi-rank step, by parity
    std::vector<int32_t> h_cptr;
    bool fin_pending = false, fin_hostable = false;
    bool fin_next_px = false, fin_for_fbs_px = false;   // (their finishes exchange across ranks, PeerX)
    wfsa::PeerX cur_px{};                                // this launch's exchange (enqueue_qn_step)
    DevBuf<unsigned> qn_halted;
    std::vector<int32_t> qn_full_of_h, qn_cptr_h;
    bool qn_fused = false;           // qn_step_kernel sums the members' bubble slots itself
    int64_t pipe_init_key = -1;               // the second weight buffer's constants copied for this key
    const double* pipe_init_w = nullptr;
    const double* pipe_init_e = nullptr;
    DevBuf<double> w_full2, ewp2;
    double* w_cur = nullptr;         // the weights the evaluation kernels read (null: w_full / ewp)
    double* ewp_cur = nullptr;
    double* qn_ring = nullptr;       // host-mapped [kQnDepth][kQnRow]
    double* qn_ring_dev = nullptr;
    // the QN update inside the stream kernel (fb_kernels.hpp QnWave; one
    // rank, every string compiled, delta stream, no rmin column;
    // WFSA_QN_INKERNEL=0: the separate qn_step_kernel): QN waves reserved by
    // the dealer (qw_waves, wave wpb - 2 of blocks [0, qw_waves)), batches of
    // constraints built at QN set-up, per-parity arrival counters and the
    // weights double-buffered by step parity (w_full2 / ewp2 above)
    bool use_qw = true;
    int32_t qw_waves = 0;            // reserved at preparation
    double qw_cost = 6.0;            // the dealer's charge per QN wave, in stream rows
    bool qw_ok = false;              // batches built for the current preparation and QN set-up
    int32_t qw_nbatch = 0;
    DevBuf<int4> qw_batch;
    DevBuf<int32_t> qw_con_of, qw_mnch, qw_mfirst;
    DevBuf<double> qw_gch;           // (build_qw_batches across ranks: the constraints' chunk counts)
    int64_t qw_agree_key = -1;       // across ranks: the in-kernel decision agreed for this key ...
    bool qw_agreed = false;          // ... and its outcome
    std::vector<int64_t> h_mchunk;   // [n_params] first contribution slot of each position's chunks (layout_slots)
    std::vector<int32_t> h_mnch;     // [n_params] its chunk count
    int64_t layout_gen = 0;          // layout_slots runs
    int64_t qw_key = -1;             // (qn set-up, layout) the batches were built for
    std::vector<int4> h_qw_batch;    // host copy of the batches (diagnostics)
    DevBuf<unsigned> qw_arrive;      // [2], zero between launches (each launch zeroes the next one's)
    DevBuf<unsigned> qw_done;        // [2] the self-finish's arrivals, likewise
    DevBuf<unsigned> qw_go;          // [kQnMaxWaves][kQnGoStride] the QN waves' go lines (fb_kernels.hpp QnWave::go)
    size_t qw_res_lds = ~size_t(0);  // qw_resident's cache: the launch's LDS and block, blocks per CU
    int qw_res_block = 0, qw_res_per_cu = 0;
    uint32_t qw_poll_limit = 0;      // polls before an in-kernel QN wave gives up (0: the kernel default)
    bool qw_poll_fault = false;      // WFSA_FAULT_QN_POLL=1 (tests): the first QN wave never sees its arrivals
    bool qw_last_self = true;        // a Run's last launch finishes its own step (WFSA_QN_LAST_SELF=0: off)
    uint64_t qw_seq = 0;             // in-kernel QN launches enqueued (their parity)
    wfsa::QnWave qw_next{};          // picked up by the next stream kernel launch (qw_next.on)
    DevBuf<unsigned long long> fbs_trace;   // timing experiments (WFSA_FBS_TRACE): per-wave stamps of the last launch

    // dense automata: the fp64 MFMA path (dense_path.hpp) replaces the
    // trellis kernels; WFSA_DENSE=0 never, =1 whenever the model qualifies
    // (any size), unset: when the transition matrix is at least 1/4 full
    std::unique_ptr<wfsa::DensePath> dense;
    int dense_mode = -1;
    bool dense_struct = false;   // the structural pass ran on the loaded corpus

    // Hessian second-order term (wfsa_dev_hf_*): slots per bubble and the
    // (j, k) pattern they sum into
    bool hf_ready = false;
    int hf_gen = -1;
    std::vector<int32_t> hf_pairs;
    DevBuf<int64_t> hf_slot_base, hf_t_ptr, hf_t_slot;
    DevBuf<double> hf_slot_val, hf_out;
    int64_t hf_n_slots = 0;
    // traversal strings: (string, V offset, |V|), their equivocal parameters, first slots, scratch
    DevBuf<int4> hft_list;
    DevBuf<int32_t> hft_v;
    DevBuf<int64_t> hft_base;
    DevBuf<double> hft_scratch;
    int32_t hft_n = 0;
    int hft_grid = 0;
    int64_t hft_stride = 0;
    int32_t hft_vm = 0;

    // communicator
    std::unique_ptr<wfsa::Collective> comm;
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
    const int32_t cap_f = int32_t(rem / 38) & ~1;
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

int trav_grid(const wfsa::SlabConfig& c, int n_cu, int64_t n_list) {
    const int block_lds = c.bytes * c.waves_per_block;
    int per_cu = std::max(1, std::min(kLdsPerCu / std::max(block_lds, 1), 32 / c.waves_per_block));
    per_cu = std::min(per_cu, 8);
    const int64_t want = (n_list + c.waves_per_block - 1) / c.waves_per_block;
    return int(std::max<int64_t>(1, std::min<int64_t>(want, int64_t(n_cu) * per_cu)));
}

wfsa::ModelView model_view(wfsa_dev* ctx) {
    wfsa::ModelView m{};
    m.o_ptr = ctx->o_ptr.ptr;
    m.o_byte = ctx->o_byte.ptr;
    m.o_dst = ctx->o_dst.ptr;
    m.x_ptr = ctx->x_ptr.ptr;
    m.pptr = ctx->pptr.ptr;
    m.pidx = ctx->pidx.ptr;
    m.ew = ctx->ew.ptr;
    m.lw = ctx->lw.ptr;
    m.erec = ctx->erec.ptr;
    m.node_end = ctx->node_end.ptr;
    m.node_end_count = ctx->node_end_count.ptr;
    m.multi_of = ctx->multi_of.ptr;
    m.multi_edge = ctx->multi_edge.ptr;
    m.n_nodes = ctx->n_nodes;
    m.start = ctx->start;
    m.n_edges = int32_t(ctx->n_edges);
    m.n_params = ctx->n_params;
    return m;
}

wfsa::TravArgs trav_args(wfsa_dev* ctx, int tier) {
    wfsa::TravArgs a{};
    a.m = model_view(ctx);
    a.sym = ctx->sym.ptr;
    a.off = ctx->off.ptr;
    a.p = ctx->p.ptr;
    a.slab = ctx->cfg[tier];
    a.lay = ctx->lay[tier];
    a.overflow = ctx->overflow.ptr;
    a.live_edges = ctx->live.ptr;
    return a;
}

// tier 2: blocks in flight, bounded by a scratch budget of 4 GiB
int wide_grid(wfsa_dev* ctx, int64_t n_list) {
    ctx->w_stride = wfsa::wide_scratch_stride(ctx->max_len, ctx->n_nodes);
    const int64_t budget = (int64_t(4) << 30) / 8;
    int64_t g = std::max<int64_t>(1, std::min<int64_t>(4 * int64_t(ctx->n_cu), budget / std::max<int64_t>(ctx->w_stride, 1)));
    return int(std::max<int64_t>(1, std::min<int64_t>(g, n_list)));
}

wfsa::WideArgs wide_args(wfsa_dev* ctx) {
    wfsa::WideArgs a{};
    a.m = model_view(ctx);
    a.w.c_ptr = ctx->w_cptr.ptr;
    a.w.dst = ctx->w_dst.ptr;
    a.w.e_ptr = ctx->w_eptr.ptr;
    a.w.e_src = ctx->w_esrc.ptr;
    a.w.e_g = ctx->w_eg.ptr;
    a.sym = ctx->sym.ptr;
    a.off = ctx->off.ptr;
    a.p = ctx->p.ptr;
    a.max_len = ctx->max_len;
    a.scratch = ctx->w_scratch.ptr;
    a.scratch_stride = ctx->w_stride;
    a.grad_lds = size_t(ctx->n_params) * sizeof(double) <= size_t(96 * 1024) ? 1 : 0;
    a.pt.K = ctx->pt_K;
    a.pt.bidx = ctx->pt_bidx.ptr;
    a.pt.n = ctx->pt_n.ptr;
    a.pt.dl_ptr = ctx->pt_dlptr.ptr;
    a.pt.dl_node = ctx->pt_dlnode.ptr;
    a.pt.e_ptr = ctx->pt_eptr.ptr;
    a.pt.ent = ctx->pt_ent.ptr;
    a.pt.sd = ctx->pt_sd.ptr;
    a.pt.w = ctx->pt_w.ptr;
    a.pt.lw = ctx->pt_w.ptr + ctx->pt_ne;
    a.pt.max_n = ctx->pt_max_n;
    if (ctx->has_pull) {
        a.pl.items = ctx->pl_items;
        a.pl.info = ctx->pl_info.ptr;
        a.pl.fhdr = ctx->pl_fhdr.ptr;
        a.pl.fcode = ctx->pl_fcode.ptr;
        a.pl.bent = ctx->pl_bent.ptr;
        a.pl.fw = ctx->pl_w.ptr;
        a.pl.bw = ctx->pl_w.ptr + ctx->pl_nf;
        a.pl.flw = ctx->pl_w.ptr + ctx->pl_nf + ctx->pl_nb;
    }
    a.scratch2 = ctx->w2_scratch.ptr;
    a.stride2 = ctx->w2_stride;
    a.hrows2 = wfsa::wide2_rows(ctx->max_len, ctx->pt_max_n, ctx->pl_items);
    a.ctr = ctx->w2_ctr.ptr;
    a.fix = ctx->w2_fix.ptr;
    a.fix_frac = ctx->w2_fix_frac;
    return a;
}

// Waves per block and the gradient table of the tier-2 wave kernel: the
// gradient table in LDS when at least 4 waves fit beside it (global fp64
// atomics cost ~7x at family B), else the most waves with global atomics.
bool wide2_config(wfsa_dev* ctx) {
    const size_t cap = size_t(kLdsPerCu) - 1024;
    const bool pull = ctx->has_pull && ctx->use_pull;
    auto lds = [&](bool lg, int w) {
        return pull ? wfsa::pull_lds(ctx->n_params, lg, w, ctx->pt_max_n) : wfsa::wide2_lds(ctx->n_params, lg, w, ctx->pt_max_n);
    };
    int best = 0;
    bool lg = false;
    const int wmax = pull ? wfsa::kPullBlock / kWave : 16;
    for (int w : {16, 12, 8, 4})
        if (!best && w <= wmax && lds(true, w) <= cap) {
            best = w;
            lg = true;
        }
    for (int w : {16, 12, 8, 4})
        if (!best && w <= wmax && lds(false, w) <= cap) best = w;
    if (!best) return false;
    ctx->w2_waves = best;
    ctx->w2_lgrad = lg;
    ctx->w2_pull = pull;
    return true;
}

// The pull layout of the pair tables (fb_kernels.hpp PullTables) from the
// pairs' edge lists: per pair, the forward's items are the destinations of
// D(b) with their in-edges, the backward's the sources of D(a) with their
// out-edges (both in the lists' order); items dealt to the 64 lanes largest
// first, each to the least loaded lane holding fewer than `items` (4, 6 or
// 8: the fewest that hold the largest D).  Skipped (has_pull = false) when a
// D(b) exceeds 64 x 8 nodes.
int build_pull_tables(wfsa_dev* ctx, int K, const std::vector<int32_t>& n, const std::vector<int32_t>& e_ptr,
                      const std::vector<int4>& ent) {
    ctx->has_pull = false;
    int32_t max_n = 0;
    for (int32_t v : n) max_n = std::max(max_n, v);
    if (max_n > kWave * wfsa::kPullItemsMax || max_n >= 32768) return WFSA_OK;
#ifdef WFSA_PULL_NI   // (layout-variant builds: make var)
    const int NI = std::max(WFSA_PULL_NI, max_n <= 4 * kWave ? 4 : (max_n <= 6 * kWave ? 6 : 8));
#else
    const int NI = max_n <= 4 * kWave ? 4 : (max_n <= 6 * kWave ? 6 : 8);
#endif
    const int64_t n_pairs = int64_t(K + 1) * K;
    std::vector<int4> info(static_cast<size_t>(n_pairs)), fhdr(static_cast<size_t>(n_pairs * kWave));
    std::vector<int32_t> fcode, fg, bg;
    std::vector<int4> bent;
    std::vector<std::vector<int32_t>> items;   // per node: its entries (indices into ent)
    std::vector<int32_t> order;
    std::vector<int64_t> load(kWave);
    std::vector<int32_t> cnt(kWave);
    std::vector<std::vector<int32_t>> lane_items(kWave);
    // deal items [0, n_items) to the lanes; returns T (entries of the most loaded lane)
    auto deal = [&](int n_items) -> int64_t {
        order.resize(size_t(n_items));
        for (int i = 0; i < n_items; ++i) order[size_t(i)] = i;
        std::stable_sort(order.begin(), order.end(),
                         [&](int32_t x, int32_t y) { return items[size_t(x)].size() > items[size_t(y)].size(); });
        std::fill(load.begin(), load.end(), 0);
        std::fill(cnt.begin(), cnt.end(), 0);
        for (auto& v : lane_items) v.clear();
        for (int32_t it : order) {
            int best = -1;
            for (int l = 0; l < kWave; ++l)
                if (cnt[size_t(l)] < NI && (best < 0 || load[size_t(l)] < load[size_t(best)])) best = l;
            lane_items[size_t(best)].push_back(it);
            load[size_t(best)] += std::max<int64_t>(1, int64_t(items[size_t(it)].size()));
            ++cnt[size_t(best)];
        }
        int64_t T = 0;
        for (int64_t v : load) T = std::max(T, v);
        return T;
    };
    for (int a = 0; a <= K; ++a) {
        for (int b = 0; b < K; ++b) {
            const int64_t q = int64_t(a) * K + b;
            const int na = n[size_t(a)], nb = n[size_t(b)];
            const int32_t e0 = e_ptr[size_t(q)], e1 = e_ptr[size_t(q) + 1];
            // forward: destinations
            items.assign(size_t(nb), {});
            for (int32_t e = e0; e < e1; ++e) items[size_t(uint32_t(ent[size_t(e)].x) >> 16)].push_back(e);
            int64_t T = deal(nb);
            for (int l = 0; l < kWave; ++l) {   // the lane's destinations
                uint32_t sw[4] = {~0u, ~0u, ~0u, ~0u};
                for (size_t k = 0; k < lane_items[size_t(l)].size(); ++k) {
                    const uint32_t d = uint32_t(lane_items[size_t(l)][k]);
                    sw[k >> 1] = (sw[k >> 1] & ~(0xffffu << (16 * (k & 1)))) | (d << (16 * (k & 1)));
                }
                fhdr[size_t(q * kWave + l)] = make_int4(int32_t(sw[0]), int32_t(sw[1]), int32_t(sw[2]), int32_t(sw[3]));
            }
            const int64_t fbase = int64_t(fcode.size());
            fcode.resize(size_t(fbase + T * kWave), 0);
            fg.resize(size_t(fbase + T * kWave), -1);
            for (int l = 0; l < kWave; ++l) {
                int64_t t = 0;
                for (int32_t d : lane_items[size_t(l)]) {
                    const auto& it = items[size_t(d)];
                    const size_t at0 = size_t(fbase + t * kWave + l);
                    if (it.empty()) {
                        fcode[at0] = int32_t((uint32_t(d) << 16) | 0x80000000u);
                        ++t;
                        continue;
                    }
                    for (size_t k = 0; k < it.size(); ++k, ++t) {
                        const int4& en = ent[size_t(it[k])];
                        const size_t at = size_t(fbase + t * kWave + l);
                        fcode[at] = int32_t((uint32_t(en.x) & 0xffffu) | (uint32_t(d) << 16) |
                                            (k + 1 == it.size() ? 0x80000000u : 0u));
                        fg[at] = en.y;
                    }
                }
            }
            const int64_t fT = T;
            // backward: sources
            items.assign(size_t(na), {});
            for (int32_t e = e0; e < e1; ++e) items[size_t(uint32_t(ent[size_t(e)].x) & 0xffffu)].push_back(e);
            T = deal(na);
            const int64_t bbase = int64_t(bent.size());
            bent.resize(size_t(bbase + (T + 1) * kWave), make_int4(0, -1, -1, -1));
            bg.resize(bent.size(), -1);
            for (int l = 0; l < kWave; ++l) {   // row 0: the lane's sources
                uint32_t sw[4] = {~0u, ~0u, ~0u, ~0u};
                for (size_t k = 0; k < lane_items[size_t(l)].size(); ++k) {
                    const uint32_t u = uint32_t(lane_items[size_t(l)][k]);
                    sw[k >> 1] = (sw[k >> 1] & ~(0xffffu << (16 * (k & 1)))) | (u << (16 * (k & 1)));
                }
                bent[size_t(bbase + l)] = make_int4(int32_t(sw[0]), int32_t(sw[1]), int32_t(sw[2]), int32_t(sw[3]));
            }
            for (int l = 0; l < kWave; ++l) {
                int64_t t = 1;
                for (int32_t u : lane_items[size_t(l)]) {
                    const auto& it = items[size_t(u)];
                    if (it.empty()) {
                        bent[size_t(bbase + t * kWave + l)] = make_int4(int32_t((uint32_t(u) << 16) | 0x80000000u), -1, -1, -1);
                        ++t;
                        continue;
                    }
                    for (size_t k = 0; k < it.size(); ++k, ++t) {
                        const int4& en = ent[size_t(it[k])];
                        bent[size_t(bbase + t * kWave + l)] =
                            make_int4(int32_t((uint32_t(en.x) >> 16) | (uint32_t(u) << 16) |
                                              (k + 1 == it.size() ? 0x80000000u : 0u)),
                                      en.y, en.z, en.w);
                        bg[size_t(bbase + t * kWave + l)] = en.y;
                    }
                }
            }
            if (fbase + fT * kWave >= (int64_t(1) << 31) || bbase + (T + 1) * kWave >= (int64_t(1) << 31)) return WFSA_OK;
            info[size_t(q)] = make_int4(int32_t(fbase), int32_t(fT), int32_t(bbase), int32_t(T));
        }
    }
    if (fcode.empty()) {
        fcode.push_back(0);
        fg.push_back(-1);
    }
    if (bent.empty()) {
        bent.push_back(make_int4(0, -1, -1, -1));
        bg.push_back(-1);
    }
    hipStream_t s = ctx->stream;
    HIP_TRY(ctx->pl_info.upload(info.data(), info.size(), s));
    HIP_TRY(ctx->pl_fhdr.upload(fhdr.data(), fhdr.size(), s));
    ctx->pl_items = NI;
    HIP_TRY(ctx->pl_fcode.upload(fcode.data(), fcode.size(), s));
    HIP_TRY(ctx->pl_bent.upload(bent.data(), bent.size(), s));
    fg.insert(fg.end(), bg.begin(), bg.end());
    HIP_TRY(ctx->pl_g.upload(fg.data(), fg.size(), s));
    ctx->pl_nf = int64_t(fcode.size());
    ctx->pl_nb = int64_t(bent.size());
    HIP_TRY(ctx->pl_w.alloc(size_t(2 * ctx->pl_nf + ctx->pl_nb)));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->has_pull = true;
    return WFSA_OK;
}

// The byte-pair tables of the tier-2 wave kernel (fb_kernels.hpp
// PairTables), from the byte-indexed in-edge lists (cptr/dst/eptr/esrc/eg).
// Skipped (has_pairs = false: tier 2 keeps the block-per-string kernel) when
// the entries would exceed 2^27.
int build_pair_tables(wfsa_dev* ctx, const wfsa::TrellisModel& tm, const std::vector<int32_t>& cptr,
                      const std::vector<int32_t>& dst, const std::vector<int32_t>& eptr,
                      const std::vector<int32_t>& esrc, const std::vector<int32_t>& eg,
                      const std::vector<int32_t>& pptr, const std::vector<int32_t>& pidx) {
    ctx->has_pairs = false;
    hipStream_t s = ctx->stream;
    std::vector<int32_t> bidx(256, -1), bytes;
    for (int c = 0; c < 256; ++c)
        if (cptr[size_t(c) + 1] > cptr[size_t(c)]) {
            bidx[size_t(c)] = int32_t(bytes.size());
            bytes.push_back(c);
        }
    const int K = int(bytes.size());
    if (K == 0) return WFSA_OK;
    // D(b) for b < K, then {start}
    std::vector<int32_t> n(size_t(K) + 1), dl_ptr(size_t(K) + 2, 0), dl_node;
    for (int b = 0; b < K; ++b) {
        const int c = bytes[size_t(b)];
        n[size_t(b)] = cptr[size_t(c) + 1] - cptr[size_t(c)];
        for (int k = cptr[size_t(c)]; k < cptr[size_t(c) + 1]; ++k) dl_node.push_back(dst[size_t(k)]);
        dl_ptr[size_t(b) + 1] = int32_t(dl_node.size());
    }
    n[size_t(K)] = 1;
    dl_node.push_back(tm.start);
    dl_ptr[size_t(K) + 1] = int32_t(dl_node.size());
    int32_t max_n = 1;
    for (int32_t v : n) max_n = std::max(max_n, v);
    {   // build cost (and table index size) bounded: pairs x groups, pairs' in-edge scans
        int64_t groups = 0;
        for (int b = 0; b <= K; ++b) groups += (int64_t(n[size_t(b)]) + kWave - 1) / kWave;
        if (int64_t(K + 1) * groups > (int64_t(1) << 22) || int64_t(K + 1) * int64_t(esrc.size()) > (int64_t(1) << 28))
            return WFSA_OK;
    }
    // node -> index in D(a), one a at a time
    if (max_n >= 65536) return WFSA_OK;   // indices are packed in 16 bits
    const int32_t N = tm.n_nodes;
    std::vector<int32_t> idx_a(size_t(N), -1), idx_b(size_t(N), -1);
    auto fill = [&](std::vector<int32_t>& idx, int a, bool on) {
        for (int32_t q = dl_ptr[size_t(a)]; q < dl_ptr[size_t(a) + 1]; ++q) idx[size_t(dl_node[size_t(q)])] = on ? q - dl_ptr[size_t(a)] : -1;
    };
    const int64_t n_pairs = int64_t(K + 1) * K;
    std::vector<int32_t> e_ptr(size_t(n_pairs) + 1, 0);
    std::vector<int4> ent;
    constexpr int64_t kCap = int64_t(1) << 27;
    for (int a = 0; a <= K; ++a) {
        fill(idx_a, a, true);
        for (int b = 0; b < K; ++b) {
            const int c = bytes[size_t(b)];
            fill(idx_b, b, true);
            // the pair's edges, by destination (the in-edge lists of D(b)) with a source in D(a)
            for (int32_t k = cptr[size_t(c)]; k < cptr[size_t(c) + 1]; ++k) {
                const int32_t di = k - cptr[size_t(c)];
                for (int32_t e = eptr[size_t(k)]; e < eptr[size_t(k) + 1]; ++e) {
                    const int32_t si = idx_a[size_t(esrc[size_t(e)])];
                    if (si < 0) continue;
                    const int32_t g = eg[size_t(e)];
                    const int32_t pc = pptr[size_t(g) + 1] - pptr[size_t(g)];
                    const int32_t p0 = pc > 2 ? -2 : (pc >= 1 ? pidx[size_t(pptr[size_t(g)])] : -1);
                    const int32_t p1 = pc == 2 ? pidx[size_t(pptr[size_t(g)]) + 1] : -1;
                    ent.push_back(make_int4(int32_t(uint32_t(si) | (uint32_t(di) << 16)), g, p0, p1));
                }
            }
            if (int64_t(ent.size()) > kCap) return WFSA_OK;
            e_ptr[size_t(int64_t(a) * K + b) + 1] = int32_t(ent.size());
            fill(idx_b, b, false);
        }
        fill(idx_a, a, false);
    }
    if (ent.empty()) ent.push_back(make_int4(0, 0, -1, -1));
    HIP_TRY(ctx->pt_bidx.upload(bidx.data(), bidx.size(), s));
    HIP_TRY(ctx->pt_n.upload(n.data(), n.size(), s));
    HIP_TRY(ctx->pt_dlptr.upload(dl_ptr.data(), dl_ptr.size(), s));
    HIP_TRY(ctx->pt_dlnode.upload(dl_node.data(), dl_node.size(), s));
    HIP_TRY(ctx->pt_eptr.upload(e_ptr.data(), e_ptr.size(), s));
    HIP_TRY(ctx->pt_ent.upload(ent.data(), ent.size(), s));
    {
        std::vector<int32_t> sdv(ent.size());
        for (size_t e = 0; e < ent.size(); ++e) sdv[e] = ent[e].x;
        HIP_TRY(ctx->pt_sd.upload(sdv.data(), sdv.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    HIP_TRY(ctx->pt_w.alloc(2 * ent.size()));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->pt_K = K;
    ctx->pt_max_n = max_n;
    ctx->pt_ne = int64_t(ent.size());
    if (int rc = build_pull_tables(ctx, K, n, e_ptr, ent)) return rc;
    ctx->has_pairs = true;
    return WFSA_OK;
}

// The equivocal parameters of one string (HessianLearner::AssembleH's
// per-string sets, src/HessianLearner.cpp:388-437): those whose count is not
// the same on every accepting path, from exact min / max counts over the
// string's trellis.  false: the string has more than cap_p parameters on its
// paths (the per-node count vectors would not fit).
bool equivocal_params(const wfsa::TrellisModel& tm, const std::vector<int32_t>& pptr,
                      const std::vector<int32_t>& pidx, const uint8_t* str, int L, std::vector<int32_t>& V,
                      size_t cap_p) {
    const int32_t N = tm.n_nodes, E = int32_t(tm.o_byte.size());
    V.clear();
    std::vector<std::vector<int32_t>> live(size_t(L) + 1);   // co-reachable (accepting) nodes per position
    {
        std::vector<std::vector<char>> fw(size_t(L) + 1, std::vector<char>(size_t(N), 0));
        fw[0][size_t(tm.start)] = 1;
        for (int i = 0; i < L; ++i)
            for (int32_t S = 0; S < N; ++S)
                if (fw[size_t(i)][size_t(S)])
                    for (int32_t g = tm.o_ptr[size_t(S)]; g < tm.o_ptr[size_t(S) + 1]; ++g)
                        if (tm.o_byte[size_t(g)] == str[i]) fw[size_t(i) + 1][size_t(tm.o_dst[size_t(g)])] = 1;
        std::vector<char> bw(size_t(N), 0), nb(size_t(N), 0);
        for (int32_t S = 0; S < N; ++S)
            if (fw[size_t(L)][size_t(S)] && tm.x_ptr[size_t(S) + 1] > tm.x_ptr[size_t(S)]) {
                bw[size_t(S)] = 1;
                live[size_t(L)].push_back(S);
            }
        for (int i = L - 1; i >= 0; --i) {
            std::fill(nb.begin(), nb.end(), 0);
            for (int32_t S = 0; S < N; ++S) {
                if (!fw[size_t(i)][size_t(S)]) continue;
                for (int32_t g = tm.o_ptr[size_t(S)]; g < tm.o_ptr[size_t(S) + 1]; ++g)
                    if (tm.o_byte[size_t(g)] == str[i] && bw[size_t(tm.o_dst[size_t(g)])]) nb[size_t(S)] = 1;
                if (nb[size_t(S)]) live[size_t(i)].push_back(S);
            }
            bw.swap(nb);
        }
    }
    // the parameters on accepting edges
    std::vector<int32_t> P;
    auto add_params = [&](int32_t g) {
        for (int32_t q = pptr[size_t(g)]; q < pptr[size_t(g) + 1]; ++q) P.push_back(pidx[size_t(q)]);
    };
    std::vector<char> on(size_t(N), 0);
    for (int i = 0; i < L; ++i) {
        for (int32_t T : live[size_t(i) + 1]) on[size_t(T)] = 1;
        for (int32_t S : live[size_t(i)])
            for (int32_t g = tm.o_ptr[size_t(S)]; g < tm.o_ptr[size_t(S) + 1]; ++g)
                if (tm.o_byte[size_t(g)] == str[i] && on[size_t(tm.o_dst[size_t(g)])]) add_params(g);
        for (int32_t T : live[size_t(i) + 1]) on[size_t(T)] = 0;
    }
    for (int32_t S : live[size_t(L)])
        for (int32_t x = tm.x_ptr[size_t(S)]; x < tm.x_ptr[size_t(S) + 1]; ++x) add_params(E + x);
    std::sort(P.begin(), P.end());
    P.erase(std::unique(P.begin(), P.end()), P.end());
    if (P.empty()) return true;
    if (P.size() > cap_p) return false;
    const size_t np = P.size();
    auto local = [&](int32_t j) { return size_t(std::lower_bound(P.begin(), P.end(), j) - P.begin()); };
    // min / max count of every parameter over the paths into each live node,
    // rows indexed by the node's place in live[i]
    const int32_t kInf = std::numeric_limits<int32_t>::max() / 4;
    std::vector<int32_t> at(size_t(N), -1);
    std::vector<int32_t> mn(np, 0), mx(np, 0), mn2, mx2;   // position 0: the start node alone
    std::vector<int32_t> cnt(np, 0);
    auto edge_counts = [&](int32_t g, int sign) {
        for (int32_t q = pptr[size_t(g)]; q < pptr[size_t(g) + 1]; ++q) cnt[local(pidx[size_t(q)])] += sign;
    };
    if (live[0].size() != 1 || live[0][0] != tm.start) return true;   // not recognized
    for (int i = 0; i < L; ++i) {
        const auto& cur = live[size_t(i)];
        const auto& nxt = live[size_t(i) + 1];
        mn2.assign(nxt.size() * np, kInf);
        mx2.assign(nxt.size() * np, -kInf);
        for (size_t t = 0; t < nxt.size(); ++t) at[size_t(nxt[t])] = int32_t(t);
        for (size_t si = 0; si < cur.size(); ++si) {
            const int32_t S = cur[si];
            for (int32_t g = tm.o_ptr[size_t(S)]; g < tm.o_ptr[size_t(S) + 1]; ++g) {
                const int32_t T = tm.o_dst[size_t(g)];
                if (tm.o_byte[size_t(g)] != str[i] || at[size_t(T)] < 0) continue;
                const size_t ti = size_t(at[size_t(T)]);
                edge_counts(g, 1);
                for (size_t j = 0; j < np; ++j) {
                    mn2[ti * np + j] = std::min(mn2[ti * np + j], mn[si * np + j] + cnt[j]);
                    mx2[ti * np + j] = std::max(mx2[ti * np + j], mx[si * np + j] + cnt[j]);
                }
                edge_counts(g, -1);
            }
        }
        for (int32_t T : nxt) at[size_t(T)] = -1;
        mn.swap(mn2);
        mx.swap(mx2);
    }
    std::vector<int32_t> fmn(np, kInf), fmx(np, -kInf);
    const auto& last = live[size_t(L)];
    for (size_t si = 0; si < last.size(); ++si) {
        const int32_t S = last[si];
        for (int32_t x = tm.x_ptr[size_t(S)]; x < tm.x_ptr[size_t(S) + 1]; ++x) {
            edge_counts(E + x, 1);
            for (size_t j = 0; j < np; ++j) {
                fmn[j] = std::min(fmn[j], mn[si * np + j] + cnt[j]);
                fmx[j] = std::max(fmx[j], mx[si * np + j] + cnt[j]);
            }
            edge_counts(E + x, -1);
        }
    }
    for (size_t j = 0; j < np; ++j)
        if (fmn[j] != fmx[j]) V.push_back(P[j]);
    return true;
}

int configure_tiers(wfsa_dev* ctx) {
    // tier 0: 4 waves per block, ~20 KB per wave (8 waves per CU), grown to
    // fit large automata; tier 1: one wave per block with the whole LDS.
    ctx->cfg[0] = wfsa::SlabConfig{};
    ctx->cfg[1] = wfsa::SlabConfig{};
    bool ok0 = false;
    for (int budget : {20480, 40960}) {
        if (make_slab(budget, ctx->max_len, ctx->n_nodes, 4, ctx->cfg[0], ctx->lay[0])) {
            ok0 = true;
            break;
        }
    }
    const bool ok1 = make_slab(kLdsPerCu - 1024, ctx->max_len, ctx->n_nodes, 1, ctx->cfg[1], ctx->lay[1]);
    if (!ok1) ctx->cfg[1] = wfsa::SlabConfig{};
    if (!ok0 && ok1) {
        ctx->cfg[0] = ctx->cfg[1];
        ctx->lay[0] = ctx->lay[1];
    }
    // neither fits (the node->slot map alone is too large): every string
    // takes tier 2 (wide_kernel, global scratch)
    ctx->prep_level = 0;
    return WFSA_OK;
}

// Structural pass (level 1) + stream compilation (level 2) for the loaded
// corpus.
void drop_graph(wfsa_dev* ctx);

int enqueue_compiled(wfsa_dev* ctx, bool with_grad, bool want_logq, const unsigned* halted = nullptr,
                     int slot = -1);
wfsa::BubbleArgs bubble_args(wfsa_dev* ctx, bool want_logq, const unsigned* halted, double* ll_part);
bool bubbles_fused(wfsa_dev* ctx, bool want_logq);
// waves per block of the stream kernel that take the small bubbles (64 each)
int small_waves_per_block(int64_t n_small, int nblk) {
    const int64_t waves = (n_small + kWave - 1) / kWave;
    return int((waves + nblk - 1) / std::max(nblk, 1));
}
// byte offset of the big bubbles' staging in the stream kernel's LDS (after w)
size_t big_stage_off(const wfsa_dev* ctx) { return (ctx->i_lds + 15) & ~size_t(15); }

// per-kernel timing events of slot `slot` (< 0: this launch is not timed;
// WFSA_TIMING=0 leaves them all out).  An event between two kernels costs a
// few microseconds of idle device, so QN runs time a sample of their steps.
hipError_t record(wfsa_dev* ctx, hipEvent_t* evs, int slot, hipStream_t s) {
    if (evs == ctx->k2 && slot >= 0) ctx->k2_kc[slot] = false;
    return ctx->kernel_timing && slot >= 0 ? hipEventRecord(evs[slot], s) : hipSuccess;
}

wfsa::Publish publish_args(wfsa_dev* ctx) {
    wfsa::Publish p{};
    p.host_out = ctx->pinned_dev;
    p.n = ctx->n_params + 1;
    p.seq = ctx->counters.ptr;
    p.host_flag = ctx->flag_dev;
    return p;
}

// Event timings of the previous call, read once its events have completed.
int collect_timing(wfsa_dev* ctx) {
    if (!ctx->timing_pending) return WFSA_OK;
    ctx->timing_pending = false;
    HIP_TRY(hipEventSynchronize(ctx->ev1));
    float c_ms = 0.f, fb_ms = 0.f, all_ms = 0.f;
    if (!ctx->graph_exec && ctx->kernel_timing) {   // events inside a captured graph are not timeable
        HIP_TRY(hipEventElapsedTime(&c_ms, ctx->k0[0], ctx->kc[0]));
        HIP_TRY(hipEventElapsedTime(&fb_ms, ctx->k0[0], ctx->k2_kc[0] ? ctx->kc[0] : ctx->k2[0]));
    }
    HIP_TRY(hipEventElapsedTime(&all_ms, ctx->ev0, ctx->ev1));
    const double fb = double(fb_ms);
    ctx->stats.fb_launches += 1;
    ctx->stats.fb_kernel_ms += fb;
    ctx->stats.last_fb_kernel_ms = fb;
    ctx->stats.last_compiled_ms = double(c_ms);
    ctx->stats.compiled_kernel_ms += double(c_ms);
    ctx->stats.last_call_ms = double(all_ms);
    ctx->stats.graph = ctx->graph_exec ? 1 : 0;
    return WFSA_OK;
}

// Wait until the published sequence number reaches `want` (wrapping
// compare): poll the host-mapped flag, and the stream now and then so a
// failed launch surfaces as an error.
int wait_published(wfsa_dev* ctx, unsigned want) {
    auto reached = [&] { return int(__atomic_load_n(ctx->flag, __ATOMIC_ACQUIRE) - want) >= 0; };
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t spin = 1;; ++spin) {
        if (reached()) {   // (a failed peer all-reduce publishes NaN: say why instead)
            if (ctx->comm && ctx->comm->check())
                return fail(WFSA_ERR_RCCL, "%s all-reduce: %s", ctx->comm->kind(), ctx->comm->last_error());
            return WFSA_OK;
        }
        if ((spin & 0x3fff) == 0) {
            const hipError_t e = hipStreamQuery(ctx->stream);
            if (e == hipSuccess) {
                if (reached()) return WFSA_OK;
                return fail(WFSA_ERR_HIP, "device finished without publishing (sequence %u)", want);
            }
            if (e != hipErrorNotReady) return fail(WFSA_ERR_HIP, "device failure: %s", hipGetErrorString(e));
            // the communicator's liveness (an RCCL error or a stalled member
            // aborts it; its pending kernels on this rank then end)
            if (ctx->comm &&
                ctx->comm->watchdog(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count()))
                return fail(WFSA_ERR_RCCL, "%s all-reduce: %s", ctx->comm->kind(), ctx->comm->last_error());
        }
        __builtin_ia32_pause();
    }
}

// Until ring row `row` holds the row with sequence number `want` (row[7] =
// status + 16 tag, qn_publish_row): the flag said it was published.
int wait_row(wfsa_dev* ctx, const double* row, unsigned want) {
    auto tag = [&] {
        const uint64_t bits = __atomic_load_n(reinterpret_cast<const uint64_t*>(row + 7), __ATOMIC_ACQUIRE);
        double v;
        std::memcpy(&v, &bits, sizeof v);
        return unsigned(uint64_t(v) >> 4);
    };
    for (uint64_t spin = 1; tag() != want; ++spin) {
        if ((spin & 0x3fff) == 0) {
            const hipError_t e = hipStreamQuery(ctx->stream);
            if (e == hipSuccess && tag() != want)
                return fail(WFSA_ERR_HIP, "device finished without writing info row %u (found %u)", want, tag());
            if (e != hipSuccess && e != hipErrorNotReady) return fail(WFSA_ERR_HIP, "device failure: %s", hipGetErrorString(e));
        }
        __builtin_ia32_pause();
    }
    return WFSA_OK;
}

// Contribution slots of the compiled bubbles in slot order pos_of (full
// parameter j at position pos_of[j]): every (bubble edge, parameter) pair
// gets a slot, parameter-major by position -- within a parameter small
// bubbles, then big, in bubble order -- and the small-bubble tables / big
// bubble slot lists are rebuilt to match; seg_ptr (by position), param_at and
// the reduction's tiles follow.  Runs again when the QN loop moves the slots
// into its trimmed order (wfsa_dev_qn_setup).
int layout_slots(wfsa_dev* ctx, const std::vector<int32_t>& pos_of) {
    hipStream_t s = ctx->stream;
    const int32_t np = ctx->n_params;
    const std::vector<int32_t>& bb = ctx->h_bubbuf;
    auto edge_code_at = [&](int32_t o, int e) { return bb[size_t(o) + 4 + 2 * size_t(e)]; };
    auto for_edge_params = [&](int32_t code, auto&& f) {   // the parameters of a bubble edge (edge_code)
        if (code >= 0) {
            if (code < np) f(code);
        } else {
            const int32_t g = -code - 2;
            for (int32_t q = ctx->h_pptr[size_t(g)]; q < ctx->h_pptr[size_t(g) + 1]; ++q) f(ctx->h_pidx[size_t(q)]);
        }
    };
    std::vector<int32_t> param_at(size_t(std::max(np, 1)), 0);
    for (int32_t j = 0; j < np; ++j) param_at[size_t(pos_of[size_t(j)])] = j;
    // Small bubbles run one per lane, 64 consecutive list entries (class A
    // then class B) per wavefront, sorted by shape: where an aligned group of
    // 2^k lanes of one class all carry parameter j on edge e, the lanes sum
    // their contributions by a butterfly and the group's first lane stores
    // one slot (fb_kernels.hip small_bubble); lvl[b * 8 + e] = k
    const int64_t n4 = int64_t(ctx->h_sm4_list.size()), nsm = n4 + int64_t(ctx->h_sm_list.size());
    auto small_o = [&](int64_t b) { return b < n4 ? ctx->h_sm4_list[size_t(b)] : ctx->h_sm_list[size_t(b - n4)]; };
    auto small_code = [&](int64_t b, int e) -> int32_t {   // its parameter on edge e, or -1
        const int32_t o = small_o(b);
        if (e >= (bb[size_t(o)] >> 16)) return -1;
        const int32_t c = edge_code_at(o, e);
        return c >= 0 && c < np ? c : -1;
    };
    std::vector<uint8_t> lvl(size_t(std::max<int64_t>(nsm, 1)) * 8, 0);
    const bool merge = [] {   // WFSA_SLOT_MERGE=0: a slot per small-bubble edge (read at each layout)
        const char* e = std::getenv("WFSA_SLOT_MERGE");
        return !(e && e[0] == '0');
    }();
    // (a wavefront's lanes: 64 consecutive entries of one class, from the
    // class's first entry -- wfsa::small_entry -- so lane = (b - base) & 63)
    auto wave_base = [&](int64_t b) { return b < n4 ? int64_t(0) : n4; };
    for (int64_t g0 = 0; merge && g0 < nsm; g0 = std::min(g0 + kWave, g0 < n4 ? n4 : nsm)) {
        const int64_t gend = std::min(g0 + kWave, g0 < n4 ? n4 : nsm);
        for (int e = 0; e < wfsa::kBubbleRegEdges; ++e)
            for (int k = 6; k >= 1; --k) {   // largest aligned groups first
                const int64_t G = int64_t(1) << k;
                for (int64_t b0 = g0; b0 + G <= gend; b0 += G) {
                    if (lvl[size_t(b0) * 8 + size_t(e)]) continue;   // inside a larger group
                    const int32_t c = small_code(b0, e);
                    bool same = c >= 0;
                    for (int64_t b = b0 + 1; same && b < b0 + G; ++b) same = small_code(b, e) == c && !lvl[size_t(b) * 8 + size_t(e)];
                    if (same)
                        for (int64_t b = b0; b < b0 + G; ++b) lvl[size_t(b) * 8 + size_t(e)] = uint8_t(k);
                }
            }
    }
    auto leader = [&](int64_t b, int e) {
        return ((b - wave_base(b)) & ((int64_t(1) << lvl[size_t(b) * 8 + size_t(e)]) - 1)) == 0;
    };
    std::vector<int32_t> pc(size_t(np) + 1, 0);   // by position
    for (int64_t b = 0; b < nsm; ++b)
        for (int e = 0; e < wfsa::kBubbleRegEdges; ++e) {
            const int32_t c = small_code(b, e);
            if (c >= 0 && leader(b, e)) pc[size_t(pos_of[size_t(c)]) + 1]++;
        }
    for (int32_t o : ctx->h_big_list)
        for (int e = 0; e < (bb[size_t(o)] >> 16); ++e)
            for_edge_params(edge_code_at(o, e), [&](int32_t jj) { pc[size_t(pos_of[size_t(jj)]) + 1]++; });
    for (size_t q = 1; q < pc.size(); ++q) pc[q] += pc[q - 1];
    std::vector<int32_t> fill(pc.begin(), pc.end() - 1);
    // Reduction groups over the positions: the QN constraints when the slots
    // follow its trimmed order (ctx->slot_groups), then runs of consecutive
    // positions (at most kReduceTileParams parameters and, unless one alone
    // has more, kMaxChunks chunks).  Parameter q's slots form chunks of
    // kSlotChunk (seg_sums, qn_device.hpp: its sum depends on its own slots
    // only), stored contiguously -- a parameter's slots are consecutive
    // addresses, so the stores of lanes whose (sorted, same-shaped) bubbles
    // share a parameter coalesce; seg_sums reads a chunk with eight lanes.
    std::vector<int32_t> cptr_pos(size_t(np) + 1, 0);   // chunks by position, cumulative
    for (int32_t q = 0; q < np; ++q)
        cptr_pos[size_t(q) + 1] = cptr_pos[size_t(q)] + (pc[size_t(q) + 1] - pc[size_t(q)] + wfsa::kSlotChunk - 1) / wfsa::kSlotChunk;
    std::vector<int32_t> gp(1, 0);
    for (size_t i = 1; i < ctx->slot_groups.size() && ctx->slot_groups[i] <= np; ++i) gp.push_back(ctx->slot_groups[i]);
    for (int32_t q = gp.back(); q < np;) {
        int32_t e = q + 1;
        while (e < np && e - q < wfsa::kReduceTileParams && cptr_pos[size_t(e) + 1] - cptr_pos[size_t(q)] <= wfsa::kMaxChunks) ++e;
        gp.push_back(e);
        q = e;
    }
    const int32_t ng = int32_t(gp.size()) - 1;
    std::vector<int64_t> gbase(size_t(ng) + 1, 0);
    std::vector<int32_t> grp_of(size_t(std::max(np, 1)), 0);
    for (int32_t g = 0; g < ng; ++g) {
        const int64_t nch = cptr_pos[size_t(gp[size_t(g) + 1])] - cptr_pos[size_t(gp[size_t(g)])];
        gbase[size_t(g) + 1] = gbase[size_t(g)] + nch * wfsa::kSlotChunk;
        for (int32_t q = gp[size_t(g)]; q < gp[size_t(g) + 1]; ++q) grp_of[size_t(q)] = g;
    }
    auto phys = [&](int32_t pos, int32_t sl) -> int32_t {   // logical slot sl of position pos
        const int32_t g = grp_of[size_t(pos)], cg = cptr_pos[size_t(gp[size_t(g)])];
        const int32_t i = sl - pc[size_t(pos)];
        return int32_t(gbase[size_t(g)] + int64_t(cptr_pos[size_t(pos)] - cg) * wfsa::kSlotChunk + i);
    };
    if (gbase.back() >= int64_t(1) << 28) return fail(WFSA_ERR_CAPACITY, "too many bubble contribution slots");
    if (ctx->n_bubbles > 0) {
        // the small bubbles' slot fields: slot | group level << 28 (every lane
        // of a group carries the group's slot; its first lane stores)
        std::vector<int32_t> sfield(size_t(std::max<int64_t>(nsm, 1)) * 8, -1);
        for (int64_t b = 0; b < nsm; ++b)
            for (int e = 0; e < wfsa::kBubbleRegEdges; ++e) {
                const int32_t c = small_code(b, e);
                if (c < 0 || !leader(b, e)) continue;
                const int32_t pos = pos_of[size_t(c)];
                const int k = lvl[size_t(b) * 8 + size_t(e)];
                const int32_t f = phys(pos, fill[size_t(pos)]++) | (int32_t(k) << 28);
                for (int64_t q = b; q < b + (int64_t(1) << k); ++q) sfield[size_t(q) * 8 + size_t(e)] = f;
            }
        // class tables: RE edges, quads = 1 + RE/2 + RE/4
        auto build_table = [&](const std::vector<int32_t>& list, int RE, std::vector<int32_t>& tbl, int64_t b_first) {
            const int Q = 1 + RE / 2 + RE / 4;
            const size_t n = list.size();
            tbl.assign(size_t(Q) * 4 * std::max<size_t>(n, 1), 0);
            auto quad = [&](int k, size_t b) { return &tbl[(size_t(k) * n + b) * 4]; };
            for (size_t b = 0; b < n; ++b) {
                const int32_t o = list[b];
                const int edges = bb[size_t(o)] >> 16;
                for (int w = 0; w < 4; ++w) quad(0, b)[w] = bb[size_t(o) + size_t(w)];
                for (int e = 0; e < RE; ++e) {
                    int32_t code = np, sd = 0, sl = -1;   // padding edges: the zero-slot code
                    if (e < edges) {
                        code = edge_code_at(o, e);
                        sd = bb[size_t(o) + 5 + 2 * size_t(e)];
                        sl = sfield[size_t(b_first + int64_t(b)) * 8 + size_t(e)];
                    }
                    quad(1 + e / 2, b)[2 * (e & 1)] = code;
                    quad(1 + e / 2, b)[2 * (e & 1) + 1] = sd;
                    quad(1 + RE / 2 + e / 4, b)[e & 3] = sl;
                }
            }
        };
        std::vector<int32_t> tbl4, tbl;
        build_table(ctx->h_sm4_list, 4, tbl4, 0);
        build_table(ctx->h_sm_list, wfsa::kBubbleRegEdges, tbl, n4);
        const int64_t nb = int64_t(ctx->h_big_list.size());
        std::vector<int32_t> big_edge_base(size_t(std::max<int64_t>(nb, 1)), 0), eslot_ptr(1, 0), eslot;
        for (int64_t i = 0; i < nb; ++i) {
            const int32_t o = ctx->h_big_list[size_t(i)];
            big_edge_base[size_t(i)] = int32_t(eslot_ptr.size()) - 1;
            for (int e = 0; e < (bb[size_t(o)] >> 16); ++e) {
                for_edge_params(edge_code_at(o, e), [&](int32_t jj) {
                    const int32_t pos = pos_of[size_t(jj)];
                    eslot.push_back(phys(pos, fill[size_t(pos)]++));
                });
                eslot_ptr.push_back(int32_t(eslot.size()));
            }
        }
        if (eslot.empty()) eslot.push_back(0);
        HIP_TRY(ctx->sm4_tbl.upload(reinterpret_cast<const int4*>(tbl4.data()), tbl4.size() / 4, s));
        HIP_TRY(ctx->sm_tbl.upload(reinterpret_cast<const int4*>(tbl.data()), tbl.size() / 4, s));
        const std::vector<int32_t>& bl = ctx->h_big_list;
        HIP_TRY(ctx->big_off.upload(bl.empty() ? eslot.data() : bl.data(), std::max<size_t>(bl.size(), 1), s));
        HIP_TRY(ctx->big_edge_base.upload(big_edge_base.data(), big_edge_base.size(), s));
        HIP_TRY(ctx->big_eslot_ptr.upload(eslot_ptr.data(), eslot_ptr.size(), s));
        HIP_TRY(ctx->big_eslot.upload(eslot.data(), eslot.size(), s));
    }
    if (ctx->n_bubbles > 0) {
        const size_t n_phys = size_t(std::max<int64_t>(gbase.back(), 1));
        HIP_TRY(ctx->contrib.alloc(n_phys));
        HIP_TRY(hipMemsetAsync(ctx->contrib.ptr, 0, n_phys * sizeof(double), s));   // padding stays zero
    }
    ctx->n_tiles = ng;
    HIP_TRY(ctx->grp_base.upload(gbase.data(), gbase.size(), s));
    {
        std::vector<int32_t> gn(size_t(std::max(ng, 1)), 0);
        for (int32_t g = 0; g < ng; ++g) gn[size_t(g)] = cptr_pos[size_t(gp[size_t(g) + 1])] - cptr_pos[size_t(gp[size_t(g)])];
        HIP_TRY(ctx->grp_nch.upload(gn.data(), gn.size(), s));
        ctx->lead_grp_nch = 1;   // the largest constraint-led group's chunk count (the QN step's LDS)
        for (size_t g = 0; g + 1 < ctx->slot_groups.size() && int32_t(g) < ng; ++g)
            ctx->lead_grp_nch = std::max(ctx->lead_grp_nch, gn[g]);
        ctx->stats.max_group_chunks = ctx->lead_grp_nch;
        ctx->stats.slot_chunks = ctx->n_bubbles > 0 ? int64_t(gbase.back()) / wfsa::kSlotChunk : 0;
    }
    {   // per position: the first contribution slot of its chunks and their count (the in-kernel QN update)
        std::vector<int64_t> mchunk(size_t(std::max(np, 1)), 0);
        std::vector<int32_t> mnch(size_t(std::max(np, 1)), 0);
        for (int32_t q = 0; q < np; ++q) {
            const int32_t g = grp_of[size_t(q)];
            mchunk[size_t(q)] = gbase[size_t(g)] + int64_t(cptr_pos[size_t(q)] - cptr_pos[size_t(gp[size_t(g)])]) * wfsa::kSlotChunk;
            mnch[size_t(q)] = cptr_pos[size_t(q) + 1] - cptr_pos[size_t(q)];
        }
        ctx->h_mchunk = std::move(mchunk);
        ctx->h_mnch = std::move(mnch);
        ++ctx->layout_gen;
    }
    HIP_TRY(ctx->chunk_ptr.upload(cptr_pos.data(), cptr_pos.size(), s));
    HIP_TRY(ctx->seg_ptr.upload(pc.data(), pc.size(), s));
    HIP_TRY(ctx->param_at.upload(param_at.data(), param_at.size(), s));
    HIP_TRY(ctx->tile_ptr.upload(gp.data(), gp.size(), s));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->h_seg_ptr = std::move(pc);
    ctx->slot_order = pos_of;
    drop_graph(ctx);   // a captured evaluation holds the old tables
    return WFSA_OK;
}

// Dense automata: no compilation; level 1 is the structural pass, one
// evaluation at all-ones weights and p: log q = log(path count), and a
// parameter is used iff its expected count is positive.
int prepare_dense(wfsa_dev* ctx, int level) {
    const auto t_start = std::chrono::steady_clock::now();
    hipStream_t s = ctx->stream;
    const int64_t S = ctx->n_strings;
    const size_t SZ = size_t(std::max<int64_t>(S, 1));
    const int32_t np = ctx->n_params;
    if (level >= 1 && !ctx->dense_struct) {
        HIP_TRY(ctx->pcount.alloc(SZ));
        HIP_TRY(ctx->recog.alloc(SZ));
        HIP_TRY(ctx->used.alloc(size_t(std::max(np, 1))));
        HIP_TRY(ctx->dense->enqueue(nullptr, true, ctx->out.ptr, ctx->logq.ptr, nullptr, s));
        std::vector<double> out(size_t(np) + 1), lq(SZ), pc(SZ);
        HIP_TRY(ctx->out.download(out.data(), out.size(), s));
        HIP_TRY(ctx->logq.download(lq.data(), size_t(S), s));
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<uint8_t> rec(SZ, 0), used(size_t(std::max(np, 1)), 0);
        for (int64_t i = 0; i < S; ++i) {
            rec[size_t(i)] = lq[size_t(i)] > -INFINITY ? 1 : 0;
            const double c = std::exp(lq[size_t(i)]);
            pc[size_t(i)] = c < 9007199254740992.0 ? std::nearbyint(c) : c;   // exact below 2^53
        }
        for (int32_t j = 0; j < np; ++j) used[size_t(j)] = out[size_t(j) + 1] < 0.0 ? 1 : 0;
        HIP_TRY(ctx->recog.upload(rec.data(), SZ, s));
        HIP_TRY(ctx->pcount.upload(pc.data(), SZ, s));
        HIP_TRY(ctx->used.upload(used.data(), used.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
        ctx->dense_struct = true;
    }
    ctx->prep_level = std::max(ctx->prep_level, 2);
    ctx->stats.compiled_strings = 0;
    ctx->stats.fallback_strings = 0;
    ctx->stats.prepare_ms +=
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    return WFSA_OK;
}

// fn(begin, end) over [0, n) on up to 16 host threads (the GPU box's CPU share)
template <class F>
void parallel_for(int64_t n, F&& fn) {
    const int64_t hc = std::max<int64_t>(1, int64_t(std::thread::hardware_concurrency()));
    const int nt = int(std::max<int64_t>(1, std::min<int64_t>({16, hc, n / 4096 + 1})));
    if (nt == 1) {
        fn(int64_t(0), n);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&fn, n, t, nt] { fn(n * t / nt, n * (t + 1) / nt); });
    for (auto& x : th) x.join();
}

// The per-iteration kernel's delta-format streams (fb_kernels.hpp): every
// compiled string's trivial words read back from the 16-bit streams,
// remapped (delta_slot), sorted and written as 10-bit steps; the strings
// regrouped by their delta rows (longest first, 64 per group) and the groups
// dealt to the waves by the same rule as the 16-bit groups.
template <class Deal>
int build_delta(wfsa_dev* ctx, const std::vector<int32_t>& comp, const std::vector<int32_t>& h_main,
                const std::vector<int64_t>& s_base, const std::vector<double>& h_p, int64_t chunks, int32_t G,
                const std::vector<int32_t>& rows16_of, Deal&& deal) {
    hipStream_t s = ctx->stream;
    const int64_t nc = int64_t(comp.size());
    std::vector<uint16_t> h16(size_t(chunks) * 8);
    HIP_TRY(ctx->stream_w.download(reinterpret_cast<uint4*>(h16.data()), size_t(chunks), s));
    HIP_TRY(hipStreamSynchronize(s));
    const int hdr16 = wfsa::stream_hdr_words(0);
    auto words_of = [&](int32_t str, std::vector<uint32_t>& r) {
        r.clear();
        const int64_t c0 = s_base[size_t(str)] / 8;   // the lane's first chunk
        for (int k = 0; k < h_main[size_t(str)]; ++k) {
            const int slot = hdr16 + k;
            const uint16_t wd = h16[size_t(c0 + int64_t(kWave) * (slot / 8)) * 8 + size_t(slot % 8)];
            r.push_back(uint32_t(wfsa::delta_slot(int32_t(wd))));
        }
        std::sort(r.begin(), r.end());
    };
    const uint32_t z_end = uint32_t(wfsa::delta_end_slot(ctx->n_params));
    auto encode = [z_end](const std::vector<uint32_t>& r, auto&& emit) {
        constexpr uint32_t M = wfsa::kDeltaMax, P = wfsa::kDeltaPeriod;
        uint32_t cur = 0;
        for (uint32_t t : r) {
            while (t - cur > M) {   // onto the farthest zero slot within one step
                const uint32_t z = (cur + M) / P * P;
                emit(z - cur);
                cur = z;
            }
            emit(t - cur);
            cur = t;
        }
        if (cur % P) emit(std::min((cur / P + 1) * P, z_end) - cur);   // end on a zero slot: the padding adds nothing
    };
    auto rows_of = [](int64_t nf) {
        return nf <= wfsa::kDeltaHdrFields
                   ? 1
                   : 1 + int32_t((nf - wfsa::kDeltaHdrFields + wfsa::kDeltaFields - 1) / wfsa::kDeltaFields);
    };
    std::vector<int32_t> drows(size_t(std::max<int64_t>(nc, 1)));
    parallel_for(nc, [&](int64_t b, int64_t e) {
        std::vector<uint32_t> r;
        for (int64_t i = b; i < e; ++i) {
            words_of(comp[size_t(i)], r);
            int64_t nf = 0;
            encode(r, [&](uint32_t) { ++nf; });
            drows[size_t(i)] = rows_of(nf);
        }
    });
    // regroup, longest first (stable counting sort over the rows)
    int32_t max_rows = 1;
    for (int64_t i = 0; i < nc; ++i) max_rows = std::max(max_rows, drows[size_t(i)]);
    if (max_rows > 0xffff) return fail(WFSA_ERR_CAPACITY, "delta stream: %d rows exceed the group header", max_rows);
    std::vector<int64_t> cnt(size_t(max_rows) + 2, 0);
    for (int64_t i = 0; i < nc; ++i) cnt[size_t(max_rows - drows[size_t(i)])]++;
    int64_t acc = 0;
    for (auto& c : cnt) {
        const int64_t t = c;
        c = acc;
        acc += t;
    }
    std::vector<int32_t> dcomp(size_t(std::max<int64_t>(nc, 1))), drow_of(size_t(std::max<int64_t>(nc, 1)));
    for (int64_t i = 0; i < nc; ++i) {
        const int64_t k = cnt[size_t(max_rows - drows[size_t(i)])]++;
        dcomp[size_t(k)] = comp[size_t(i)];
        drow_of[size_t(k)] = drows[size_t(i)];
    }
    std::vector<int32_t> grows(size_t(std::max(G, 1)), 0);
    for (int32_t g = 0; g < G; ++g) grows[size_t(g)] = drow_of[size_t(g) * kWave];
    // the bubble charges in delta rows: a wave's stream time goes with its
    // bytes, so scale by the two formats' total rows
    double rows16 = 0.0, rowsd = 0.0;
    for (int32_t g = 0; g < G; ++g) {
        rows16 += double(rows16_of[size_t(g)]);
        rowsd += double(grows[size_t(g)]);
    }
    std::vector<int32_t> dorder, dwf;
    deal(grows, dorder, dwf, rows16 > 0.0 ? rowsd / rows16 : 1.0);
    ctx->qw_mean_rows = rowsd / double(std::max(1, ctx->i_grid * (ctx->i_block / kWave) - 1));
    std::vector<int64_t> dg_base(size_t(G) + 1, 0);
    std::vector<int32_t> dg_len(size_t(std::max(G, 1)), 0), dl_str(size_t(std::max(G, 1)) * kWave, -1);
    int64_t dch = 0;
    for (int32_t g = 0; g < G; ++g) {
        const int32_t src = dorder[size_t(g)];
        dg_base[size_t(g)] = dch;
        dg_len[size_t(g)] = grows[size_t(src)];
        for (int l = 0; l < kWave; ++l) {
            const int64_t ks = int64_t(src) * kWave + l;
            if (ks < nc) dl_str[size_t(g) * kWave + size_t(l)] = dcomp[size_t(ks)];
        }
        dch += int64_t(kWave) * dg_len[size_t(g)];
    }
    dg_base[size_t(G)] = dch;
    std::vector<uint32_t> hd(size_t(std::max<int64_t>(dch, 1)) * 4, 0u);
    parallel_for(int64_t(G), [&](int64_t b, int64_t e) {
        std::vector<uint32_t> r;
        for (int64_t g = b; g < e; ++g)
            for (int l = 0; l < kWave; ++l) {
                const int64_t base = dg_base[size_t(g)] + l;   // the lane's first row (chunk units)
                const int32_t str = dl_str[size_t(g) * kWave + size_t(l)];
                uint32_t* h = &hd[size_t(base) * 4];
                const double pv = str >= 0 ? h_p[size_t(str)] : 0.0;
                uint64_t pb;
                std::memcpy(&pb, &pv, sizeof pb);
                h[0] = uint32_t(pb);
                h[1] = uint32_t(pb >> 32);
                h[2] = uint32_t(dg_len[size_t(g)]);
                if (str < 0) continue;
                words_of(str, r);
                int64_t q = 0;
                encode(r, [&](uint32_t f) {
                    const int64_t row =
                        q < wfsa::kDeltaHdrFields ? 0 : 1 + (q - wfsa::kDeltaHdrFields) / wfsa::kDeltaFields;
                    const int slot = q < wfsa::kDeltaHdrFields
                                         ? int(wfsa::kDeltaFields - wfsa::kDeltaHdrFields + q)
                                         : int((q - wfsa::kDeltaHdrFields) % wfsa::kDeltaFields);
                    uint32_t* d = &hd[size_t(base + int64_t(kWave) * row) * 4];
                    d[slot / 3] |= f << (wfsa::kDeltaBits * (slot % 3));   // three fields per dword
                    ++q;
                });
            }
    });
    HIP_TRY(ctx->dstream.upload(reinterpret_cast<const uint4*>(hd.data()), size_t(std::max<int64_t>(dch, 1)), s));
    HIP_TRY(ctx->d_g_base.upload(dg_base.data(), dg_base.size(), s));
    HIP_TRY(ctx->d_g_len.upload(dg_len.data(), dg_len.size(), s));
    HIP_TRY(ctx->d_l_str.upload(dl_str.data(), dl_str.size(), s));
    HIP_TRY(ctx->d_wave_first.upload(dwf.data(), dwf.size(), s));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->delta_on = true;
    ctx->d_tab = wfsa::delta_table(ctx->n_params);
    ctx->d_stream_bytes = dch * 16;
    return WFSA_OK;
}

// The per-iteration (or, per_iteration false, the preparation-time) stream
// kernel's view of the compiled streams
void stream_args(const wfsa_dev* ctx, wfsa::CompiledArgs& c, bool per_iteration) {
    const bool d = per_iteration && ctx->delta_on;
    c.stream = d ? ctx->dstream.ptr : ctx->stream_w.ptr;
    c.g_base = d ? ctx->d_g_base.ptr : ctx->g_base.ptr;
    c.g_len = d ? ctx->d_g_len.ptr : ctx->g_len.ptr;
    c.l_str = d ? ctx->d_l_str.ptr : ctx->l_str.ptr;
    c.l_len = ctx->l_len.ptr;   // (the 16-bit layout's: only the gradient pass reads it)
    c.wave_first = d ? ctx->d_wave_first.ptr : ctx->wave_first.ptr;
    c.wide = ctx->wide;
    c.n_groups = ctx->n_groups;
    c.d_tab = d ? ctx->d_tab : 0;
}

int prepare(wfsa_dev* ctx, int level) {
    if (ctx->dense) return prepare_dense(ctx, level);
    if (ctx->mpath) {   // nothing to compile: the structure came with the matrices
        ctx->prep_level = 2;
        return WFSA_OK;
    }
    const auto t_start = std::chrono::steady_clock::now();
    drop_graph(ctx);
    hipStream_t s = ctx->stream;
    const int64_t S = ctx->n_strings;
    const size_t SZ = size_t(std::max<int64_t>(S, 1));
    HIP_TRY(ctx->overflow.alloc(SZ));
    HIP_TRY(ctx->pcount.alloc(SZ));
    HIP_TRY(ctx->recog.alloc(SZ));
    HIP_TRY(ctx->used.alloc(size_t(std::max(ctx->n_params, 1))));
    DevBuf<int32_t> c_main, c_bub, c_nbub;
    HIP_TRY(c_main.alloc(SZ));
    HIP_TRY(c_bub.alloc(SZ));
    HIP_TRY(c_nbub.alloc(SZ));
    HIP_TRY(hipMemsetAsync(ctx->overflow.ptr, 0, SZ, s));
    HIP_TRY(hipMemsetAsync(ctx->used.ptr, 0, size_t(std::max(ctx->n_params, 1)), s));
    HIP_TRY(hipMemsetAsync(c_main.ptr, 0, SZ * sizeof(int32_t), s));
    HIP_TRY(hipMemsetAsync(c_bub.ptr, 0xff, SZ * sizeof(int32_t), s));   // -1: not compiled
    HIP_TRY(hipMemsetAsync(c_nbub.ptr, 0, SZ * sizeof(int32_t), s));

    // 1. counting pass, tier 0 then tier 1 for strings that overflow; the
    // live trellis edges of every string accumulate in ctx->live (a structural
    // count: the work of one evaluation, whatever the weights)
    HIP_TRY(hipMemsetAsync(ctx->live.ptr, 0, sizeof(unsigned long long), s));
    std::vector<uint8_t> ovf(SZ, 0);
    std::vector<uint8_t> tier(SZ, 0);
    auto count_pass = [&](int t, const int32_t* list, int64_t n) -> int {
        wfsa::TravArgs a = trav_args(ctx, t);
        a.list = list;
        a.n_list = int32_t(n);
        a.path_count = ctx->pcount.ptr;
        a.recognized = ctx->recog.ptr;
        a.used = ctx->used.ptr;
        a.c_main = level >= 2 ? c_main.ptr : nullptr;
        a.c_bub = level >= 2 ? c_bub.ptr : nullptr;
        a.c_nbub = level >= 2 ? c_nbub.ptr : nullptr;
        HIP_TRY(wfsa::launch_trav(wfsa::MODE_COUNT, a, trav_grid(ctx->cfg[t], ctx->n_cu, n), s));
        return WFSA_OK;
    };
    if (S > 0 && ctx->cfg[0].bytes > 0 && !ctx->force_tier2) {
        if (int rc = count_pass(0, ctx->list_all.ptr, S)) return rc;
        HIP_TRY(ctx->overflow.download(ovf.data(), size_t(S), s));
        HIP_TRY(hipStreamSynchronize(s));
    } else {
        std::fill(ovf.begin(), ovf.end(), uint8_t(S > 0 ? 1 : 0));
    }
    std::vector<int32_t> l1, l2;
    for (int64_t i = 0; i < S; ++i)
        if (ovf[size_t(i)]) l1.push_back(int32_t(i));
    DevBuf<int32_t> d_l1, d_l2;
    if (!l1.empty() && ctx->cfg[1].bytes > 0 && !ctx->force_tier2) {
        HIP_TRY(d_l1.upload(l1.data(), l1.size(), s));
        HIP_TRY(hipMemsetAsync(ctx->overflow.ptr, 0, SZ, s));
        if (int rc = count_pass(1, d_l1.ptr, int64_t(l1.size()))) return rc;
        HIP_TRY(ctx->overflow.download(ovf.data(), size_t(S), s));
        HIP_TRY(hipStreamSynchronize(s));
        for (int32_t i : l1) {
            if (ovf[size_t(i)]) l2.push_back(i);
            else tier[size_t(i)] = 1;
        }
    } else {
        l2 = l1;
    }
    // tier 2: the strings no LDS slab holds
    if (!l2.empty()) {
        for (int32_t i : l2) tier[size_t(i)] = 2;
        const int g2 = wide_grid(ctx, int64_t(l2.size()));
        HIP_TRY(ctx->w_scratch.alloc(size_t(g2) * size_t(ctx->w_stride)));
        HIP_TRY(d_l2.upload(l2.data(), l2.size(), s));
        wfsa::WideArgs a = wide_args(ctx);
        a.list = d_l2.ptr;
        a.n_list = int32_t(l2.size());
        a.path_count = ctx->pcount.ptr;
        a.recognized = ctx->recog.ptr;
        a.used = ctx->used.ptr;
        a.live_edges = ctx->live.ptr;
        HIP_TRY(wfsa::launch_wide(true, a, g2, s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    ctx->tier2_strings = int32_t(l2.size());
    const int32_t n_tier1 = int32_t(l1.size() - l2.size());
    {
        unsigned long long live = 0;
        HIP_TRY(ctx->live.download(&live, 1, s));
        HIP_TRY(hipStreamSynchronize(s));
        ctx->stats.last_live_edges = int64_t(live);
    }

    if (level < 2) {
        ctx->stats.tier1_strings = n_tier1;
        ctx->prep_level = 1;
        return WFSA_OK;
    }

    // 2. groups of 64 strings with similar stream length
    std::vector<int32_t> h_main(SZ, 0), h_bub(SZ, -1), h_nb(SZ, 0);
    if (S > 0) {
        HIP_TRY(c_main.download(h_main.data(), size_t(S), s));
        HIP_TRY(c_bub.download(h_bub.data(), size_t(S), s));
        HIP_TRY(c_nbub.download(h_nb.data(), size_t(S), s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    std::vector<int32_t> comp, fb[3];
    int32_t max_main = 0;
    for (int64_t i = 0; i < S; ++i) {
        if (h_bub[size_t(i)] >= 0) {
            comp.push_back(int32_t(i));
            max_main = std::max(max_main, h_main[size_t(i)]);
        } else {
            fb[tier[size_t(i)]].push_back(int32_t(i));
        }
    }
    {   // counting sort, longest first
        std::vector<int64_t> cnt(size_t(max_main) + 2, 0);
        for (int32_t i : comp) cnt[size_t(max_main - h_main[size_t(i)])]++;
        int64_t acc = 0;
        for (auto& c : cnt) { const int64_t t = c; c = acc; acc += t; }
        std::vector<int32_t> sorted(comp.size());
        for (int32_t i : comp) sorted[size_t(cnt[size_t(max_main - h_main[size_t(i)])]++)] = i;
        comp.swap(sorted);
    }
    const int64_t nc = int64_t(comp.size());
    const int32_t G = int32_t((nc + kWave - 1) / kWave);
    // 16-byte chunks of 8 narrow / 4 wide words; chunk c of lane l at
    // g_base + 64 c + l (chunk units); s_base in word (element) units; each
    // lane's first chunk starts with the group header
    const int per = ctx->wide ? 4 : 8, hdr = wfsa::stream_hdr_words(ctx->wide);
    std::vector<int32_t> rows0(size_t(std::max(G, 1)), 0);   // rows of each group (sorted order)
    for (int32_t g = 0; g < G; ++g) {
        rows0[size_t(g)] = (h_main[size_t(comp[size_t(g) * kWave])] + hdr + per - 1) / per;
        if (!ctx->wide && rows0[size_t(g)] > 0xffff)
            return fail(WFSA_ERR_CAPACITY, "string %d: %d stream words exceed the narrow group header",
                        comp[size_t(g) * kWave], h_main[size_t(comp[size_t(g) * kWave])]);
    }
    // the per-iteration kernel's geometry: w staged in LDS when it fits, 16
    // waves per block, one block per CU (every block stages the whole table,
    // so fewer blocks stage less: measured 1/CU beats 2/CU at c3)
    // the per-iteration kernel reads the delta format (fb_kernels.hpp) when it
    // stages the weights and no stream word is a multi-parameter composite
    const bool delta_want = ctx->use_delta && !ctx->wide && ctx->n_multi == 0 && nc > 0;
    {
        const size_t table_bytes = size_t(ctx->n_params) * sizeof(double);
        size_t stage_bytes = table_bytes + 16;   // + the zero slot, even count
        if (delta_want) stage_bytes = std::max(stage_bytes, size_t(wfsa::delta_table(ctx->n_params)) * sizeof(double));
        ctx->i_tables = stage_bytes <= size_t(kLdsPerCu - 1024) ? 1 : 0;
        ctx->i_lds = ctx->i_tables ? stage_bytes : 0;
        // two 512-thread blocks per CU when two tables fit in LDS (same 16
        // waves per CU; c3: fbs 31.3 -> 30.1 us, profiles/r01/v19_block_sweep.txt),
        // else one 1024-thread block
        ctx->i_block = (ctx->i_tables && 2 * stage_bytes <= size_t(kLdsPerCu - 1024)) ? 512 : 1024;
        const int i_wpb = ctx->i_block / kWave;
        int i_per_cu = std::max(1, kIterWavesPerCu / i_wpb);
        if (ctx->i_tables)
            i_per_cu = std::min<int>(i_per_cu, int(size_t(kLdsPerCu) / std::max<size_t>(stage_bytes, 1)));
        i_per_cu = std::max(1, i_per_cu);
        ctx->i_grid = int(std::max<int64_t>(1, std::min<int64_t>(int64_t(ctx->n_cu) * i_per_cu,
                                                                 (int64_t(G) + i_wpb - 1) / i_wpb)));
    }
    // Groups dealt to the per-iteration kernel's waves, longest first, each
    // to the least loaded wave (rows, plus the bubble work the kernel gives
    // the first waves -- small bubbles, one per lane -- and the last -- big
    // ones, one per wave; the big ones are estimated here from the counted
    // record sizes: a string whose bubbles average more than 8 edges has at
    // least one).  Each wave's groups are then laid out contiguously.
    const int i_wpb = ctx->i_block / kWave, i_nw = ctx->i_grid * i_wpb;
    std::vector<int32_t> order;
    std::vector<int32_t> wave_first(size_t(i_nw) + 1, 0);
    std::vector<double> load0(size_t(i_nw), 0.0);   // each wave's bubble work, in stream rows
    // groups (row counts in sorted order) to waves: longest first, each to the
    // least loaded wave; each wave's groups then lie contiguously
    // (scale: the bubble work in this format's rows -- the costs below are
    // in 16-bit rows)
    auto deal = [&](const std::vector<int32_t>& grows, std::vector<int32_t>& ord, std::vector<int32_t>& wf,
                    double scale) {
        using Item = std::pair<double, int32_t>;
        std::priority_queue<Item, std::vector<Item>, std::greater<Item>> heap;
        for (int w = 0; w < i_nw; ++w) heap.push({load0[size_t(w)] * scale, w});
        std::vector<std::vector<int32_t>> lists(static_cast<size_t>(i_nw));
        for (int32_t g = 0; g < G; ++g) {
            Item it = heap.top();
            heap.pop();
            lists[size_t(it.second)].push_back(g);
            it.first += grows[size_t(g)];
            heap.push(it);
        }
        ord.clear();
        ord.reserve(size_t(G));
        wf.assign(size_t(i_nw) + 1, 0);
        for (int w = 0; w < i_nw; ++w) {
            wf[size_t(w)] = int32_t(ord.size());
            ord.insert(ord.end(), lists[size_t(w)].begin(), lists[size_t(w)].end());
        }
        wf[size_t(i_nw)] = G;
    };
    {
        // costs in stream rows; small 18: the 16-20 optimum of the sweep after
        // the slot stores became coalesced (profiles/r02/v12_small_cost_sweep.txt:
        // fbs 24.6 -> 23.4 us at c3; it was 32 before, profiles/r01/v18_cost_sweep.txt)
        double small_cost = 18.0, big_cost = 8.0;
        int64_t n_b = 0, n_big_est = 0;
        for (int32_t i : comp) {
            n_b += h_nb[size_t(i)];
            if (h_nb[size_t(i)] > 0 && h_bub[size_t(i)] > wfsa::bubble_record_words(wfsa::kBubbleRegEdges) * h_nb[size_t(i)])
                ++n_big_est;
        }
        const int nblk = ctx->i_grid;
        const int small_wpb = small_waves_per_block(n_b - n_big_est, nblk);
        const int64_t small_waves = (n_b - n_big_est + kWave - 1) / kWave;
        // the in-kernel QN update's waves (wave i_wpb - 2 of the first
        // blocks; fb_kernels.hpp QnWave): about one per 48 parameters (a
        // batch holds at most 64 members), each charged qw_cost rows so its
        // stream share ends early
        // (reserved whatever WFSA_QN_INKERNEL says: the layout, and so every
        // fixed-order sum, is then the same with the update in or out)
        constexpr int64_t per_qw = 48;   // parameters per QN wave (40 / 36 / 32: no gain, profiles/r05)
        ctx->qw_waves = (i_wpb >= 3 && delta_want && ctx->i_tables)
                            ? int(std::min<int64_t>({nblk, int64_t(wfsa::kQnMaxWaves),
                                                     (int64_t(ctx->n_params) + per_qw - 1) / per_qw})) : 0;
        for (int w = 0; w < i_nw; ++w) {
            const int bid = w / i_wpb, wib = w % i_wpb;
            if (bid == 0 && wib == i_wpb - 1) {   // the QN finish's wave (fbs_kernel): no groups
                load0[size_t(w)] = 1e300;
                continue;
            }
            if (wib == i_wpb - 2 && bid < ctx->qw_waves) load0[size_t(w)] += ctx->qw_cost;
            if (wib < small_wpb && int64_t(wib) * nblk + bid < small_waves) load0[size_t(w)] += small_cost;   // (fbs_kernel's chunk order)
            const int64_t r = wfsa::big_rank(bid, wib, nblk, i_wpb, ctx->qw_waves);
            if (r < n_big_est) load0[size_t(w)] += big_cost;
        }
        deal(rows0, order, wave_first, 1.0);
    }
    std::vector<int64_t> g_base(size_t(G) + 1, 0), s_base(SZ, 0), b_base(SZ, 0);
    std::vector<int32_t> g_len(size_t(std::max(G, 1)), 0), l_str(size_t(G) * kWave, -1), l_len(size_t(G) * kWave, 0);
    std::vector<int32_t> b_first(SZ, 0);
    int64_t chunks = 0, words = 0;
    for (int32_t g = 0; g < G; ++g) {
        const int32_t src = order[size_t(g)];   // the group in sorted order
        g_base[size_t(g)] = chunks;
        g_len[size_t(g)] = rows0[size_t(src)];
        for (int l = 0; l < kWave; ++l) {
            const int64_t k = int64_t(g) * kWave + l, ks = int64_t(src) * kWave + l;
            if (ks >= nc) break;
            const int32_t str = comp[size_t(ks)];
            l_str[size_t(k)] = str;
            l_len[size_t(k)] = h_main[size_t(str)];
            s_base[size_t(str)] = (chunks + l) * per;
            words += h_main[size_t(str)];
        }
        chunks += int64_t(kWave) * g_len[size_t(g)];
    }
    g_base[size_t(G)] = chunks;
    int64_t bwords = 0, nbub = 0;
    for (int32_t str : comp) {
        b_base[size_t(str)] = bwords;
        b_first[size_t(str)] = int32_t(nbub);
        bwords += h_bub[size_t(str)];
        nbub += h_nb[size_t(str)];
    }
    ctx->h_bfirst = b_first;
    ctx->h_nbub = h_nb;
    if (bwords >= (int64_t(1) << 31) - 2) return fail(WFSA_ERR_CAPACITY, "bubble buffer exceeds 2^31 words");

    // 3. emit the streams (same tier as counted)
    const size_t chunk_alloc = size_t(chunks) + size_t(wfsa::kStreamTailChunks);
    HIP_TRY(ctx->stream_w.alloc(chunk_alloc));
    HIP_TRY(hipMemsetAsync(ctx->stream_w.ptr, 0xff, chunk_alloc * sizeof(uint4), s));
    HIP_TRY(ctx->bub.alloc(size_t(bwords) + size_t(wfsa::kBubbleSlackWords)));
    HIP_TRY(hipMemsetAsync(ctx->bub.ptr, 0, (size_t(bwords) + size_t(wfsa::kBubbleSlackWords)) * sizeof(int32_t), s));
    HIP_TRY(ctx->bub_off.alloc(size_t(std::max<int64_t>(nbub, 1))));
    if (nc > 0) {
        DevBuf<int64_t> d_sb, d_bb;
        DevBuf<int32_t> d_bf;
        HIP_TRY(d_sb.upload(s_base.data(), size_t(S), s));
        HIP_TRY(d_bb.upload(b_base.data(), size_t(S), s));
        HIP_TRY(d_bf.upload(b_first.data(), size_t(S), s));
        std::vector<int32_t> el[2];
        for (int32_t str : comp) el[std::min<int>(tier[size_t(str)], 1)].push_back(str);
        DevBuf<int32_t> d_el[2];
        for (int t = 0; t < 2; ++t) {
            if (el[t].empty()) continue;
            HIP_TRY(d_el[t].upload(el[t].data(), el[t].size(), s));
            wfsa::TravArgs a = trav_args(ctx, t);
            a.list = d_el[t].ptr;
            a.n_list = int32_t(el[t].size());
            a.stream = ctx->stream_w.ptr;
            a.wide = ctx->wide;
            a.s_base = d_sb.ptr;
            a.bub = ctx->bub.ptr;
            a.b_base = d_bb.ptr;
            a.b_first = d_bf.ptr;
            a.bub_off = ctx->bub_off.ptr;
            HIP_TRY(wfsa::launch_trav(wfsa::MODE_EMIT, a, trav_grid(ctx->cfg[t], ctx->n_cu, int64_t(el[t].size())), s));
        }
        HIP_TRY(hipStreamSynchronize(s));
    }
    HIP_TRY(ctx->g_base.upload(g_base.data(), size_t(G) + 1, s));
    HIP_TRY(ctx->g_len.upload(g_len.data(), g_len.size(), s));
    HIP_TRY(ctx->l_str.upload(l_str.data(), l_str.size(), s));
    HIP_TRY(ctx->l_len.upload(l_len.data(), l_len.size(), s));
    HIP_TRY(ctx->wave_first.upload(wave_first.data(), wave_first.size(), s));
    // bubbles: small ones into the structure-of-arrays tables, big ones kept
    // as records; every (bubble edge, parameter) pair gets a slot in the
    // parameter-major contribution array (layout_slots)
    ctx->n_bubbles = int32_t(nbub);
    ctx->n_small4 = ctx->n_small = ctx->n_big = 0;
    if (nbub > 0) {
        std::vector<int32_t> h_bubbuf(static_cast<size_t>(bwords)), h_off(static_cast<size_t>(nbub));
        HIP_TRY(ctx->bub.download(h_bubbuf.data(), size_t(bwords), s));
        HIP_TRY(ctx->bub_off.download(h_off.data(), size_t(nbub), s));
        HIP_TRY(hipStreamSynchronize(s));
        auto edge_code_at = [&](int32_t o, int e) { return h_bubbuf[size_t(o) + 4 + 2 * size_t(e)]; };
        std::vector<int32_t> small4, small, big;
        ctx->max_bub_nodes = 1;
        for (int32_t o : h_off) {
            const int hdr = h_bubbuf[size_t(o)];
            const int nodes = hdr & 0xffff, edges = hdr >> 16;
            ctx->max_bub_nodes = std::max(ctx->max_bub_nodes, nodes);
            bool sm = edges <= wfsa::kBubbleRegEdges && nodes <= wfsa::kBubbleRegNodes;
            for (int e = 0; sm && e < edges; ++e) sm = edge_code_at(o, e) >= 0;
            (!sm ? big : (edges <= 4 && nodes <= 4 ? small4 : small)).push_back(o);
        }
        // same-shaped bubbles (equal edge codes and structure) next to each
        // other: the lanes of a wave then take the same branches and write a
        // parameter's consecutive contribution slots (layout_slots)
        auto shape_less = [&](int32_t x, int32_t y) {
            const int ex = h_bubbuf[size_t(x)] >> 16, ey = h_bubbuf[size_t(y)] >> 16;
            if (h_bubbuf[size_t(x)] != h_bubbuf[size_t(y)]) return h_bubbuf[size_t(x)] < h_bubbuf[size_t(y)];
            for (int k = 0; k < 2 * std::min(ex, ey); ++k)
                if (h_bubbuf[size_t(x) + 4 + size_t(k)] != h_bubbuf[size_t(y) + 4 + size_t(k)])
                    return h_bubbuf[size_t(x) + 4 + size_t(k)] < h_bubbuf[size_t(y) + 4 + size_t(k)];
            return false;
        };
        std::stable_sort(small4.begin(), small4.end(), shape_less);
        std::stable_sort(small.begin(), small.end(), shape_less);
        {   // list position of every bubble (the fused rmin values are stored there)
            std::unordered_map<int32_t, int32_t> idx_of;
            idx_of.reserve(h_off.size());
            for (size_t i = 0; i < h_off.size(); ++i) idx_of[h_off[i]] = int32_t(i);
            std::vector<int32_t> bpos(h_off.size(), 0);
            int32_t pos = 0;
            for (const auto* list : {&small4, &small, &big})
                for (int32_t o : *list) bpos[size_t(idx_of.at(o))] = pos++;
            HIP_TRY(ctx->rm_bpos.upload(bpos.data(), bpos.size(), s));
            HIP_TRY(ctx->rm_sv.alloc(bpos.size()));
            HIP_TRY(hipStreamSynchronize(s));
            ctx->h_bpos = std::move(bpos);
        }
        ctx->h_bubbuf = std::move(h_bubbuf);
        ctx->h_sm4_list = std::move(small4);
        ctx->h_sm_list = std::move(small);
        ctx->h_big_list = std::move(big);
        ctx->n_small4 = int32_t(ctx->h_sm4_list.size());
        ctx->n_small = int32_t(ctx->h_sm_list.size());
        ctx->n_big = int32_t(ctx->h_big_list.size());
        ctx->big_lds_edges = 2;
        for (int32_t o : ctx->h_big_list) ctx->big_lds_edges = std::max(ctx->big_lds_edges, (ctx->h_bubbuf[size_t(o)] >> 16) + 1);
        ctx->big_lds_edges &= ~1;   // even
        ctx->b_waves = wfsa::bubble_waves(ctx->n_small4, ctx->n_small, ctx->n_big);
        HIP_TRY(hipStreamSynchronize(s));
    } else {
        ctx->b_waves = 0;
        ctx->h_bubbuf.clear();
        ctx->h_sm4_list.clear();
        ctx->h_sm_list.clear();
        ctx->h_big_list.clear();
    }
    // the delta deal's bubble charges from the classified bubbles, in delta
    // rows: fitted to the waves' measured stream-phase ends (the experiments
    // build's deal fit: end = c0 + c1 rows + a charge per kind of extra work)
    // and then swept round-robin on one box (profiles/r05/dealer_fit.txt):
    // class A 9, class B 17, big 13, the QN wave 6 -- c3 29.6 -> 28.1 us per
    // step against the earlier 18 / 36 / 8 / 8; big 15 after the QN batches
    // were capped at 48 chunks (the refit's 15.0 rows; -0.3 us per step,
    // profiles/r05/option_sweeps.txt)
    constexpr double kChargeA = 9.0, kChargeB = 17.0, kChargeBig = 15.0;
    {
        const double small_cost = kChargeA, small_cost_b = kChargeB, big_cost = kChargeBig;
        const int nblk = ctx->i_grid;
        const int64_t nch = wfsa::small_chunks(ctx->n_small4, ctx->n_small), na = (int64_t(ctx->n_small4) + kWave - 1) / kWave;
        const int small_wpb = small_waves_per_block(nch * kWave, nblk);
        for (int w = 0; w < i_nw; ++w) {
            const int bid = w / i_wpb, wib = w % i_wpb;
            if (bid == 0 && wib == i_wpb - 1) continue;   // the finish wave (charged 1e300 above)
            double c = 0.0;
            if (wib == i_wpb - 2 && bid < ctx->qw_waves) c += ctx->qw_cost;
            const int64_t ch = int64_t(wib) * nblk + bid;   // fbs_kernel's chunk of this wave (wfsa::small_entry)
            if (wib < small_wpb && ch < nch) c += ch >= na ? small_cost_b : small_cost;
            const int64_t r = wfsa::big_rank(bid, wib, nblk, i_wpb, ctx->qw_waves);
            if (r < ctx->n_big) c += big_cost;
            load0[size_t(w)] = c;
        }
    }
    {   // the group headers: p of each lane's string and the group's rows
        std::vector<double> h_p(S > 0 ? size_t(S) : 1, 0.0), pl(std::max<size_t>(l_str.size(), 1), 0.0);
        if (S > 0) HIP_TRY(ctx->p.download(h_p.data(), size_t(S), s));
        HIP_TRY(hipStreamSynchronize(s));
        for (size_t k = 0; k < l_str.size(); ++k)
            if (l_str[k] >= 0) pl[k] = h_p[size_t(l_str[k])];
        DevBuf<double> d_pl;
        HIP_TRY(d_pl.upload(pl.data(), pl.size(), s));
        HIP_TRY(wfsa::launch_stream_headers(ctx->stream_w.ptr, ctx->g_base.ptr, ctx->g_len.ptr, d_pl.ptr, G,
                                            ctx->wide, s));
        HIP_TRY(hipStreamSynchronize(s));
        ctx->delta_on = false;
        ctx->d_tab = 0;
        if (delta_want && ctx->i_tables)
            if (int rc = build_delta(ctx, comp, h_main, s_base, h_p, chunks, G, rows0, deal)) return rc;
        // The one-launch step's critical path is the last bubble arrival, a
        // go line and a QN batch; the two-kernel step's is the stream's end, a
        // launch and the QN kernel.  So the one launch pays when the stream
        // covers the bubble tail: the deal's mean stream rows per wave against
        // the heaviest bubble wave's charge, at the ratio where c3's family
        // crosses over (750k strings: 12.9 rows, two kernels 1.6 us faster;
        // 1M: 17.2 rows, one launch 2.6 us faster; profiles/r06/xrank.txt)
        const double heaviest = ctx->n_small > 0 ? kChargeB : ctx->n_big > 0 ? kChargeBig : ctx->n_small4 > 0 ? kChargeA : 0.0;
        ctx->qw_cover = !ctx->delta_on || ctx->qw_mean_rows >= 15.0 / kChargeB * heaviest;
    }
    ctx->n_groups = G;
    ctx->n_compiled = nc;

    {   // slot layout: the QN loop's trimmed order when it is set up, else the identity
        std::vector<int32_t> order = ctx->slot_order;
        if (order.size() != size_t(ctx->n_params)) {
            order.resize(size_t(ctx->n_params));
            for (int32_t j = 0; j < ctx->n_params; ++j) order[size_t(j)] = j;
        }
        if (int rc = layout_slots(ctx, order)) return rc;
    }

    // the preparation-time gradient pass: one wavefront per block (its
    // accumulation is then deterministic), the gradient in LDS when it fits
    // (else each block's own slab in HBM); the slabs are summed in order
    const size_t table_bytes = size_t(ctx->n_params) * sizeof(double);
    ctx->c_tables = table_bytes <= size_t(kLdsPerCu - 1024) ? 1 : 0;
    ctx->c_lds = ctx->c_tables ? table_bytes : 0;
    {
        const int per_cu = ctx->c_tables ? std::max(1, std::min<int>(8, int(size_t(kLdsPerCu) / std::max<size_t>(table_bytes, 1))))
                                         : 2;
        ctx->c_grid = int(std::max<int64_t>(1, std::min<int64_t>(int64_t(ctx->n_cu) * per_cu, G)));
    }
    HIP_TRY(ctx->gpart.alloc(size_t(ctx->c_grid) * size_t(std::max(ctx->n_params, 1))));
    HIP_TRY(ctx->fixed_grad.alloc(size_t(std::max(ctx->n_params, 1))));

    // traversal fallback lists
    ctx->h_tier.assign(size_t(ctx->n_strings), int8_t(-1));
    for (int t = 0; t < 3; ++t) for (int32_t i : fb[t]) ctx->h_tier[size_t(i)] = int8_t(t);
    for (int t = 0; t < 3; ++t) {
        ctx->n_fall[t] = int32_t(fb[t].size());
        ctx->fall_grid[t] = fb[t].empty() ? 0
                            : (t == 2 ? wide_grid(ctx, int64_t(fb[t].size()))
                                      : trav_grid(ctx->cfg[t], ctx->n_cu, int64_t(fb[t].size())));
        if (!fb[t].empty()) HIP_TRY(ctx->fall[t].upload(fb[t].data(), fb[t].size(), s));
    }
    ctx->w2_grid = 0;
    ctx->w2_n = 0;
    std::vector<int32_t> w2l = fb[2];
    if (ctx->w2_all) {
        w2l.insert(w2l.end(), fb[0].begin(), fb[0].end());
        w2l.insert(w2l.end(), fb[1].begin(), fb[1].end());
    }
    // the wave kernel's fixed-point gradient holds a block's partial in 64
    // bits with at least 20 fraction bits (below): longer strings than that
    // bound allows stay on the fp64 tiers
    int32_t fix_pe = 1;
    for (size_t g = 0; g + 1 < ctx->h_pptr.size(); ++g) fix_pe = std::max(fix_pe, ctx->h_pptr[g + 1] - ctx->h_pptr[g]);
    const double fix_bound = (double(ctx->max_len) + 2.0) * double(fix_pe);
    if (!w2l.empty() && ctx->use_wide2 && ctx->has_pairs && fix_bound <= std::ldexp(1.0, 63 - 20) &&
        wide2_config(ctx)) {   // wave per string, a block per CU
        {   // longest first: the waves take strings from a counter, the short ones fill the tail
            std::vector<int64_t> off(size_t(S) + 1);
            HIP_TRY(ctx->off.download(off.data(), off.size(), s));
            HIP_TRY(hipStreamSynchronize(s));
            {   // the pass's work, for the roofline: alpha entries and pair-list edges per evaluation
                std::vector<uint8_t> sy(static_cast<size_t>(off[size_t(S)]));
                std::vector<int32_t> bid(256), pn(size_t(ctx->pt_K) + 1), ep(size_t(int64_t(ctx->pt_K + 1) * ctx->pt_K) + 1);
                HIP_TRY(ctx->sym.download(sy.data(), sy.size(), s));
                HIP_TRY(ctx->pt_bidx.download(bid.data(), 256, s));
                HIP_TRY(ctx->pt_n.download(pn.data(), pn.size(), s));
                HIP_TRY(ctx->pt_eptr.download(ep.data(), ep.size(), s));
                HIP_TRY(hipStreamSynchronize(s));
                int64_t rows = 0, edges = 0;
                const int K = ctx->pt_K;
                for (int32_t i : w2l) {
                    int a = K;
                    for (int64_t q = off[size_t(i)]; q < off[size_t(i) + 1]; ++q) {
                        const int b = bid[sy[size_t(q)]];
                        if (b < 0) break;
                        rows += pn[size_t(b)];
                        edges += ep[size_t(a * K + b) + 1] - ep[size_t(a * K + b)];
                        a = b;
                    }
                }
                ctx->stats.wave_row_entries = rows;
                ctx->stats.wave_pair_edges = edges;
            }
            std::stable_sort(w2l.begin(), w2l.end(), [&](int32_t x, int32_t y) {
                return off[size_t(x) + 1] - off[size_t(x)] > off[size_t(y) + 1] - off[size_t(y)];
            });
            HIP_TRY(ctx->w2_list.upload(w2l.data(), w2l.size(), s));
            ctx->w2_n = int32_t(w2l.size());
        }
        const int wpb = ctx->w2_waves;
        ctx->w2_stride = wfsa::wide2_stride(ctx->max_len, ctx->pt_max_n, ctx->pl_items);
        const int64_t budget = (int64_t(16) << 30) / 8;   // 16 GiB of alpha rows at most
        int64_t g = std::min<int64_t>(ctx->n_cu, (int64_t(w2l.size()) + wpb - 1) / wpb);
        g = std::min<int64_t>(g, budget / (int64_t(wpb) * ctx->w2_stride));
        ctx->w2_grid = int(std::max<int64_t>(g, 1));
        const size_t n2 = size_t(ctx->w2_grid) * wpb * size_t(ctx->w2_stride);
        HIP_TRY(ctx->w2_scratch.alloc(n2));
        HIP_TRY(ctx->w2_ctr.alloc(2));
        HIP_TRY(hipMemsetAsync(ctx->w2_ctr.ptr, 0, 2 * sizeof(unsigned), s));
        // fixed-point gradient: a parameter's sum over strings is at most
        // (max_len + 2) x (parameters per edge) in magnitude (sum p = 1; every
        // position's edge and the end weight, each parameter once per
        // occurrence), so a block's partial fits a signed 64-bit word with
        // the rest as fraction (c3-like max_len 128: 2^-54)
        ctx->w2_fix_frac = std::max(20, std::min(60, 63 - int(std::ceil(std::log2(fix_bound)))));
        const size_t nfix = 2 * size_t(std::max(ctx->n_params, 1)) + 3;
        HIP_TRY(ctx->w2_fix.alloc(nfix));
        HIP_TRY(hipMemsetAsync(ctx->w2_fix.ptr, 0, nfix * sizeof(unsigned long long), s));
    }
    const size_t waves = std::max(size_t(ctx->c_grid), size_t(ctx->i_grid) * size_t(ctx->i_block / kWave)) +
                         size_t(ctx->b_waves) +
                         size_t(ctx->fall_grid[0]) * size_t(ctx->cfg[0].waves_per_block) +
                         size_t(ctx->fall_grid[1]) * size_t(ctx->cfg[1].waves_per_block) +
                         size_t(std::max(ctx->fall_grid[2], ctx->w2_grid));
    // two halves: a device-resident QN step's finish reads its partials
    // while the next step writes the other half
    HIP_TRY(ctx->ll_part.alloc(2 * waves));
    ctx->ll_stride = waves;
    ctx->ll_cur = ctx->ll_part.ptr;
    HIP_TRY(hipStreamSynchronize(s));

    // the trivial words' gradient, once: compiled pass with gradient at
    // w = 0 (its log-weights are discarded), then the slab sum
    if (nc > 0) {
        HIP_TRY(hipMemsetAsync(ctx->w_full.ptr, 0, (size_t(ctx->n_params) + 2) * sizeof(double), s));
        if (int rc = enqueue_compiled(ctx, true, false)) return rc;
        HIP_TRY(hipMemcpyAsync(ctx->fixed_grad.ptr, ctx->out.ptr + 1, size_t(ctx->n_params) * sizeof(double),
                               hipMemcpyDeviceToDevice, s));
        // with a communicator the constant part is summed over the ranks once
        // here; the per-step all-reduce then carries only what varies
        if (ctx->comm && ctx->n_params > 0)
            COMM_TRY(ctx, ctx->fixed_grad.ptr, size_t(ctx->n_params), wfsa::RedOp::SumF64, s);
    } else {
        HIP_TRY(hipMemsetAsync(ctx->fixed_grad.ptr, 0, size_t(std::max(ctx->n_params, 1)) * sizeof(double), s));
        if (ctx->comm && ctx->n_params > 0)   // (every rank joins the collective)
            COMM_TRY(ctx, ctx->fixed_grad.ptr, size_t(ctx->n_params), wfsa::RedOp::SumF64, s);
    }
    HIP_TRY(hipStreamSynchronize(s));

    ctx->stats.compiled_strings = nc;
    ctx->stats.fallback_strings = int64_t(fb[0].size() + fb[1].size() + fb[2].size());
    ctx->stats.tier2_strings = ctx->tier2_strings;
    ctx->stats.wave_strings = ctx->w2_grid > 0 ? ctx->w2_n : 0;
    ctx->stats.wave_pull = ctx->w2_grid > 0 && ctx->w2_pull ? ctx->pl_items : 0;
    if (ctx->w2_grid == 0) ctx->stats.wave_row_entries = ctx->stats.wave_pair_edges = 0;
    ctx->stats.stream_words = words;
    ctx->stats.stream_bytes = ctx->delta_on ? ctx->d_stream_bytes : chunks * 16;   // what the per-iteration pass reads
    ctx->stats.n_bubbles = nbub;
    ctx->stats.bubble_words = bwords;
    ctx->stats.tier1_strings = n_tier1;
    ctx->stats.waves_per_block = ctx->cfg[0].waves_per_block;
    ctx->stats.prepare_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    ctx->prep_level = 2;
    ++ctx->prep_gen;
    return WFSA_OK;
}

// The compiled-stream kernel over the weights in w_full, preceded by the
// edge-weight kernel unless the kernel folds that into its prologue (it does
// when it stages w in LDS).  with_grad: the preparation-time gradient pass
// (followed by its slab reduction into out); else the per-iteration pass.
int enqueue_compiled(wfsa_dev* ctx, bool with_grad, bool want_logq, const unsigned* halted, int slot) {
    hipStream_t s = ctx->stream;
    const int32_t np = ctx->n_params;
    const int tables = with_grad ? ctx->c_tables : ctx->i_tables;
    const bool fused = ctx->n_groups > 0 && tables >= 1;
    if (!fused)
        HIP_TRY(wfsa::launch_edge_weights(ctx->w_full.ptr, ctx->pptr.ptr, ctx->pidx.ptr, ctx->lw.ptr, ctx->ew.ptr,
                                          ctx->erec.ptr, ctx->n_edges + ctx->n_end, ctx->out.ptr, int64_t(np) + 1, s));
    // the stream kernel's timing: events attached to its dispatch (start and
    // end of the kernel itself), else recorded around it
    const bool ktimed = !with_grad && ctx->kernel_timing && slot >= 0;
    if (ktimed && ctx->n_groups == 0) HIP_TRY(record(ctx, ctx->k0, slot, s));
    if (ctx->n_groups > 0) {
        wfsa::CompiledArgs c{};
        c.m = model_view(ctx);
        c.p = ctx->p.ptr;
        stream_args(ctx, c, !with_grad);
        c.n_params = np;
        c.tables = tables;
        c.with_grad = with_grad ? 1 : 0;
        c.multi = ctx->n_multi > 0 ? 1 : 0;
        c.w = ctx->w_cur ? ctx->w_cur : ctx->w_full.ptr;
        c.grad = ctx->out.ptr + 1;
        c.gpart = ctx->gpart.ptr;
        c.n_comb = ctx->n_edges + ctx->n_end;
        c.lw_out = ctx->lw.ptr;
        c.ew_out = ctx->ew.ptr;
        c.erec_out = ctx->erec.ptr;
        c.out = ctx->out.ptr;
        c.no_slice = (!with_grad && ctx->eval_no_slice) ? 1 : 0;
        c.ll_part = ctx->ll_cur;
        c.logq = want_logq ? ctx->logq.ptr : nullptr;
        c.halted = halted;
        if (!with_grad) {   // a pending QN finish rides in block 0 (consumed)
            c.fin = ctx->fin_for_fbs;
            ctx->fin_for_fbs.active = 0;
            if (c.fin.active && ctx->fin_for_fbs_px) {   // across ranks: this launch's exchange
                c.fin.px = ctx->cur_px;
                c.fin.px_slot = 0;
            }
        }
        size_t lds = with_grad ? ctx->c_lds : ctx->i_lds;
        if (!with_grad && bubbles_fused(ctx, want_logq)) {
            c.bub = bubble_args(ctx, false, halted, nullptr);
            if (c.bub.rmin_acc) {
                c.bub.rmin_sv = ctx->rm_sv.ptr;
                ctx->rm_sv_used = true;
            }
            c.bub_on = 1;
            c.bub.small_wpb = small_waves_per_block(wfsa::small_chunks(ctx->n_small4, ctx->n_small) * kWave, ctx->i_grid);
            c.bub.qw_waves = ctx->qw_waves;
            if (ctx->n_big > 0) {
                c.bub.big_lds_edges = ctx->big_lds_edges;
                c.bub.big_lds_off = int32_t(big_stage_off(ctx));
                lds = big_stage_off(ctx) + size_t(ctx->i_block / kWave) * size_t(wfsa::big_stage_bytes(ctx->big_lds_edges));
            }
        }
#ifdef WFSA_EXPERIMENTS
        if (!with_grad && std::getenv("WFSA_FBS_TRACE")) {   // per-wave stamps (fb_kernels.hip WFSA_STAMP)
            const size_t nw = size_t(ctx->i_grid) * size_t(ctx->i_block / kWave) * 16;
            HIP_TRY(ctx->fbs_trace.alloc(nw));
            HIP_TRY(hipMemsetAsync(ctx->fbs_trace.ptr, 0, nw * sizeof(unsigned long long), ctx->stream));
            c.trace = ctx->fbs_trace.ptr;
        }
#endif
        if (!with_grad && ctx->qw_next.on) {   // this step's QN update rides in this launch
            c.qw = ctx->qw_next;
            ctx->qw_next.on = 0;
            c.bub.wt = 1;   // the QN waves read the slots in this launch
            if (ctx->rm_bpart_cur) {   // ... and the rmin column (RminFold)
                c.rf.bk = ctx->rm_bk.ptr;
                c.rf.mpos = ctx->rm_mpos.ptr;
                c.rf.cnt = ctx->rm_cnt.ptr;
                c.rf.trav = ctx->rm_trav.ptr;
                c.rf.n_trav = ctx->rm_n_trav;
                c.rf.rmin_log = ctx->rm_rs.ptr;
                c.rf.part = ctx->rm_bpart_cur;
                ctx->rm_bpart_cur = nullptr;
            }
        }
        if (with_grad && tables == 0)   // the blocks accumulate into their slabs
            HIP_TRY(hipMemsetAsync(ctx->gpart.ptr, 0, size_t(ctx->c_grid) * size_t(np) * sizeof(double), s));
        if (with_grad) HIP_TRY(wfsa::launch_compiled(c, ctx->c_grid, kGradBlock, lds, s));
        else HIP_TRY(wfsa::launch_compiled(c, ctx->i_grid, ctx->i_block, lds, s, ktimed ? ctx->k0[slot] : nullptr,
                                           ktimed ? ctx->kc[slot] : nullptr));
    }
    if (ktimed && ctx->n_groups == 0) HIP_TRY(record(ctx, ctx->kc, slot, s));
    if (with_grad) {
        if (ctx->n_groups > 0) HIP_TRY(wfsa::launch_slab_sum(ctx->gpart.ptr, ctx->c_grid, np, ctx->out.ptr, s));
        else HIP_TRY(hipMemsetAsync(ctx->out.ptr, 0, (size_t(np) + 1) * sizeof(double), s));
    }
    return WFSA_OK;
}

// The device work of one objective/gradient evaluation, enqueued on the
// context's stream (captured into a graph on first use): weights in, the
// compiled streams (with the per-edge weights) + bubbles (timed by k0..k1),
// traversal fallback (k1..k2), the tail reduction (which adds the trivial
// words' constant gradient), and -- without a communicator -- the results out.
wfsa::BubbleArgs bubble_args(wfsa_dev* ctx, bool want_logq, const unsigned* halted, double* ll_part) {
    wfsa::BubbleArgs b{};
    b.m = model_view(ctx);
    b.rmin_acc = ctx->rm_eval ? ctx->rm_rs.ptr : nullptr;
    b.sm4_tbl = ctx->sm4_tbl.ptr;
    b.n_small4 = ctx->n_small4;
    b.sm_tbl = ctx->sm_tbl.ptr;
    b.n_small = ctx->n_small;
    b.bub = ctx->bub.ptr;
    b.big_off = ctx->big_off.ptr;
    b.n_big = ctx->n_big;
    b.big_edge_base = ctx->big_edge_base.ptr;
    b.big_eslot_ptr = ctx->big_eslot_ptr.ptr;
    b.big_eslot = ctx->big_eslot.ptr;
    b.contrib = ctx->contrib.ptr;
    b.w = ctx->w_cur ? ctx->w_cur : ctx->w_full.ptr;
    b.ewp = ctx->ewp_cur ? ctx->ewp_cur : ctx->ewp.ptr;
    b.ll_part = ll_part;
    b.logq = want_logq ? ctx->logq.ptr : nullptr;
    b.halted = halted;
    static const int dbg = experiment_knob("WFSA_BUB_DBG");
    b.dbg = dbg;
    return b;
}

int enqueue_bubbles(wfsa_dev* ctx, bool want_logq, const unsigned* halted, int32_t wave_off, hipStream_t s) {
    wfsa::BubbleArgs b = bubble_args(ctx, want_logq, halted, ctx->ll_cur + wave_off);
    if (b.rmin_acc) {   // the rmin values per bubble, as the fused form stores them
        b.rmin_sv = ctx->rm_sv.ptr;
        ctx->rm_sv_used = true;
    }
    HIP_TRY(wfsa::launch_bubbles(b, s));
    return WFSA_OK;
}

// The bubbles ride in the stream kernel's waves when the kernel stages the
// weights (and log q is not wanted: both would write the strings' entries).
bool bubbles_fused(wfsa_dev* ctx, bool want_logq) {
    if (!(ctx->n_bubbles > 0 && !want_logq && ctx->n_groups > 0 && ctx->i_tables >= 1))
        return false;
    // at most one chunk of 64 small bubbles per wave; the big bubbles' staging must fit beside w
    // (the last wave of block 0 is the QN finish's: no bubbles)
    if (ctx->i_block / kWave < 2 ||
        small_waves_per_block(wfsa::small_chunks(ctx->n_small4, ctx->n_small) * kWave, ctx->i_grid) > ctx->i_block / kWave - 1)
        return false;
    return ctx->n_big == 0 || big_stage_off(ctx) + size_t(ctx->i_block / kWave) *
                                                       size_t(wfsa::big_stage_bytes(ctx->big_lds_edges)) <=
                                  size_t(kLdsPerCu - 1024);
}

// The evaluation kernels; with_tail: finish out = [LL, grad_full] with the
// reduction kernel -- adding the constant trivial-word gradient unless a
// communicator is attached (its all-reduced copy is added after the
// all-reduce) -- else the consumer (the fused QN step) sums the bubble slots,
// adds fixed_grad and sums ll_part[0, *n_ll).
wfsa::ReduceArgs reduce_args(wfsa_dev* ctx, const unsigned* halted, int32_t n_ll) {
    wfsa::ReduceArgs r{};
    r.contrib = ctx->n_bubbles > 0 ? ctx->contrib.ptr : nullptr;
    r.grp_base = ctx->grp_base.ptr;
    r.seg_ptr = ctx->seg_ptr.ptr;
    r.chunk_ptr = ctx->chunk_ptr.ptr;
    r.param_at = ctx->param_at.ptr;
    r.tile_ptr = ctx->tile_ptr.ptr;
    r.n_tiles = ctx->n_tiles;
    r.fixed = (ctx->n_groups > 0 && !ctx->comm) ? ctx->fixed_grad.ptr : nullptr;
    r.ll_part = ctx->ll_cur;
    r.n_ll = n_ll;
    r.out = ctx->out.ptr;
    r.halted = halted;
    return r;
}

// The traversal strings (strings that do not compile): the tier kernels in
// weighted mode, gradient into out[1..] (zeroed and the per-edge weights
// written before them), ll partials from slot wave_off on (advanced past
// theirs).
bool has_traversal(const wfsa_dev* ctx) {
    return ctx->n_fall[0] + ctx->n_fall[1] + ctx->n_fall[2] > 0 || (ctx->w2_grid > 0 && ctx->w2_all);
}
int32_t trav_ll_waves(const wfsa_dev* ctx) {   // the ll partial slots enqueue_traversal fills
    const bool w2_covers_01 = ctx->w2_grid > 0 && ctx->w2_all;
    int32_t n = 0;
    for (int t = 0; t < 2 && !w2_covers_01; ++t)
        if (ctx->n_fall[t]) n += ctx->fall_grid[t] * ctx->cfg[t].waves_per_block;
    if (ctx->n_fall[2] || w2_covers_01) n += ctx->w2_grid > 0 ? ctx->w2_grid : ctx->fall_grid[2];
    return n;
}
int enqueue_traversal(wfsa_dev* ctx, bool want_logq, const unsigned* halted, int32_t& wave_off) {
    hipStream_t s = ctx->stream;
    const bool w2_covers_01 = ctx->w2_grid > 0 && ctx->w2_all;
    for (int t = 0; t < 2 && !w2_covers_01; ++t) {
        if (!ctx->n_fall[t]) continue;
        wfsa::TravArgs a = trav_args(ctx, t);
        a.list = ctx->fall[t].ptr;
        a.n_list = ctx->n_fall[t];
        a.grad = ctx->out.ptr + 1;
        a.ll_part = ctx->ll_cur + wave_off;
        a.logq = want_logq ? ctx->logq.ptr : nullptr;
        a.halted = halted;
        a.rmin_log = ctx->rm_eval ? ctx->rm_rs.ptr : nullptr;
        HIP_TRY(wfsa::launch_trav(wfsa::MODE_WEIGHTED, a, ctx->fall_grid[t], s));
        wave_off += ctx->fall_grid[t] * ctx->cfg[t].waves_per_block;
    }
    if (ctx->n_fall[2] || w2_covers_01) {
        wfsa::WideArgs a = wide_args(ctx);
        a.list = ctx->fall[2].ptr;
        a.n_list = ctx->n_fall[2];
        a.grad = ctx->out.ptr + 1;
        a.ll_part = ctx->ll_cur + wave_off;
        a.logq = want_logq ? ctx->logq.ptr : nullptr;
        a.halted = halted;
        a.rmin_log = ctx->rm_eval ? ctx->rm_rs.ptr : nullptr;
        if (ctx->w2_grid > 0) {
            a.list = ctx->w2_list.ptr;
            a.n_list = ctx->w2_n;
            a.grad_lds = ctx->w2_lgrad ? 1 : 0;
            static const int w2dbg = experiment_knob("WFSA_W2_DBG");
            a.dbg = w2dbg;
            if (ctx->w2_pull) {
                HIP_TRY(wfsa::launch_pull_weights(ctx->pl_g.ptr, ctx->pl_nf + ctx->pl_nb, ctx->pl_nf, ctx->ew.ptr,
                                                  ctx->lw.ptr, ctx->pl_w.ptr, ctx->pl_w.ptr + ctx->pl_nf + ctx->pl_nb, s));
                const size_t lds = wfsa::pull_lds(ctx->n_params, ctx->w2_lgrad, ctx->w2_waves, ctx->pt_max_n);
                HIP_TRY(wfsa::launch_wave_pull(a, ctx->w2_grid, ctx->w2_waves, lds, s));
            } else {
                HIP_TRY(wfsa::launch_pair_weights(ctx->pt_ent.ptr, ctx->pt_ne, ctx->ew.ptr, ctx->lw.ptr, ctx->pt_w.ptr, s));
                const size_t lds = wfsa::wide2_lds(ctx->n_params, ctx->w2_lgrad, ctx->w2_waves, ctx->pt_max_n);
                HIP_TRY(wfsa::launch_wide2(a, ctx->w2_grid, ctx->w2_waves, lds, s));
            }
            wave_off += ctx->w2_grid;
        } else {
            HIP_TRY(wfsa::launch_wide(false, a, ctx->fall_grid[2], s));
            wave_off += ctx->fall_grid[2];
        }
    }
    return WFSA_OK;
}

int enqueue_evaluation(wfsa_dev* ctx, bool want_logq, const unsigned* halted, int slot, bool with_tail = true,
                       int32_t* n_ll = nullptr) {
    hipStream_t s = ctx->stream;
    if (ctx->mpath) {   // matrix-file mode: out is complete when it returns
        HIP_TRY(record(ctx, ctx->k0, slot, s));
        HIP_TRY(ctx->mpath->enqueue(ctx->w_full.ptr, ctx->out.ptr, want_logq ? ctx->logq.ptr : nullptr, halted, s));
        HIP_TRY(record(ctx, ctx->kc, slot, s));
        HIP_TRY(record(ctx, ctx->k2, slot, s));
        if (n_ll) *n_ll = 0;
        return WFSA_OK;
    }
    if (ctx->dense) {   // fp64 MFMA path: out is complete when it returns
        HIP_TRY(record(ctx, ctx->k0, slot, s));
        HIP_TRY(ctx->dense->enqueue(ctx->ewp.ptr, false, ctx->out.ptr, want_logq ? ctx->logq.ptr : nullptr, halted, s));
        HIP_TRY(record(ctx, ctx->kc, slot, s));
        HIP_TRY(record(ctx, ctx->k2, slot, s));
        if (n_ll) *n_ll = 0;
        return WFSA_OK;
    }
    // (a bubble kernel on a second stream beside the stream kernel: the
    // cross-stream fork / join cost more idle time, 5-20 us, than the
    // overlap saved -- measured and removed)
    ctx->rm_sv_used = false;   // (set by the stream kernel's launch when it stores the bubbles' rmin values)
    const bool fusedb = bubbles_fused(ctx, want_logq);
    const bool trav = has_traversal(ctx);
    // the ll partials: the stream kernel's blocks, then the bubble kernel's
    // waves, then the traversal kernels' -- the same slots whatever order the
    // kernels run in (the finish sums them in slot order)
    int32_t wave_off = ctx->n_groups > 0 ? ctx->i_grid : 0;   // one per stream-kernel block
    const int32_t trav_off = wave_off + ((ctx->n_bubbles > 0 && !fusedb) ? ctx->b_waves : 0);
    // With this step's QN update in the stream kernel, the traversal strings
    // run first: their gradient (in out, which the QN waves then read) and
    // log-likelihood partials are complete at the stream kernel's start.
    // The per-edge weights and the zeroed result they need come from the
    // edge-weights kernel (the stream kernel's own slice of them would be
    // too late).
    const bool trav_first = trav && ctx->qw_next.on;
    if (trav_first) {
        HIP_TRY(wfsa::launch_edge_weights(ctx->w_cur ? ctx->w_cur : ctx->w_full.ptr, ctx->pptr.ptr, ctx->pidx.ptr,
                                          ctx->lw.ptr, ctx->ew.ptr, ctx->erec.ptr, ctx->n_edges + ctx->n_end,
                                          ctx->out.ptr, int64_t(ctx->n_params) + 1, s));
        int32_t off = trav_off;
        if (int rc = enqueue_traversal(ctx, want_logq, halted, off)) return rc;
    }
    // the per-edge weights and the zeroed result are for the traversal
    // kernels and the reduction: the fused QN step over compiled strings
    // alone reads neither, so the stream kernel skips writing them (and with
    // the traversal strings first it must: out holds their gradient)
    ctx->eval_no_slice = !with_tail && (!trav || trav_first);
    // the QN update in the stream kernel reads the bubble slots: a separate
    // bubble kernel then runs before it (its slots visible at the boundary)
    const bool bub_first = ctx->qw_next.on && ctx->n_bubbles > 0 && !fusedb;
    if (bub_first)
        if (int rc = enqueue_bubbles(ctx, want_logq, halted, wave_off, s)) return rc;
    const int crc = enqueue_compiled(ctx, false, want_logq, halted, slot);
    ctx->eval_no_slice = false;
    if (crc) return crc;
    if (ctx->n_bubbles > 0 && !fusedb && !bub_first) {
        if (int rc = enqueue_bubbles(ctx, want_logq, halted, wave_off, s)) return rc;
    }
    wave_off = trav_off;
    if (trav_first) wave_off += trav_ll_waves(ctx);
    else if (int rc = enqueue_traversal(ctx, want_logq, halted, wave_off)) return rc;
    if (n_ll) *n_ll = wave_off;
    if (!with_tail) {
        const bool after_kc = (ctx->n_bubbles > 0 && !fusedb && !bub_first) || (trav && !trav_first);
        if (!after_kc && slot >= 0) ctx->k2_kc[slot] = true;
        else HIP_TRY(record(ctx, ctx->k2, slot, s));
        return WFSA_OK;
    }
    HIP_TRY(wfsa::launch_reduce(reduce_args(ctx, halted, wave_off), s));
    HIP_TRY(record(ctx, ctx->k2, slot, s));
    return WFSA_OK;
}

// Across ranks, once per prepared corpus: the combine's key pair and every
// rank's string count -> this rank's first global string index.
int rmin_rank_base(wfsa_dev* ctx) {
    hipStream_t s = ctx->stream;
    HIP_TRY(ctx->rm_key.alloc(2));
    if (ctx->comm) {
        const int nr = ctx->comm->nranks();
        std::vector<double> cnt(size_t(nr), 0.0);
        cnt[size_t(ctx->comm->rank())] = double(ctx->n_strings);
        DevBuf<double> t;
        HIP_TRY(t.upload(cnt.data(), cnt.size(), s));
        COMM_TRY(ctx, t.ptr, cnt.size(), wfsa::RedOp::SumF64, s);
        HIP_TRY(t.download(cnt.data(), cnt.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
        ctx->rm_base = 0.0;
        for (int r = 0; r < ctx->comm->rank(); ++r) ctx->rm_base += cnt[size_t(r)];
    }
    return WFSA_OK;
}

// The rmin column at the weights of the evaluation just enqueued (w_full,
// ewp and the per-edge weights on the device): bubbles, then the traversal
// tiers in min mode, then the reduction into res[0..1].
int rmin_prepare(wfsa_dev* ctx) {
    hipStream_t s = ctx->stream;
    const size_t S = size_t(std::max<int64_t>(ctx->n_strings, 1));
    if (ctx->rm_gen != ctx->prep_gen) {   // once per prepared corpus: the ambiguous strings
        std::vector<double> pc(S);
        HIP_TRY(ctx->pcount.download(pc.data(), size_t(ctx->n_strings), s));
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<int4> amb;
        for (int64_t i = 0; i < ctx->n_strings; ++i) {
            if (!(pc[size_t(i)] > 1.5)) continue;
            const bool comp = ctx->h_tier[size_t(i)] < 0;
            amb.push_back(make_int4(int32_t(i), comp ? ctx->h_bfirst[size_t(i)] : 0, comp ? ctx->h_nbub[size_t(i)] : -1, 0));
        }
        ctx->rm_n_amb = int64_t(amb.size());
        if (!amb.empty()) HIP_TRY(ctx->rm_amb.upload(amb.data(), amb.size(), s));
        {   // the folded form's tables (RminFold): per bubble position its string's bubble count and
            // run; each multi-bubble string's positions in bubble order; the traversal strings
            const size_t nb = size_t(std::max(ctx->n_bubbles, 1));
            std::vector<int2> bk(nb, make_int2(0, 0));
            std::vector<int32_t> mpos, trav;
            for (const int4& e : amb) {
                if (e.z < 0) {
                    trav.push_back(e.x);
                    continue;
                }
                const int32_t run = e.z > 1 ? int32_t(mpos.size()) : 0;
                for (int32_t j = 0; j < e.z; ++j) {
                    const int32_t pos = ctx->h_bpos.at(size_t(e.y + j));
                    bk[size_t(pos)] = make_int2(e.z, run);
                    if (e.z > 1) mpos.push_back(pos);
                }
            }
            const int32_t n_trav = int32_t(trav.size());
            if (mpos.empty()) mpos.push_back(0);
            if (trav.empty()) trav.push_back(0);
            HIP_TRY(ctx->rm_bk.upload(bk.data(), bk.size(), s));
            HIP_TRY(ctx->rm_mpos.upload(mpos.data(), mpos.size(), s));
            HIP_TRY(ctx->rm_cnt.alloc(mpos.size()));
            HIP_TRY(hipMemsetAsync(ctx->rm_cnt.ptr, 0, mpos.size() * sizeof(unsigned), s));
            HIP_TRY(ctx->rm_trav.upload(trav.data(), trav.size(), s));
            ctx->rm_n_trav = n_trav;
            HIP_TRY(ctx->rm_bpart.alloc(4 * size_t(std::max(ctx->i_grid, 1))));
        }
        HIP_TRY(ctx->rm_part.alloc(4 * size_t(wfsa::rmin_blocks(ctx->rm_n_amb))));   // two halves (QN parity)
        HIP_TRY(ctx->rm_rs.alloc(S));
        HIP_TRY(hipMemsetAsync(ctx->rm_rs.ptr, 0, S * sizeof(double), s));   // fused accumulation starts at 0
        HIP_TRY(ctx->rm_vb.alloc(size_t(std::max(ctx->n_bubbles, 1))));
        if (int rc = rmin_rank_base(ctx)) return rc;
        HIP_TRY(hipStreamSynchronize(s));   // amb is freed on return
        ctx->rm_gen = ctx->prep_gen;
    }
    return WFSA_OK;
}

// trav_done: the evaluation just enqueued already produced every string's
// value (ctx->rm_eval: its weighted traversal passes ran the min forward and
// its bubble passes accumulated log(min path / Z) per string)
// across ranks: res -> the global (rmin, string index); every rank calls it
int combine_rmin(wfsa_dev* ctx, double* res, hipStream_t s) {
    if (!ctx->comm) return WFSA_OK;
    double* key = ctx->rm_key.ptr;
    HIP_TRY(wfsa::launch_rmin_rank(res, key, ctx->rm_base, 0, s));
    COMM_TRY(ctx, key, 1, wfsa::RedOp::MinF64, s);
    HIP_TRY(wfsa::launch_rmin_rank(res, key, ctx->rm_base, 1, s));
    COMM_TRY(ctx, key + 1, 1, wfsa::RedOp::MinF64, s);
    HIP_TRY(wfsa::launch_rmin_rank(res, key, ctx->rm_base, 2, s));
    return WFSA_OK;
}

int enqueue_rmin(wfsa_dev* ctx, const unsigned* halted, double* res, int par = 0, wfsa::QnFinish* q = nullptr,
                 bool trav_done = false, wfsa::QnArgs* fold = nullptr) {
    hipStream_t s = ctx->stream;
    if (ctx->mpath) {
        HIP_TRY(ctx->mpath->enqueue_rmin(res, halted, s));
        return WFSA_OK;
    }
    if (ctx->dense) {   // the (min, +) trellis over the evaluation's row slots (dense_path.hip)
        if (ctx->rm_gen != ctx->prep_gen) {
            if (int rc = rmin_rank_base(ctx)) return rc;
            ctx->rm_gen = ctx->prep_gen;
        }
        HIP_TRY(ctx->dense->enqueue_rmin(res, halted, s));
        return WFSA_OK;
    }
    if (int rc = rmin_prepare(ctx)) return rc;
    for (int t = 0; t < 2 && !trav_done; ++t) {
        if (!ctx->n_fall[t]) continue;
        wfsa::TravArgs a = trav_args(ctx, t);
        a.list = ctx->fall[t].ptr;
        a.n_list = ctx->n_fall[t];
        a.rmin_log = ctx->rm_rs.ptr;
        a.halted = halted;
        HIP_TRY(wfsa::launch_trav(wfsa::MODE_MIN, a, ctx->fall_grid[t], s));
    }
    if (ctx->n_fall[2] && !trav_done) {
        wfsa::WideArgs a = wide_args(ctx);
        a.list = ctx->fall[2].ptr;
        a.n_list = ctx->n_fall[2];
        a.rmin_log = ctx->rm_rs.ptr;
        a.halted = halted;
        HIP_TRY(wfsa::launch_wide(false, a, ctx->fall_grid[2], s, true));
    }
    wfsa::RminArgs r{};
    r.m = model_view(ctx);
    r.bub = ctx->bub.ptr;
    r.bub_off = ctx->bub_off.ptr;
    r.n_bub = ctx->n_bubbles;
    r.max_nodes = ctx->max_bub_nodes;
    r.vb = trav_done ? nullptr : ctx->rm_vb.ptr;   // fused: the evaluation accumulated the bubbles
    if (trav_done && ctx->rm_sv_used) {            // ... or stored them per bubble
        r.sv = ctx->rm_sv.ptr;
        r.bpos = ctx->rm_bpos.ptr;
    }
    r.w = ctx->w_full.ptr;
    r.ewp = ctx->ewp.ptr;
    r.rmin_log = ctx->rm_rs.ptr;
    r.amb = ctx->rm_amb.ptr;
    r.n_amb = ctx->rm_n_amb;
    const int nb = wfsa::rmin_blocks(ctx->rm_n_amb);
    r.part = ctx->rm_part.ptr + size_t(par) * 2 * size_t(nb);
    r.res = res;
    r.halted = halted;
    if (fold && q && trav_done && !r.vb) {   // the strings pass rides in the QN step kernel's blocks
        fold->rm = r;
        fold->rm_on = 1;
        fold->rm_blocks = wfsa::rmin_blocks(ctx->rm_n_amb);
    } else {
        HIP_TRY(wfsa::launch_rmin(r, s, q == nullptr));
    }
    if (q) {   // the step's finish reduces the block minima (one launch fewer per step)
        q->rmin_part = r.part;
        q->rmin_n_part = nb;
    }
    return WFSA_OK;
}

// One objective/gradient evaluation for the host: weights staged from the
// host-mapped buffer, the evaluation, and -- without a communicator -- the
// results published (with one, _begin all-reduces first).
int enqueue_iteration(wfsa_dev* ctx, bool want_logq) {
    hipStream_t s = ctx->stream;
    const int32_t np = ctx->n_params;
    HIP_TRY(wfsa::launch_stage(ctx->pinned_dev + weights_off(np), ctx->w_full.ptr, ctx->ewp.ptr, np, s));
    if (int rc = enqueue_evaluation(ctx, want_logq, nullptr, 0)) return rc;
    if (!ctx->comm) HIP_TRY(wfsa::launch_publish(ctx->out.ptr, publish_args(ctx), s));
    return WFSA_OK;
}

// One device-resident QuasiNewton step e: the evaluation at the device's
// w_full, then -- fused (one rank, bubbles laid out in trimmed order) -- the
// QN step kernel that completes the members' gradients itself, or the
// reduction, the all-reduce (communicator) and the QN step kernel.  The QN
// kernel's last block publishes the step's info row (ring slot e % depth).
int flush_qn_finish(wfsa_dev* ctx);

// The in-kernel QN update's batches (fb_kernels.hpp QnWave): runs of
// consecutive constraints of at most kQnWaveMembers members and
// 64 * kQnWaveChunkRounds slot chunks (their chunks are consecutive in the
// contribution array: constraint c's group follows c - 1's).  qw_ok = false
// when a constraint alone exceeds either, or has no member.
int build_qw_batches(wfsa_dev* ctx) {
    const int64_t key = ctx->qn_setup_gen * 1000003 + ctx->layout_gen;
    if (ctx->qw_key == key) return WFSA_OK;
    ctx->qw_key = key;
    ctx->qw_ok = false;
    ctx->qw_nbatch = 0;
    const int32_t n = ctx->qn_n, k = ctx->qn_k;
    const std::vector<int32_t>& cptr = ctx->h_cptr;
    // a batch's chunks are spread 8 lanes each, 8 per round: the target cap
    // bounds a QN wave's rounds (48: six; c3 -0.3 us/step against 256,
    // profiles/r05/option_sweeps.txt), raised to the largest constraint's
    // chunks when one alone needs more (then the hard limit, 256, decides)
    constexpr int32_t target = 48;   // (40 / 32 chunks: +0.2 us)
    const int32_t limit = kWave * wfsa::kQnWaveChunkRounds;
    constexpr int32_t mcap = wfsa::kQnWaveMembers;   // members per batch (45 / 36: 31.9-32.7 us)
    if (!ctx->qn_fused || k <= 0 || n <= 0 || int64_t(cptr.size()) != int64_t(k) + 1 ||
        int64_t(ctx->h_mchunk.size()) < n || ctx->slot_order.size() != size_t(ctx->n_params))
        return WFSA_OK;
    auto chunks = [&](int32_t c0, int32_t c1) {   // this rank's slot chunks of constraints [c0, c1)
        int64_t t = 0;
        for (int32_t i = cptr[size_t(c0)]; i < cptr[size_t(c1)]; ++i) t += ctx->h_mnch[size_t(i)];
        return t;
    };
    // Across ranks the batches are the same on every rank (the in-kernel
    // exchange pairs batch b with batch b): their bounds come from each
    // constraint's largest chunk count over the ranks, each rank's batch then
    // holds its own chunks.  The counts travel as a sum of every rank's row
    // (rank r fills row r) -- the peer path's sum, with its wait limit -- when
    // the rows fit a peer slot, else as a Min of the negated counts
    std::vector<double> gch(static_cast<size_t>(k));
    for (int32_t c = 0; c < k; ++c) gch[size_t(c)] = double(chunks(c, c + 1));
    if (ctx->comm) {
        const int nr = ctx->comm->nranks(), me = ctx->comm->rank();
        if (size_t(k) * size_t(nr) <= wfsa::kPeerCap) {
            std::vector<double> rows(size_t(k) * size_t(nr), 0.0);
            std::copy(gch.begin(), gch.end(), rows.begin() + std::ptrdiff_t(size_t(me) * size_t(k)));
            HIP_TRY(ctx->qw_gch.upload(rows.data(), rows.size(), ctx->stream));
            COMM_TRY(ctx, ctx->qw_gch.ptr, rows.size(), wfsa::RedOp::SumF64, ctx->stream);
            HIP_TRY(ctx->qw_gch.download(rows.data(), rows.size(), ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            COMM_CHECK(ctx);
            for (int32_t c = 0; c < k; ++c)
                for (int r = 0; r < nr; ++r) gch[size_t(c)] = std::max(gch[size_t(c)], rows[size_t(r) * size_t(k) + size_t(c)]);
        } else {
            for (double& v : gch) v = -v;
            HIP_TRY(ctx->qw_gch.upload(gch.data(), gch.size(), ctx->stream));
            COMM_TRY(ctx, ctx->qw_gch.ptr, gch.size(), wfsa::RedOp::MinF64, ctx->stream);
            HIP_TRY(ctx->qw_gch.download(gch.data(), gch.size(), ctx->stream));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            for (double& v : gch) v = -v;
        }
    }
    auto gchunks = [&](int32_t c0, int32_t c1) {   // the batching's chunk count: the ranks' largest
        int64_t t = 0;
        for (int32_t c = c0; c < c1; ++c) t += int64_t(gch[size_t(c)]);
        return t;
    };
    int64_t widest = 0;
    for (int32_t c = 0; c < k; ++c) {
        const int32_t nm = cptr[size_t(c) + 1] - cptr[size_t(c)];
        const int64_t nc = gchunks(c, c + 1);
        if (nm < 1 || nm > wfsa::kQnWaveMembers || nc > limit) return WFSA_OK;
        widest = std::max(widest, nc);
    }
    const int64_t cap = std::min<int64_t>(limit, std::max<int64_t>(widest, target > 0 ? target : limit));
    std::vector<int4> batch;
    std::vector<int32_t> con_of(size_t(n), 0), mfirst(size_t(n), 0);
    for (int32_t c0 = 0; c0 < k;) {
        int32_t c1 = c0 + 1;
        int64_t gn = gchunks(c0, c1);
        while (c1 < k && cptr[size_t(c1) + 1] - cptr[size_t(c0)] <= mcap) {
            const int64_t more = gchunks(c1, c1 + 1);
            if (gn + more > cap) break;
            gn += more;
            ++c1;
        }
        const int64_t nch = chunks(c0, c1);   // (this rank's: at most gn)
        const int32_t m0 = cptr[size_t(c0)], m1 = cptr[size_t(c1)];
        const int64_t base = ctx->h_mchunk[size_t(m0)];
        int64_t q = 0;
        for (int32_t c = c0; c < c1; ++c)
            for (int32_t i = cptr[size_t(c)]; i < cptr[size_t(c) + 1]; ++i) {
                if (ctx->h_mnch[size_t(i)] > 0 && ctx->h_mchunk[size_t(i)] != base + q * wfsa::kSlotChunk)
                    return WFSA_OK;   // (never: the layout keeps a batch's chunks consecutive)
                con_of[size_t(i)] = c;
                mfirst[size_t(i)] = int32_t(q);
                q += ctx->h_mnch[size_t(i)];
            }
        batch.push_back(make_int4(c0, c1, m0, m1));
        batch.push_back(make_int4(int32_t(nch), int32_t(uint32_t(uint64_t(base))), int32_t(uint64_t(base) >> 32), 0));
        c0 = c1;
    }
    hipStream_t s = ctx->stream;
    HIP_TRY(ctx->qw_batch.upload(batch.data(), batch.size(), s));
    HIP_TRY(ctx->qw_con_of.upload(con_of.data(), con_of.size(), s));
    HIP_TRY(ctx->qw_mfirst.upload(mfirst.data(), mfirst.size(), s));
    HIP_TRY(ctx->qw_mnch.upload(ctx->h_mnch.data(), size_t(n), s));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->qw_nbatch = int32_t(batch.size() / 2);
    ctx->h_qw_batch = batch;
    ctx->qw_ok = true;
    return WFSA_OK;
}

// The QN update rides in the stream kernel (fb_kernels.hpp QnWave) when the
// compiled strings use the delta stream and the QN batches were built; the
// rmin column needs the bubbles fused into the stream kernel (RminFold);
// traversal strings run before the launch; across ranks the peer path must be
// on (PeerX) -- and every rank must agree (qn_run_impl)
//
// The QN waves wait for every block's arrival, so every block of the grid
// must be resident at once: the grid is checked against the CUs times the
// blocks one CU holds at the launch's actual LDS (the big-bubble staging
// included) -- else the update stays a kernel of its own.
size_t qn_launch_lds(wfsa_dev* ctx) {   // enqueue_compiled's LDS for the per-iteration launch (no log q)
    if (bubbles_fused(ctx, false) && ctx->n_big > 0)
        return big_stage_off(ctx) + size_t(ctx->i_block / kWave) * size_t(wfsa::big_stage_bytes(ctx->big_lds_edges));
    return ctx->i_lds;
}
bool qw_resident(wfsa_dev* ctx) {
    const size_t lds = qn_launch_lds(ctx);
    if (ctx->qw_res_lds != lds || ctx->qw_res_block != ctx->i_block) {
        ctx->qw_res_lds = lds;
        ctx->qw_res_block = ctx->i_block;
        ctx->qw_res_per_cu = wfsa::fbs_qn_blocks_per_cu(ctx->i_block, lds);
    }
    return int64_t(ctx->i_grid) <= int64_t(ctx->n_cu) * ctx->qw_res_per_cu;
}
bool qw_usable(wfsa_dev* ctx) {
    // (the rmin column rides along when the bubbles run in the stream kernel: RminFold)
    const bool rmin_ok = !ctx->qn_rmin || ctx->n_bubbles == 0 || bubbles_fused(ctx, false);
    // (across ranks: through the peer areas, PeerX -- the peer path on, the
    // batches within the areas' flags)
    const bool comm_ok = !ctx->comm || (std::strcmp(ctx->comm->peer_state(), "on") == 0 &&
                                        ctx->qw_nbatch <= wfsa::kPeerMaxQnBatches);
    return ctx->use_qw && (ctx->qw_cover || ctx->qw_force) && ctx->qw_ok && ctx->qw_waves > 0 && ctx->qn_fused &&
           comm_ok && !ctx->dense &&
           !ctx->mpath && rmin_ok && ctx->n_groups > 0 && ctx->delta_on && ctx->i_tables >= 1 &&
           ctx->fixed_t_on && ctx->qn_k > 0 &&
           ctx->i_block / kWave >= 3 && qw_resident(ctx);
}

int enqueue_qn_step(wfsa_dev* ctx, double eta, double tol, int64_t e, bool timed, bool inkern, bool last) {
    hipStream_t s = ctx->stream;
    const int32_t np = ctx->n_params;
    const int par = int(e & 1);
    const int slot = int(e % kQnDepth);
    bool self_fin = false;
    ctx->ll_cur = ctx->ll_part.ptr + size_t(par) * ctx->ll_stride;
    const bool trellis = !ctx->dense && !ctx->mpath;
    const bool fused = trellis && ctx->qn_fused && !ctx->comm;
    int32_t n_ll = 0;
    const bool fuse_rmin = ctx->qn_rmin && trellis;   // traversal strings' rmin inside their weighted passes
    if (fuse_rmin)
        if (int rc = rmin_prepare(ctx)) return rc;
    if (ctx->fin_pending) {   // the previous step's finish: in this step's stream kernel, or its own launch
        if (ctx->fin_hostable && trellis && ctx->n_groups > 0 && (!ctx->fin_next_px || inkern)) {
            ctx->fin_for_fbs = ctx->fin_next;
            ctx->fin_for_fbs_px = ctx->fin_next_px;
            ctx->fin_pending = false;
        } else if (int rc = flush_qn_finish(ctx)) {
            return rc;
        }
    }
    wfsa::QnArgs q{};
    wfsa::QnFinish& f = q.fin;
    q.out = ctx->out.ptr;
    q.use_out = !fused || ctx->n_fall[0] + ctx->n_fall[1] + ctx->n_fall[2] > 0;
    f.out0 = ctx->out.ptr;
    if (fused) {
        q.fixed = ctx->n_groups > 0 ? ctx->fixed_grad.ptr : nullptr;
        q.fixed_t = ctx->fixed_t_on ? ctx->fixed_t.ptr : nullptr;
        q.contrib = ctx->n_bubbles > 0 ? ctx->contrib.ptr : nullptr;
        q.grp_base = ctx->grp_base.ptr;   // constraint c = reduction group c
        q.grp_nch = ctx->grp_nch.ptr;
        q.seg_ptr = ctx->seg_ptr.ptr;
        q.chunk_ptr = ctx->chunk_ptr.ptr;
        f.ll_part = ctx->ll_cur;
    } else if (trellis && ctx->comm && ctx->n_groups > 0) {
        q.fixed = ctx->fixed_grad.ptr;   // all-reduced once at preparation
    }
    if (trellis && ctx->comm && inkern) {   // in-kernel across ranks: the local partials, summed over the
                                            // ranks by the finish's exchange
        f.ll_part = ctx->ll_cur;
        f.rm_base = double(ctx->rm_base);
    } else if (trellis && ctx->comm) {   // the step's log-likelihood for its finish, which then rides in the next stream kernel
        if (ctx->ll_stash.n < 2) HIP_TRY(ctx->ll_stash.alloc(2));
        q.ll_stash = ctx->ll_stash.ptr + par;
        f.ll_part = ctx->ll_stash.ptr + par;
        f.n_ll = 1;
    }
    q.n_full = np;
    q.n = ctx->qn_n;
    q.k = ctx->qn_k;
    q.full_of = ctx->qn_full_of.ptr;
    q.trim = ctx->qn_trim.ptr;
    q.cptr = ctx->qn_cptr.ptr;
    q.x = ctx->qn_x.ptr;
    q.lambda = ctx->qn_lambda.ptr;
    q.expx = ctx->qn_expx.ptr;
    q.grad = ctx->qn_grad.ptr;
    q.w_full = ctx->w_full.ptr;
    q.ewp = ctx->ewp.ptr;
    q.partial = ctx->qn_partial.ptr;
    q.eta = eta;
    q.exp_lambda = ctx->qn_exp_lambda;
    q.halted = ctx->qn_halted.ptr;
    q.seg_cap = ctx->qn_max_nm;
    q.chunk_cap = (fused && ctx->n_bubbles > 0) ? std::min(ctx->lead_grp_nch, wfsa::kMaxChunks) : 1;
    f.partial = ctx->qn_partial.ptr;
    f.n_blocks = std::max(ctx->qn_k, 1);
    f.k = ctx->qn_k;
    f.plogp = ctx->qn_plogp;
    f.tol = tol;
    f.ring_slot = slot;
    f.tag = ctx->seq + 1u;   // (qn_run increments ctx->seq once per enqueued step)
    f.halted = ctx->qn_halted.ptr;
    f.halt_pending = ctx->qn_halted.ptr + 1;
    f.seq = ctx->counters.ptr;
    f.host_flag = ctx->flag_dev;
    f.host_ring = ctx->qn_ring_dev;
    if (inkern) {   // the update in the stream kernel: step e reads the weights of parity e, writes parity e + 1
        ctx->w_cur = par ? ctx->w_full2.ptr : ctx->w_full.ptr;
        ctx->ewp_cur = par ? ctx->ewp2.ptr : ctx->ewp.ptr;
        wfsa::QnWave& w = ctx->qw_next;
        w = wfsa::QnWave{};
        w.on = 1;
        w.n_batches = ctx->qw_nbatch;
        w.n_waves = ctx->qw_waves;
        w.parity = int32_t(ctx->qw_seq & 1u);
        w.n_arrive = ctx->i_grid;
        w.batch = ctx->qw_batch.ptr;
        w.con_of = ctx->qw_con_of.ptr;
        w.mfirst = ctx->qw_mfirst.ptr;
        w.mnch = ctx->qw_mnch.ptr;
        w.cptr = ctx->qn_cptr.ptr;
        w.full_of = ctx->qn_full_of.ptr;
        w.fixed_t = ctx->fixed_t.ptr;
        w.out = has_traversal(ctx) ? ctx->out.ptr : nullptr;   // (their gradient, before this launch)
        w.contrib = ctx->n_bubbles > 0 ? ctx->contrib.ptr : nullptr;
        w.x = ctx->qn_x.ptr;
        w.lambda = ctx->qn_lambda.ptr;
        w.grad = ctx->qn_grad.ptr;
        w.w_next = par ? ctx->w_full.ptr : ctx->w_full2.ptr;
        w.ewp_next = par ? ctx->ewp.ptr : ctx->ewp2.ptr;
        w.partial = ctx->qn_partial.ptr;
        w.eta = eta;
        w.exp_lambda = ctx->qn_exp_lambda;
        w.arrive = ctx->qw_arrive.ptr;
        w.halted = ctx->qn_halted.ptr;
        w.done = ctx->qw_done.ptr;   // (every launch zeroes the other parity's counter)
        w.go = ctx->qw_go.ptr;
        w.poll_limit = ctx->qw_poll_limit;
        if (ctx->comm) {   // across ranks: this launch's exchanges (one sequence number)
            if (!ctx->comm->peer_exchange(w.px)) return fail(WFSA_ERR_RCCL, "the peer exchange is not available");
            ctx->cur_px = w.px;
        }
        w.poll_fault = ctx->qw_poll_fault ? 1 : 0;
        if (ctx->qn_rmin) {   // the rmin column folded into the launch: its block minima for the finish
            ctx->rm_bpart_cur = ctx->rm_bpart.ptr + size_t(par) * 2 * size_t(ctx->i_grid);
            f.rmin_part = ctx->rm_bpart_cur;
            f.rmin_n_part = ctx->i_grid;
        }
        w.fin = f;
        // the Run's last launch finishes its own step (its stream kernel's
        // blocks' ll partials), so its row needs no finish kernel of its own
        // after it (WFSA_QN_LAST_SELF=0: that kernel; every launch finishing
        // its own step put the finish's write-through reads on the critical
        // path, 36.2 vs 28.6 us, profiles/r05)
        self_fin = last && ctx->qw_last_self;
        if (self_fin) {
            w.self_finish = 1;
            w.fin.px = w.px;   // (across ranks: the exchange of a launch finishing its own step)
            w.fin.px_slot = 1;
            w.fin.ll_part = ctx->ll_cur;
            // the stream kernel's blocks, then (bubbles not fused: the bubble
            // kernel ran first) the bubble kernel's waves -- enqueue_evaluation's order
            w.fin.n_ll = ctx->i_grid + ((ctx->n_bubbles > 0 && !bubbles_fused(ctx, false)) ? ctx->b_waves : 0) +
                         trav_ll_waves(ctx);
        }
        ++ctx->qw_seq;
    }
    ctx->rm_eval = fuse_rmin;
    const int erc = enqueue_evaluation(ctx, false, ctx->qn_halted.ptr, timed ? slot : -1, !fused && !inkern && trellis,
                                       &n_ll);
    ctx->rm_eval = false;
    ctx->rm_bpart_cur = nullptr;
    if (erc) return erc;
    if (ctx->qw_next.on) return fail(WFSA_ERR_HIP, "the in-kernel QN update was not launched");
    if (fused || inkern) f.n_ll = n_ll;
    if (inkern && self_fin) {   // the step published its own row: no finish pending
        const int32_t want = ctx->i_grid + ((ctx->n_bubbles > 0 && !bubbles_fused(ctx, false)) ? ctx->b_waves : 0) +
                             trav_ll_waves(ctx);
        if (n_ll != want) return fail(WFSA_ERR_HIP, "self-finish: %d log-likelihood partials, not %d", n_ll, want);
        ctx->fin_pending = false;
        ctx->fin_next.active = 0;
        return WFSA_OK;
    }
    if (ctx->comm && !inkern) COMM_TRY(ctx, ctx->out.ptr, size_t(np) + 1, wfsa::RedOp::SumF64, s);
    if (ctx->qn_rmin && !inkern) {
        constexpr bool fold_rmin = true;   // the strings pass in the QN step kernel's blocks (one launch fewer)
        double* res = ctx->rm_res.ptr + 2 * par;
        if (ctx->mpath || (ctx->dense && !ctx->comm)) {
            if (int rc = enqueue_rmin(ctx, ctx->qn_halted.ptr, res)) return rc;
            f.rmin = res;
        } else if (ctx->comm) {   // the rank's minimum, then the global one
            if (int rc = enqueue_rmin(ctx, ctx->qn_halted.ptr, res, par, nullptr, true)) return rc;
            if (int rc = combine_rmin(ctx, res, s)) return rc;
            f.rmin = res;
        } else if (int rc = enqueue_rmin(ctx, ctx->qn_halted.ptr, res, par, &f, true, fold_rmin ? &q : nullptr)) {
            return rc;
        }
    }
    if (!inkern) HIP_TRY(wfsa::launch_qn_step(q, fused, s));
    // the finish reads the step's log-likelihood partials: it can ride in the
    // next step's stream kernel when those are not in `out` (which that
    // kernel zeroes); else it is launched when the next step is enqueued
    ctx->fin_next = f;
    ctx->fin_next.active = 1;
    ctx->fin_next_px = inkern && ctx->comm;   // (its exchange takes the sequence number of the launch it runs in)
    ctx->fin_pending = true;
    ctx->fin_hostable = (fused || (trellis && ctx->comm)) && ctx->n_groups > 0 && f.ll_part != nullptr;
    return WFSA_OK;
}

// the pending finish of the last enqueued QN step as its own launch
int flush_qn_finish(wfsa_dev* ctx) {
    if (!ctx->fin_pending) return WFSA_OK;
    ctx->fin_pending = false;
    if (ctx->fin_next_px) {   // across ranks: a sequence number of its own
        if (!ctx->comm || !ctx->comm->peer_exchange(ctx->fin_next.px))
            return fail(WFSA_ERR_RCCL, "the peer exchange is not available");
        ctx->fin_next.px_slot = 0;
    }
    HIP_TRY(wfsa::launch_qn_finish(ctx->fin_next, ctx->stream));
    return WFSA_OK;
}

void drop_graph(wfsa_dev* ctx) {
    if (ctx->graph_exec) (void)hipGraphExecDestroy(ctx->graph_exec);
    if (ctx->graph) (void)hipGraphDestroy(ctx->graph);
    ctx->graph_exec = nullptr;
    ctx->graph = nullptr;
    ctx->graph_failed = false;
}

// weights in / results out, sized by n_params
int alloc_param_buffers(wfsa_dev* ctx) {
    HIP_TRY(ctx->w_full.alloc(size_t(ctx->n_params) + 2));
    HIP_TRY(ctx->ewp.alloc(size_t(ctx->n_params) + 2));
    HIP_TRY(ctx->out.alloc(size_t(ctx->n_params) + 2));
    const size_t pinned_need = weights_off(ctx->n_params) + size_t(ctx->n_params) + 2;
    if (ctx->pinned_n < pinned_need) {
        if (ctx->pinned) (void)hipHostFree(ctx->pinned);
        ctx->pinned = nullptr;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->pinned), pinned_need * sizeof(double),
                              hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->pinned_dev), ctx->pinned, 0));
        ctx->pinned_n = pinned_need;
        std::memset(ctx->pinned, 0, pinned_need * sizeof(double));   // incl. the weights' zero slot
    }
    return WFSA_OK;
}

// the loaded corpus handed to the dense path (host copies from the device)
int dense_load_corpus(wfsa_dev* ctx, const uint8_t* sym, const int64_t* off, const double* p) {
    hipStream_t s = ctx->stream;
    const hipError_t e = ctx->dense->load_corpus(sym, off, p, ctx->n_strings, s);
    if (e != hipSuccess)
        return fail(WFSA_ERR_HIP, "dense path: corpus of %lld strings does not fit (%s)", (long long)ctx->n_strings,
                    hipGetErrorString(e));
    ctx->dense_struct = false;
    ctx->prep_level = 0;
    ctx->prep_gen++;   // (the rmin pass's rank base is per corpus)
    ctx->stats.dense_rows = ctx->dense->rows();
    ctx->stats.dense_steps = ctx->dense->steps();
    ctx->stats.dense_np = ctx->dense->np();
    ctx->stats.dense_blas = ctx->dense->engine();
    return WFSA_OK;
}

int load_dense_model(wfsa_dev* ctx, const wfsa::DenseModel& dm) {
    hipStream_t s = ctx->stream;
    auto d = std::make_unique<wfsa::DensePath>(ctx->n_cu);
    if (hipError_t e = d->load_model(dm, s); e != hipSuccess)
        return fail(WFSA_ERR_HIP, "dense path: model upload failed (%s)", hipGetErrorString(e));
    ctx->dense = std::move(d);
    ctx->n_params = dm.n_params;
    ctx->n_nodes = dm.n_states;
    ctx->n_edges = dm.n_transitions;
    ctx->n_end = 0;
    ctx->start = 0;
    ctx->n_groups = 0;
    ctx->n_bubbles = 0;
    ctx->n_fall[0] = ctx->n_fall[1] = ctx->n_fall[2] = 0;
    if (int rc = alloc_param_buffers(ctx)) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    ctx->has_model = true;
    ctx->stats.n_nodes = ctx->n_nodes;
    ctx->stats.n_edges = ctx->n_edges;
    ctx->stats.n_end_edges = 0;
    ctx->stats.dense = 1;
    ctx->prep_level = 0;
    if (!ctx->has_corpus) return WFSA_OK;
    const size_t S = size_t(ctx->n_strings);
    std::vector<int64_t> off(S + 1);
    std::vector<double> p(std::max<size_t>(S, 1));
    HIP_TRY(ctx->off.download(off.data(), S + 1, s));
    HIP_TRY(ctx->p.download(p.data(), S, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<uint8_t> sym(std::max<size_t>(size_t(off[S]), 1));
    HIP_TRY(ctx->sym.download(sym.data(), size_t(off[S]), s));
    HIP_TRY(hipStreamSynchronize(s));
    return dense_load_corpus(ctx, sym.data(), off.data(), p.data());
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
    HIP_TRY(wfsa::configure_kernels(kLdsPerCu));
    std::unique_ptr<wfsa_dev> ctx(new wfsa_dev());
    ctx->device = device;
    ctx->n_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : kNumCu;
    if (const char* e = std::getenv("WFSA_GRAPH")) ctx->use_graph = e[0] == '1';
    if (const char* e = std::getenv("WFSA_TIMING")) ctx->kernel_timing = e[0] != '0';
    if (const char* e = std::getenv("WFSA_DELTA")) ctx->use_delta = e[0] != '0';
    if (const char* e = std::getenv("WFSA_DENSE"); e && e[0]) ctx->dense_mode = e[0] == '0' ? 0 : 1;
    if (const char* e = std::getenv("WFSA_TIER2")) ctx->force_tier2 = e[0] == '1';
    if (const char* e = std::getenv("WFSA_WIDE2")) ctx->use_wide2 = e[0] != '0';
    if (const char* e = std::getenv("WFSA_PULL")) ctx->use_pull = e[0] != '0';
    if (const char* e = std::getenv("WFSA_QN_INKERNEL")) {   // (unset: by the cover rule; 1: whenever possible; 0: never)
        ctx->use_qw = e[0] != '0';
        ctx->qw_force = e[0] == '1';
    }
    // fault injection (tests/test_gpu_qn_inkernel.py): the first QN wave waits
    // for an arrival that never comes and gives up after a few polls
    if (const char* e = std::getenv("WFSA_FAULT_QN_POLL"); e && e[0] == '1') {
        ctx->qw_poll_fault = true;
        ctx->qw_poll_limit = 256;
    }
    if (const char* e = std::getenv("WFSA_QN_LAST_SELF")) ctx->qw_last_self = e[0] != '0';

    HIP_TRY(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&ctx->ev0));
    HIP_TRY(hipEventCreate(&ctx->ev1));
    for (int i = 0; i < kQnDepth; ++i)
        for (hipEvent_t* ev : {&ctx->k0[i], &ctx->kc[i], &ctx->k2[i]}) HIP_TRY(hipEventCreate(ev));
    HIP_TRY(ctx->live.alloc(1));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->flag), 64, hipHostMallocMapped | hipHostMallocCoherent));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->flag_dev), ctx->flag, 0));
    *ctx->flag = 0;
    HIP_TRY(ctx->counters.alloc(1));
    HIP_TRY(hipMemsetAsync(ctx->counters.ptr, 0, sizeof(unsigned), ctx->stream));
    HIP_TRY(ctx->qw_arrive.alloc(2));
    HIP_TRY(hipMemsetAsync(ctx->qw_arrive.ptr, 0, 2 * sizeof(unsigned), ctx->stream));
    constexpr size_t n_go = size_t(wfsa::kQnMaxWaves) * wfsa::kQnGoStride;
    HIP_TRY(ctx->qw_go.alloc(n_go));
    HIP_TRY(hipMemsetAsync(ctx->qw_go.ptr, 0, n_go * sizeof(unsigned), ctx->stream));
    HIP_TRY(ctx->qw_done.alloc(2));
    HIP_TRY(hipMemsetAsync(ctx->qw_done.ptr, 0, 2 * sizeof(unsigned), ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    *out = ctx.release();
    return WFSA_OK;
}

void wfsa_dev_destroy(wfsa_dev* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    drop_graph(ctx);
    ctx->comm.reset();
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->flag) (void)hipHostFree(ctx->flag);
    for (hipEvent_t ev : {ctx->ev0, ctx->ev1})
        if (ev) (void)hipEventDestroy(ev);
    for (int i = 0; i < kQnDepth; ++i)
        for (hipEvent_t ev : {ctx->k0[i], ctx->kc[i], ctx->k2[i]})
            if (ev) (void)hipEventDestroy(ev);
    if (ctx->qn_ring) (void)hipHostFree(ctx->qn_ring);
    if (ctx->qst) (void)hipHostFree(ctx->qst);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int wfsa_dev_load_model(wfsa_dev* ctx, const wfsa_model_desc* model) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!model) return fail(WFSA_ERR_ARG, "null model");
    drop_graph(ctx);
    ctx->slot_order.clear();   // (a QN set-up belongs to the previous model)
    ctx->slot_groups.clear();
    ctx->qn_fused = false;
    if (ctx->mpath) {   // leaving matrix-file mode: the corpus went with the matrices
        ctx->mpath.reset();
        ctx->has_corpus = false;
    }
    ctx->dense.reset();
    ctx->dense_struct = false;
    ctx->stats.dense = 0;
    ctx->stats.dense_rows = ctx->stats.dense_steps = ctx->stats.dense_np = 0;
    if (ctx->dense_mode != 0) {
        wfsa::DenseModel dm;
        if (wfsa::dense_model_build(*model, ctx->dense_mode == 1, dm).empty()) return load_dense_model(ctx, dm);
    }
    wfsa::TrellisModel tm;
    const std::string err = wfsa::compile_trellis_model(*model, tm);
    if (!err.empty()) return fail(WFSA_ERR_MODEL, "automaton rejected: %s", err.c_str());
    // combined edge space: [0, E) byte edges, [E, E+X) end edges
    const int64_t E = int64_t(tm.o_byte.size()), X = int64_t(tm.x_pptr.size()) - 1;
    std::vector<int32_t> pptr(tm.o_pptr);
    std::vector<int32_t> pidx(tm.o_pidx);
    const int32_t shift = int32_t(tm.o_pidx.size());
    for (int64_t x = 1; x <= X; ++x) pptr.push_back(tm.x_pptr[size_t(x)] + shift);
    pidx.insert(pidx.end(), tm.x_pidx.begin(), tm.x_pidx.end());
    hipStream_t s = ctx->stream;
    HIP_TRY(ctx->o_ptr.upload(tm.o_ptr.data(), tm.o_ptr.size(), s));
    HIP_TRY(ctx->o_byte.upload(tm.o_byte.data(), tm.o_byte.size(), s));
    HIP_TRY(ctx->o_dst.upload(tm.o_dst.data(), tm.o_dst.size(), s));
    HIP_TRY(ctx->x_ptr.upload(tm.x_ptr.data(), tm.x_ptr.size(), s));
    HIP_TRY(ctx->pptr.upload(pptr.data(), pptr.size(), s));
    HIP_TRY(ctx->pidx.upload(pidx.data(), pidx.size(), s));
    ctx->h_pptr = pptr;
    ctx->h_pidx = pidx;
    {
        std::vector<int32_t> mof(size_t(E + X), -1), medge;
        for (int64_t g = 0; g < E + X; ++g)
            if (pptr[size_t(g) + 1] - pptr[size_t(g)] >= 2) {
                mof[size_t(g)] = int32_t(medge.size());
                medge.push_back(int32_t(g));
            }
        ctx->n_multi = int32_t(medge.size());
        HIP_TRY(ctx->multi_of.upload(mof.data(), mof.size(), s));
        HIP_TRY(ctx->multi_edge.upload(medge.data(), medge.size(), s));
    }
    // narrow (16-bit) stream words unless parameters or multi edges overflow them
    ctx->wide = (tm.n_params >= 0x8000 || ctx->n_multi >= 0x7fff) ? 1 : 0;
    HIP_TRY(ctx->node_end_count.upload(tm.node_end_count.data(), tm.node_end_count.size(), s));
    {   // tier 2: for each byte c, every destination of a byte-c edge once, with its in-edges
        std::vector<std::vector<std::pair<int32_t, int32_t>>> by(256);   // (dst, edge)
        for (int32_t u = 0; u < tm.n_nodes; ++u)
            for (int32_t g = tm.o_ptr[size_t(u)]; g < tm.o_ptr[size_t(u) + 1]; ++g)
                by[tm.o_byte[size_t(g)]].push_back({tm.o_dst[size_t(g)], g});
        std::vector<int32_t> edge_src(static_cast<size_t>(E));
        for (int32_t u = 0; u < tm.n_nodes; ++u)
            for (int32_t g = tm.o_ptr[size_t(u)]; g < tm.o_ptr[size_t(u) + 1]; ++g) edge_src[size_t(g)] = u;
        std::vector<int32_t> cptr(257, 0), dst, eptr, esrc, eg;
        for (int c = 0; c < 256; ++c) {
            auto& v = by[size_t(c)];
            std::stable_sort(v.begin(), v.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
            for (size_t i = 0; i < v.size(); ++i) {
                if (i == 0 || v[i].first != v[i - 1].first) {
                    dst.push_back(v[i].first);
                    eptr.push_back(int32_t(esrc.size()));
                }
                esrc.push_back(edge_src[size_t(v[i].second)]);
                eg.push_back(v[i].second);
            }
            cptr[size_t(c) + 1] = int32_t(dst.size());
            v.clear();
            v.shrink_to_fit();
        }
        eptr.push_back(int32_t(esrc.size()));
        if (dst.empty()) dst.push_back(0);
        if (esrc.empty()) { esrc.push_back(0); eg.push_back(0); }
        HIP_TRY(ctx->w_cptr.upload(cptr.data(), cptr.size(), s));
        HIP_TRY(ctx->w_dst.upload(dst.data(), std::max<size_t>(dst.size(), 1), s));
        HIP_TRY(ctx->w_eptr.upload(eptr.data(), eptr.size(), s));
        HIP_TRY(ctx->w_esrc.upload(esrc.data(), std::max<size_t>(esrc.size(), 1), s));
        HIP_TRY(ctx->w_eg.upload(eg.data(), std::max<size_t>(eg.size(), 1), s));
        if (int rc = build_pair_tables(ctx, tm, cptr, dst, eptr, esrc, eg, pptr, pidx)) return rc;
        HIP_TRY(hipStreamSynchronize(s));
    }
    HIP_TRY(ctx->lw.alloc(size_t(E + X)));
    HIP_TRY(ctx->ew.alloc(size_t(E + X)));
    HIP_TRY(ctx->erec.alloc(size_t(E + X)));
    HIP_TRY(ctx->node_end.alloc(size_t(tm.n_nodes)));
    ctx->n_edges = E;
    ctx->n_end = X;
    ctx->n_params = tm.n_params;
    ctx->n_nodes = tm.n_nodes;
    ctx->start = tm.start;
    if (int rc = alloc_param_buffers(ctx)) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    ctx->h_tm = std::make_unique<wfsa::TrellisModel>(std::move(tm));
    ctx->has_model = true;
    ctx->stats.n_nodes = ctx->n_nodes;
    ctx->stats.n_edges = ctx->n_edges;
    ctx->stats.n_end_edges = ctx->n_end;
    ctx->prep_level = 0;
    if (ctx->has_corpus) return configure_tiers(ctx);
    return WFSA_OK;
}

int wfsa_dev_load_corpus(wfsa_dev* ctx, const uint8_t* sym, const int64_t* off, const double* p, int64_t n_strings) {
    if (int rc = check_ctx(ctx)) return rc;
    if (ctx->mpath) return fail(WFSA_ERR_ARG, "matrix-file mode has no automaton: load a model first");
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
    HIP_TRY(ctx->logq.alloc(size_t(std::max<int64_t>(n_strings, 1))));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->n_strings = n_strings;
    ctx->total_sym = total;
    ctx->max_len = int32_t(max_len);
    ctx->has_corpus = true;
    ctx->prep_level = 0;
    ctx->stats.n_strings = n_strings;
    ctx->stats.total_symbols = total;
    ctx->stats.max_len = int32_t(max_len);
    drop_graph(ctx);
    if (ctx->dense) return dense_load_corpus(ctx, sym, off, p);
    if (ctx->has_model) return configure_tiers(ctx);
    return WFSA_OK;
}

static int recognize_impl(wfsa_dev* ctx, uint8_t* recognized, double* path_count, uint8_t* used_param) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->has_model || !ctx->has_corpus) return fail(WFSA_ERR_ARG, "load a model and a corpus first");
    if (ctx->dense ? !ctx->dense_struct : ctx->prep_level < 1)
        if (int rc = prepare(ctx, 1)) return rc;
    hipStream_t s = ctx->stream;
    const size_t S = size_t(ctx->n_strings);
    if (ctx->comm && ctx->n_params > 0)
        COMM_TRY(ctx, ctx->used.ptr, size_t(ctx->n_params), wfsa::RedOp::MaxU8, s);
    if (recognized) HIP_TRY(ctx->recog.download(recognized, S, s));
    if (path_count) HIP_TRY(ctx->pcount.download(path_count, S, s));
    if (used_param) HIP_TRY(ctx->used.download(used_param, size_t(ctx->n_params), s));
    HIP_TRY(hipStreamSynchronize(s));
    return WFSA_OK;
}

int wfsa_dev_load_paths(wfsa_dev* ctx, int32_t n_params, int64_t n_paths, const int64_t* prow, const int32_t* pcol,
                        const double* pdata, int64_t n_strings, const int64_t* mrow, const int64_t* mcol,
                        const double* p) {
    if (int rc = check_ctx(ctx)) return rc;
    if (n_params < 0 || n_paths < 0 || n_strings < 0 || !prow || !mrow || (n_strings > 0 && !p))
        return fail(WFSA_ERR_ARG, "bad path matrices");
    if (prow[0] != 0 || mrow[0] != 0) return fail(WFSA_ERR_ARG, "CSR rows must start at 0");
    for (int64_t l = 0; l < n_paths; ++l)
        if (prow[l + 1] < prow[l]) return fail(WFSA_ERR_ARG, "P rows not ascending at %lld", (long long)l);
    for (int64_t k = 0; k < prow[n_paths]; ++k)
        if (pcol[k] < 0 || pcol[k] >= n_params)
            return fail(WFSA_ERR_ARG, "Size mismatch: more path indexes than parameters in the automaton!");
    for (int64_t i = 0; i < n_strings; ++i)
        if (mrow[i + 1] < mrow[i]) return fail(WFSA_ERR_ARG, "M rows not ascending at %lld", (long long)i);
    for (int64_t k = 0; k < mrow[n_strings]; ++k)
        if (mcol[k] < 0 || mcol[k] >= n_paths) return fail(WFSA_ERR_ARG, "M cols != P rows");
    if (n_strings >= (int64_t(1) << 31) - 1) return fail(WFSA_ERR_ARG, "too many strings for one device");
    drop_graph(ctx);
    ctx->dense.reset();
    ctx->dense_struct = false;
    hipStream_t s = ctx->stream;
    auto mp = std::make_unique<wfsa::MatrixPath>();
    if (hipError_t e = mp->load(n_params, n_paths, prow, pcol, pdata, n_strings, mrow, mcol, p, s); e != hipSuccess)
        return fail(WFSA_ERR_HIP, "matrix-file mode: upload failed (%s)", hipGetErrorString(e));
    ctx->n_params = n_params;
    ctx->n_nodes = ctx->n_edges = ctx->n_end = 0;
    ctx->n_groups = 0;
    ctx->n_bubbles = 0;
    ctx->n_fall[0] = ctx->n_fall[1] = ctx->n_fall[2] = 0;
    if (int rc = alloc_param_buffers(ctx)) return rc;
    const size_t SZ = size_t(std::max<int64_t>(n_strings, 1));
    std::vector<uint8_t> rec(SZ, 0);
    for (int64_t i = 0; i < n_strings; ++i) rec[size_t(i)] = mp->path_counts()[size_t(i)] > 0 ? 1 : 0;
    HIP_TRY(ctx->pcount.upload(mp->path_counts().data(), size_t(n_strings), s));
    HIP_TRY(ctx->recog.upload(rec.data(), SZ, s));
    HIP_TRY(ctx->used.upload(mp->used().data(), mp->used().size(), s));
    HIP_TRY(ctx->logq.alloc(SZ));
    HIP_TRY(hipStreamSynchronize(s));
    ctx->mpath = std::move(mp);
    ctx->n_strings = n_strings;
    ctx->total_sym = 0;
    ctx->max_len = 0;
    ctx->has_model = true;
    ctx->has_corpus = true;
    ctx->prep_level = 2;
    ctx->prep_gen++;
    ctx->stats = wfsa_dev_stats{};
    ctx->stats.n_strings = n_strings;
    return WFSA_OK;
}

int wfsa_dev_sym_factor(wfsa_dev* ctx, int64_t n, const double* a, int64_t inertia[3], double* log_abs_det,
                        int32_t* det_sign) {
    if (int rc = check_ctx(ctx)) return rc;
    if (n < 0 || (n > 0 && !a)) return fail(WFSA_ERR_ARG, "bad matrix");
    if (ctx->in_flight) return fail(WFSA_ERR_ARG, "an evaluation is in flight");
    if (!ctx->ldlt) ctx->ldlt = std::make_unique<wfsa::SymSolver>();
    wfsa::SymFactor f;
    if (const char* e = ctx->ldlt->factor(a, n, ctx->stream, &f)) return fail(WFSA_ERR_HIP, "sym_factor: %s", e);
    if (inertia) {
        inertia[0] = f.positive;
        inertia[1] = f.negative;
        inertia[2] = f.zero;
    }
    if (log_abs_det) *log_abs_det = f.log_abs_det;
    if (det_sign) *det_sign = f.det_sign;
    return WFSA_OK;
}

int wfsa_dev_sym_factor_coo(wfsa_dev* ctx, int64_t n, int64_t nnz, const int32_t* i, const int32_t* j,
                            const double* v, double* b, int64_t inertia[3], double* log_abs_det, int32_t* det_sign,
                            int32_t* method) {
    if (int rc = check_ctx(ctx)) return rc;
    if (n < 0 || nnz < 0 || (nnz > 0 && (!i || !j || !v))) return fail(WFSA_ERR_ARG, "bad matrix entries");
    if (ctx->in_flight) return fail(WFSA_ERR_ARG, "an evaluation is in flight");
    if (!ctx->ldlt) ctx->ldlt = std::make_unique<wfsa::SymSolver>();
    wfsa::SymFactor f;
    int m = 0;
    if (const char* e = ctx->ldlt->factor_coo(n, nnz, i, j, v, b, ctx->stream, &f, &m))
        return fail(WFSA_ERR_HIP, "sym_factor_coo: %s", e);
    if (inertia) {
        inertia[0] = f.positive;
        inertia[1] = f.negative;
        inertia[2] = f.zero;
    }
    if (log_abs_det) *log_abs_det = f.log_abs_det;
    if (det_sign) *det_sign = f.det_sign;
    if (method) *method = m;
    return WFSA_OK;
}

int wfsa_dev_sym_solve(wfsa_dev* ctx, double* b) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->ldlt) return fail(WFSA_ERR_ARG, "sym_solve: no factorisation");
    if (const char* e = ctx->ldlt->solve(b, ctx->stream)) return fail(WFSA_ERR_HIP, "sym_solve: %s", e);
    return WFSA_OK;
}

static int rmin_impl(wfsa_dev* ctx, double* rmin, int64_t* string_index) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->has_model || !ctx->has_corpus) return fail(WFSA_ERR_ARG, "load a model and a corpus first");
    if (ctx->in_flight) return fail(WFSA_ERR_ARG, "an evaluation is in flight");
    if (ctx->dense ? !ctx->dense->weighted() : ctx->prep_level < 2)
        return fail(WFSA_ERR_ARG, "rmin: evaluate the objective first");
    if (ctx->mpath && ctx->comm)   // its index is a path of this rank's matrices: no global counterpart
        return fail(WFSA_ERR_ARG, "rmin: matrix-file mode runs the rmin column on one rank only");
    if (ctx->rm_res.n < 4) HIP_TRY(ctx->rm_res.alloc(4));
    if (int rc = enqueue_rmin(ctx, nullptr, ctx->rm_res.ptr)) return rc;
    if (int rc = combine_rmin(ctx, ctx->rm_res.ptr, ctx->stream)) return rc;
    double h[2];
    HIP_TRY(ctx->rm_res.download(h, 2, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    if (rmin) *rmin = h[0];
    if (string_index) *string_index = int64_t(h[1]);
    return WFSA_OK;
}

int wfsa_dev_string_tiers(wfsa_dev* ctx, int8_t* tier) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->has_model || !ctx->has_corpus) return fail(WFSA_ERR_ARG, "load a model and a corpus first");
    if (!tier) return fail(WFSA_ERR_ARG, "null output");
    if (ctx->dense || ctx->mpath) {
        std::memset(tier, ctx->dense ? 3 : 4, size_t(ctx->n_strings));
        return WFSA_OK;
    }
    if (ctx->prep_level < 2)
        if (int rc = prepare(ctx, 2)) return rc;
    std::memcpy(tier, ctx->h_tier.data(), size_t(ctx->n_strings));
    return WFSA_OK;
}

static int objective_grad_begin_impl(wfsa_dev* ctx, const double* w_full, int want_logq) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->has_model || !ctx->has_corpus) return fail(WFSA_ERR_ARG, "load a model and a corpus first");
    if (ctx->in_flight) return fail(WFSA_ERR_ARG, "objective_grad_begin called twice without _end");
    if (ctx->prep_level < 2)
        if (int rc = prepare(ctx, 2)) return rc;
    if (int rc = collect_timing(ctx)) return rc;
    if (std::getenv("WFSA_VERBOSE") && !ctx->h_seg_ptr.empty() && ctx->qn_fused) {   // slots per constraint
        const int32_t k = ctx->qn_k;
        const std::vector<int32_t>& cptr = ctx->h_cptr;
        std::vector<int64_t> sz;
        for (int32_t c = 0; c < k; ++c) sz.push_back(ctx->h_seg_ptr[size_t(cptr[size_t(c) + 1])] - ctx->h_seg_ptr[size_t(cptr[size_t(c)])]);
        std::sort(sz.begin(), sz.end());
        if (!sz.empty())
            std::fprintf(stderr, "[wfsa] slots per constraint: total %lld, max %lld, p99 %lld, p50 %lld\n",
                         (long long)ctx->h_seg_ptr.back(), (long long)sz.back(), (long long)sz[sz.size() * 99 / 100],
                         (long long)sz[sz.size() / 2]);
    }
    hipStream_t s = ctx->stream;
    const int32_t np = ctx->n_params;
    double* win = ctx->pinned + weights_off(np);   // weights in (w_full == NULL: already written there)
    if (!w_full && np > 0 && !ctx->weights_staged)
        return fail(WFSA_ERR_ARG, "null weights, and none written through wfsa_dev_weights_staging since the last call");
    ctx->weights_staged = false;
    if (np > 0 && w_full) std::memcpy(win, w_full, size_t(np) * sizeof(double));
    HIP_TRY(hipEventRecord(ctx->ev0, s));
    if (ctx->use_graph && !ctx->graph_exec && !ctx->graph_failed) {
        // capture once; a capture the runtime rejects falls back to eager launches
        if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) == hipSuccess) {
            const int rc = enqueue_iteration(ctx, true);
            hipGraph_t g = nullptr;
            const hipError_t e = hipStreamEndCapture(s, &g);
            if (rc == WFSA_OK && e == hipSuccess && g &&
                hipGraphInstantiate(&ctx->graph_exec, g, nullptr, nullptr, 0) == hipSuccess) {
                ctx->graph = g;
            } else {
                if (g) (void)hipGraphDestroy(g);
                ctx->graph_exec = nullptr;
                ctx->graph_failed = true;
                (void)hipGetLastError();
            }
        } else {
            ctx->graph_failed = true;
            (void)hipGetLastError();
        }
    }
    if (ctx->graph_exec) HIP_TRY(hipGraphLaunch(ctx->graph_exec, s));
    else if (int rc = enqueue_iteration(ctx, want_logq != 0)) return rc;
    if (ctx->comm) {
        COMM_TRY(ctx, ctx->out.ptr, size_t(np) + 1, wfsa::RedOp::SumF64, s);
        wfsa::Publish pub = publish_args(ctx);   // + the constant gradient, all-reduced once at preparation
        if (!ctx->dense && !ctx->mpath && ctx->n_groups > 0) pub.add = ctx->fixed_grad.ptr;
        HIP_TRY(wfsa::launch_publish(ctx->out.ptr, pub, s));
    }
    HIP_TRY(hipEventRecord(ctx->ev1, s));
    ++ctx->seq;
    ctx->in_flight = true;
    ctx->logq_ready = want_logq != 0 || ctx->graph_exec != nullptr;
    return WFSA_OK;
}

static int objective_grad_end_impl(wfsa_dev* ctx, double* loglik, double* grad_full, double* logq) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->in_flight) return fail(WFSA_ERR_ARG, "objective_grad_end without _begin");
    ctx->in_flight = false;
    hipStream_t s = ctx->stream;
    const int32_t np = ctx->n_params;
    if (int rc = wait_published(ctx, ctx->seq)) return rc;
    ctx->timing_pending = true;
    if (loglik) *loglik = ctx->pinned[0];
    if (grad_full && np > 0) std::memcpy(grad_full, ctx->pinned + 1, size_t(np) * sizeof(double));
    if (logq) {
        if (!ctx->logq_ready) return fail(WFSA_ERR_ARG, "log q was not requested at _begin");
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(ctx->logq.download(logq, size_t(ctx->n_strings), s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    return WFSA_OK;
}

double* wfsa_dev_weights_staging(wfsa_dev* ctx) {
    if (!ctx || !ctx->has_model || !ctx->pinned || ctx->in_flight) return nullptr;
    ctx->weights_staged = true;   // (the next _begin may take its weights from here)
    return ctx->pinned + weights_off(ctx->n_params);
}

int wfsa_dev_objective_grad(wfsa_dev* ctx, const double* w_full, double* loglik, double* grad_full, double* logq) {
    if (!w_full && ctx && ctx->n_params > 0) return fail(WFSA_ERR_ARG, "null weights");   // (only _begin takes staged weights)
    if (int rc = wfsa_dev_objective_grad_begin(ctx, w_full, logq != nullptr)) return rc;
    return wfsa_dev_objective_grad_end(ctx, loglik, grad_full, logq);
}

static int qn_setup_impl(wfsa_dev* ctx, const wfsa_qn_desc* d) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!d || d->n_params < 0 || d->n_constraints < 0) return fail(WFSA_ERR_ARG, "bad QN description");
    if (!ctx->has_model) return fail(WFSA_ERR_ARG, "load a model first");
    const int32_t nf = ctx->n_params, n = d->n_params, k = d->n_constraints;
    if ((nf > 0 && !d->trim) || (n > 0 && !d->ccol)) return fail(WFSA_ERR_ARG, "null trim/ccol");
    std::vector<int32_t> full_of(size_t(std::max(n, 1)), -1), cptr(size_t(k) + 1, 0);
    for (int32_t j = 0; j < nf; ++j) {
        const int32_t t = d->trim[j];
        if (t >= n || t < -2) return fail(WFSA_ERR_ARG, "trimmed index %d of parameter %d out of range", t, j);
        if (t >= 0) {
            if (full_of[size_t(t)] >= 0) return fail(WFSA_ERR_ARG, "trimmed index %d used twice", t);
            full_of[size_t(t)] = j;
        }
    }
    for (int32_t i = 0; i < n; ++i) {
        if (full_of[size_t(i)] < 0) return fail(WFSA_ERR_ARG, "kept parameter %d has no full index", i);
        const int32_t c = d->ccol[i];
        if (c < 0 || c >= k) return fail(WFSA_ERR_ARG, "constraint %d of parameter %d out of range", c, i);
        // Learner::BuildConstraints numbers the members of a group consecutively
        if (i > 0 && c < d->ccol[i - 1]) return fail(WFSA_ERR_ARG, "constraint columns must be non-decreasing");
        cptr[size_t(c) + 1]++;
    }
    for (int32_t c = 0; c < k; ++c) cptr[size_t(c) + 1] += cptr[size_t(c)];
    hipStream_t s = ctx->stream;
    if (nf > 0) HIP_TRY(ctx->qn_trim.upload(d->trim, size_t(nf), s));
    HIP_TRY(ctx->qn_full_of.upload(full_of.data(), full_of.size(), s));

    if (n > 0) HIP_TRY(ctx->qn_ccol.upload(d->ccol, size_t(n), s));
    HIP_TRY(ctx->qn_cptr.upload(cptr.data(), cptr.size(), s));
    for (DevBuf<double>* b : {&ctx->qn_x, &ctx->qn_expx, &ctx->qn_grad}) HIP_TRY(b->alloc(size_t(std::max(n, 1))));
    HIP_TRY(ctx->qn_lambda.alloc(size_t(std::max(k, 1))));
    HIP_TRY(ctx->qn_partial.alloc(size_t(std::max(k, 1)) * 8));   // two halves: the pipelined loop
    HIP_TRY(ctx->qn_halted.alloc(3));   // halted, halt_pending, an in-kernel QN wave timed out
    if (!ctx->qn_ring) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->qn_ring), sizeof(double) * kQnDepth * wfsa::kQnRow,
                              hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->qn_ring_dev), ctx->qn_ring, 0));
    }
    HIP_TRY(hipStreamSynchronize(s));
    ctx->qn_n = n;
    ctx->qn_k = k;
    ctx->qn_plogp = d->plogp;
    ctx->qn_exp_lambda = d->exponential_lambda ? 1 : 0;
    if (d->info_rmin && ctx->mpath && ctx->comm)
        return fail(WFSA_ERR_ARG, "rmin: matrix-file mode runs the rmin column on one rank only");
    ctx->qn_rmin = d->info_rmin != 0;
    if (ctx->qn_rmin) HIP_TRY(ctx->rm_res.alloc(4));
    // the contribution slots in trimmed order (kept parameters first, the
    // rest after), so the fused QN step sums each constraint's run in place
    int32_t max_nm = 0;
    for (int32_t c = 0; c < k; ++c) max_nm = std::max(max_nm, cptr[size_t(c) + 1] - cptr[size_t(c)]);
    // (with a communicator too: the in-kernel update across ranks reads the
    // slots in this order; the separate kernel path there reduces first)
    ctx->qn_fused = max_nm <= wfsa::kQnMaxSeg;
    ctx->qn_max_nm = std::max(1, std::min(max_nm, wfsa::kQnMaxSeg));
    if (ctx->qn_fused) {
        std::vector<int32_t> pos_of(size_t(nf), -1);
        for (int32_t i = 0; i < n; ++i) pos_of[size_t(full_of[size_t(i)])] = i;
        int32_t nxt = n;
        for (int32_t j = 0; j < nf; ++j)
            if (pos_of[size_t(j)] < 0) pos_of[size_t(j)] = nxt++;
        ctx->slot_order = pos_of;
        ctx->slot_groups = cptr;   // the constraints lead the reduction groups
        if (ctx->prep_level >= 2 && !ctx->dense && !ctx->mpath)
            if (int rc = layout_slots(ctx, pos_of)) return rc;
    }
    ctx->qw_ok = false;   // (its batches are built at the next run: build_qw_batches)
    ctx->h_cptr = cptr;
    ctx->qn_setup_gen++;
    ctx->qn_flags_clear = false;
    ctx->qn_ready = true;
    return WFSA_OK;
}

namespace {
int ensure_qst(wfsa_dev* ctx) {
    const size_t need = 2 * size_t(ctx->qn_n) + size_t(ctx->qn_k) + 1;
    if (ctx->qst_n >= need) return WFSA_OK;
    if (ctx->qst) (void)hipHostFree(ctx->qst);
    ctx->qst = nullptr;
    ctx->qst_n = 0;
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&ctx->qst), need * sizeof(double),
                          hipHostMallocMapped | hipHostMallocCoherent));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->qst_dev), ctx->qst, 0));
    ctx->qst_n = need;
    return WFSA_OK;
}
}  // namespace

int wfsa_dev_qn_set_state(wfsa_dev* ctx, const double* x, const double* lambda) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->qn_ready) return fail(WFSA_ERR_ARG, "wfsa_dev_qn_setup has not run");
    if ((ctx->qn_n > 0 && !x) || (ctx->qn_k > 0 && !lambda)) return fail(WFSA_ERR_ARG, "null state");
    if (ctx->in_flight) return fail(WFSA_ERR_ARG, "an evaluation is in flight");
    hipStream_t s = ctx->stream;
    if (int rc = ensure_qst(ctx)) return rc;
    const size_t n = size_t(ctx->qn_n), k = size_t(ctx->qn_k);
    HIP_TRY(ctx->qn_x.alloc(n));
    HIP_TRY(ctx->qn_lambda.alloc(k));
    if (n) std::memcpy(ctx->qst, x, n * sizeof(double));
    if (k) std::memcpy(ctx->qst + n, lambda, k * sizeof(double));
    HIP_TRY(wfsa::launch_copy(ctx->qst_dev, ctx->qn_x.ptr, int64_t(n), s));
    HIP_TRY(wfsa::launch_copy(ctx->qst_dev + n, ctx->qn_lambda.ptr, int64_t(k), s));
    HIP_TRY(wfsa::launch_qn_weights(ctx->qn_x.ptr, ctx->qn_trim.ptr, ctx->n_params, ctx->w_full.ptr, ctx->ewp.ptr, s));
    HIP_TRY(hipStreamSynchronize(s));
    return WFSA_OK;
}

int wfsa_dev_qn_get_state(wfsa_dev* ctx, double* x, double* lambda, double* grad) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->qn_ready) return fail(WFSA_ERR_ARG, "wfsa_dev_qn_setup has not run");
    hipStream_t s = ctx->stream;
    if (int rc = ensure_qst(ctx)) return rc;
    const size_t n = size_t(ctx->qn_n), k = size_t(ctx->qn_k);
    if ((n && (!ctx->qn_x.ptr || !ctx->qn_grad.ptr)) || (k && !ctx->qn_lambda.ptr))
        return fail(WFSA_ERR_ARG, "the QN state has not been set");
    if (x && n) HIP_TRY(wfsa::launch_copy(ctx->qn_x.ptr, ctx->qst_dev, int64_t(n), s));
    if (lambda && k) HIP_TRY(wfsa::launch_copy(ctx->qn_lambda.ptr, ctx->qst_dev + n, int64_t(k), s));
    if (grad && n) HIP_TRY(wfsa::launch_copy(ctx->qn_grad.ptr, ctx->qst_dev + n + k, int64_t(n), s));
    HIP_TRY(hipStreamSynchronize(s));
    if (x && n) std::memcpy(x, ctx->qst, n * sizeof(double));
    if (lambda && k) std::memcpy(lambda, ctx->qst + n, k * sizeof(double));
    if (grad && n) std::memcpy(grad, ctx->qst + n + k, n * sizeof(double));
    return WFSA_OK;
}

static int qn_run_impl(wfsa_dev* ctx, double eta, double tol, int32_t max_steps, double* info_rows,
                    int32_t* steps_done, int32_t* status) {
    if (int rc = check_ctx(ctx)) return rc;
    if (steps_done) *steps_done = 0;
    if (status) *status = 0;
    if (!ctx->qn_ready) return fail(WFSA_ERR_ARG, "wfsa_dev_qn_setup has not run");
    if (!ctx->has_corpus) return fail(WFSA_ERR_ARG, "load a corpus first");
    if (ctx->in_flight) return fail(WFSA_ERR_ARG, "an evaluation is in flight");
    if (max_steps <= 0) return WFSA_OK;
    using clk = std::chrono::steady_clock;
    static const bool trace = std::getenv("WFSA_VERBOSE") != nullptr;
    const auto tr0 = clk::now();
    auto tr_ms = [&](clk::time_point t) { return std::chrono::duration<double, std::micro>(t - tr0).count(); };
    clk::time_point tr_pro{}, tr_first{}, tr_last{}, tr_end{}, tr_enq1{};
    clk::time_point tp[8]{};   // (the prologue's phases, WFSA_VERBOSE)
    auto mark = [&](int i) {
        if (trace) tp[i] = clk::now();
    };
    if (ctx->prep_level < 2)
        if (int rc = prepare(ctx, 2)) return rc;
    mark(0);
    if (int rc = collect_timing(ctx)) return rc;
    mark(5);
    if (std::getenv("WFSA_VERBOSE") && !ctx->h_seg_ptr.empty() && ctx->qn_fused) {   // slots per constraint
        const int32_t k = ctx->qn_k;
        const std::vector<int32_t>& cptr = ctx->h_cptr;
        std::vector<int64_t> sz;
        for (int32_t c = 0; c < k; ++c) sz.push_back(ctx->h_seg_ptr[size_t(cptr[size_t(c) + 1])] - ctx->h_seg_ptr[size_t(cptr[size_t(c)])]);
        std::sort(sz.begin(), sz.end());
        if (!sz.empty())
            std::fprintf(stderr, "[wfsa] slots per constraint: total %lld, max %lld, p99 %lld, p50 %lld\n",
                         (long long)ctx->h_seg_ptr.back(), (long long)sz.back(), (long long)sz[sz.size() * 99 / 100],
                         (long long)sz[sz.size() / 2]);
    }
    hipStream_t s = ctx->stream;
    mark(6);
    if (!ctx->qn_flags_clear) HIP_TRY(hipMemsetAsync(ctx->qn_halted.ptr, 0, 3 * sizeof(unsigned), s));
    ctx->qn_flags_clear = false;
    ctx->fin_pending = false;
    ctx->fin_for_fbs.active = 0;
    // the constant trivial-word gradient in trimmed order, so the fused QN
    // step loads it with its members' x (no load round on their full index);
    // made once per preparation and QN set-up
    const int64_t ft_key = ctx->prep_gen * 1000003 + ctx->qn_setup_gen;
    if (ctx->qn_fused && !ctx->dense && !ctx->mpath && ctx->n_groups > 0 && ctx->qn_n > 0) {
        if (!ctx->fixed_t_on || ctx->fixed_t_key != ft_key) {
            HIP_TRY(ctx->fixed_t.alloc(size_t(ctx->qn_n)));
            HIP_TRY(wfsa::launch_gather(ctx->fixed_grad.ptr, ctx->qn_full_of.ptr, ctx->qn_n, ctx->fixed_t.ptr, s));
            ctx->fixed_t_on = true;
            ctx->fixed_t_key = ft_key;
        }
    } else {
        ctx->fixed_t_on = false;
    }
    mark(1);
    if (ctx->use_qw && ctx->qw_waves > 0)
        if (int rc = build_qw_batches(ctx)) return rc;
    mark(2);
    bool inkern = qw_usable(ctx);
    mark(3);
    if (ctx->comm) {   // every rank takes the same path (the in-kernel exchange pairs the ranks' launches):
                       // agreed once per preparation, QN set-up, layout and rmin setting
        const int64_t key = ((ctx->prep_gen * 1000003 + ctx->qn_setup_gen) * 1000003 + ctx->layout_gen) * 2 +
                            (ctx->qn_rmin ? 1 : 0);
        if (ctx->qw_agree_key != key) {   // (a sum of "cannot" votes: the peer path's sum, with its wait limit)
            double bad = inkern ? 0.0 : 1.0;
            HIP_TRY(ctx->qw_gch.alloc(std::max<size_t>(ctx->qw_gch.n, 1)));
            HIP_TRY(hipMemcpyAsync(ctx->qw_gch.ptr, &bad, sizeof bad, hipMemcpyHostToDevice, s));
            COMM_TRY(ctx, ctx->qw_gch.ptr, 1, wfsa::RedOp::SumF64, s);
            HIP_TRY(hipMemcpyAsync(&bad, ctx->qw_gch.ptr, sizeof bad, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            COMM_CHECK(ctx);
            ctx->qw_agree_key = key;
            ctx->qw_agreed = bad == 0.0;
        }
        inkern = ctx->qw_agreed;
    }
    if (!inkern && ctx->use_qw && std::getenv("WFSA_VERBOSE"))
        std::fprintf(stderr, "[wfsa] QN update as its own kernel: cover %d (%.1f rows per wave) batches %d waves %d "
                     "fused %d comm %d rmin %d delta %d fallback %d bubbles fused %d fixed_t %d k %d\n", int(ctx->qw_cover),
                     ctx->qw_mean_rows, int(ctx->qw_ok), ctx->qw_waves, int(ctx->qn_fused),
                     int(ctx->comm != nullptr), int(ctx->qn_rmin), int(ctx->delta_on),
                     ctx->n_fall[0] + ctx->n_fall[1] + ctx->n_fall[2],
                     int(ctx->n_bubbles == 0 || bubbles_fused(ctx, false)), int(ctx->fixed_t_on), ctx->qn_k);
    ctx->stats.qn_inkernel_waves = inkern ? ctx->qw_waves : 0;
    ctx->stats.qn_batches = inkern ? ctx->qw_nbatch : 0;
    if (inkern) {   // the second weight buffer
        HIP_TRY(ctx->w_full2.alloc(size_t(ctx->n_params) + 2));
        HIP_TRY(ctx->ewp2.alloc(size_t(ctx->n_params) + 2));
        // its entries the QN steps never write (the trimmed-away parameters'
        // constants and the zero slot) copied from the first buffer once per
        // preparation and QN set-up (two copies before every Run's first
        // kernel delayed it by two blit launches)
        if (ctx->pipe_init_key != ft_key || ctx->pipe_init_w != ctx->w_full2.ptr || ctx->pipe_init_e != ctx->ewp2.ptr) {
            HIP_TRY(hipMemcpyAsync(ctx->w_full2.ptr, ctx->w_full.ptr, (size_t(ctx->n_params) + 2) * sizeof(double),
                                   hipMemcpyDeviceToDevice, s));
            HIP_TRY(hipMemcpyAsync(ctx->ewp2.ptr, ctx->ewp.ptr, (size_t(ctx->n_params) + 2) * sizeof(double),
                                   hipMemcpyDeviceToDevice, s));
            ctx->pipe_init_key = ft_key;
            ctx->pipe_init_w = ctx->w_full2.ptr;
            ctx->pipe_init_e = ctx->ewp2.ptr;
        }
    }
    mark(4);
    // steps whose kernels are timed: every stride-th (not the first), or the
    // last of a run shorter than the stride
    auto timed_step = [&](int32_t e) {
        const int32_t k = ctx->timing_stride;
        return e % k == k - 1 || (max_steps < k && e == max_steps - 1);
    };
    const unsigned base = ctx->seq;
    int32_t enq = 0, done = 0, st = 0;
    bool stop = false;
    double c_ms_sum = 0.0, fb_ms_sum = 0.0;
    int64_t timed = 0;
    if (trace) tr_pro = clk::now();
    while (done < max_steps) {
        // dense steps take ~0.2 s each: two in flight keep the device busy, and
        // after a halt fewer no-op steps remain queued (their library GEMMs do not skip)
        while (!stop && enq < max_steps && enq - done < (ctx->dense ? 2 : kQnDepth)) {
            const bool tm = timed_step(enq);
            if (int rc = enqueue_qn_step(ctx, eta, tol, enq, tm, inkern, enq + 1 == max_steps))
                return rc;
            ++enq;
            ++ctx->seq;
            if (trace && enq == 1) tr_enq1 = clk::now();
        }
        if (stop || enq == max_steps)   // no next step will carry the last one's finish
            if (int rc = flush_qn_finish(ctx)) return rc;
        if (done >= enq) break;
        if (int rc = wait_published(ctx, base + unsigned(done) + 1u)) return rc;
        if (trace) (done == 0 ? tr_first : tr_last) = clk::now();
        const int slot = done % kQnDepth;
        const double* row = ctx->qn_ring + size_t(slot) * wfsa::kQnRow;
        // the row itself carries its sequence number: the flag may become
        // visible before the row's data does (and two rows published by one
        // launch may take their sequence numbers in either order)
        if (int rc = wait_row(ctx, row, base + unsigned(done) + 1u)) return rc;
        const unsigned rs = unsigned(uint64_t(row[7]) & 15u);
        if (ctx->kernel_timing && timed_step(done)) {
            float c = 0.f, f = 0.f;
            const hipEvent_t end = ctx->k2_kc[slot] ? ctx->kc[slot] : ctx->k2[slot];
            // (complete by now: the row was published by a later kernel; a
            // query, not a synchronize, which may sleep the thread for a wake-up)
            hipError_t q;
            while ((q = hipEventQuery(end)) == hipErrorNotReady) __builtin_ia32_pause();
            if (q == hipSuccess &&
                hipEventElapsedTime(&c, ctx->k0[slot], ctx->kc[slot]) == hipSuccess &&
                hipEventElapsedTime(&f, ctx->k0[slot], end) == hipSuccess) {
                c_ms_sum += c;
                fb_ms_sum += f;
                ++timed;
                ctx->stats.last_compiled_ms = c;
                ctx->stats.last_fb_kernel_ms = f;
            }
        }
        if (rs == wfsa::kQnSkipped) return fail(WFSA_ERR_HIP, "QN step %d skipped before a halt", done);
        if (rs == wfsa::kQnTimedOut)
            return fail(WFSA_ERR_HIP, "QN step %d: an in-kernel update wave's arrival wait timed out "
                        "(not every block of the stream kernel was resident)", done);
        if (rs > wfsa::kQnSkipped) return fail(WFSA_ERR_HIP, "QN step %d: malformed info row (status %u)", done, rs);
        if (info_rows)
            for (int i = 0; i < 7; ++i) info_rows[size_t(done) * 7 + size_t(i)] = row[i];
        ++done;
        if (rs == wfsa::kQnHalted || rs == wfsa::kQnNonFinite) {
            st = int(rs);
            stop = true;
            break;
        }
    }
    // drain the steps enqueued after a halt (they are no-ops)
    if (int rc = flush_qn_finish(ctx)) return rc;
    if (enq > done)
        if (int rc = wait_published(ctx, base + unsigned(enq))) return rc;
    if (inkern) {   // the weights of the final x back in the parity-0 buffers
        ctx->w_cur = ctx->ewp_cur = nullptr;
        // step e writes the weights of parity e + 1: after an even number of
        // steps, none skipped by a halt, they are in the parity-0 buffers already
        if (st != 0 || (enq & 1))
            HIP_TRY(wfsa::launch_qn_weights(ctx->qn_x.ptr, ctx->qn_trim.ptr, ctx->n_params, ctx->w_full.ptr,
                                            ctx->ewp.ptr, s));
    }
    // the last step's row is in: the stream's tail (the end of the kernel
    // that published it) is left to run beside the caller's return -- every
    // later use of the device state is ordered behind it on this stream, and
    // a failure surfaces at the next call; here only an error already known
    {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipSuccess && e != hipErrorNotReady)
            return fail(WFSA_ERR_HIP, "device failure: %s", hipGetErrorString(e));
    }
#ifdef WFSA_EXPERIMENTS
    if (std::getenv("WFSA_FBS_TRACE") && ctx->fbs_trace.ptr) {   // the last launch's per-wave stamps
        const int wpb = ctx->i_block / kWave, nw = ctx->i_grid * wpb;
        std::vector<unsigned long long> t(size_t(nw) * 16);
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(ctx->fbs_trace.download(t.data(), t.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
        unsigned long long t0 = ~0ull;
        for (int w = 0; w < nw; ++w)
            if (t[size_t(w) * 16]) t0 = std::min(t0, t[size_t(w) * 16]);
        const int small_wpb = small_waves_per_block(wfsa::small_chunks(ctx->n_small4, ctx->n_small) * kWave, ctx->i_grid);
        const char* names[8] = {"entry", "staged", "bubbles", "arrived", "stream", "qn-poll", "qn-done", "exit"};
        for (int grp = 0; grp < 3; ++grp) {
            for (int k = 0; k < 8; ++k) {
                std::vector<double> v;
                for (int w = 0; w < nw; ++w) {
                    const int wib = w % wpb, bid = w / wpb;
                    const bool qn = wib == wpb - 2 && bid < ctx->qw_waves, sb = wib < small_wpb;
                    if ((grp == 1 && !sb) || (grp == 2 && !qn)) continue;
                    const unsigned long long x = t[size_t(w) * 16 + size_t(k)];
                    if (x) v.push_back(double(x - t0) / 100.0);   // 100 MHz -> us
                }
                if (v.empty()) continue;
                std::sort(v.begin(), v.end());
                auto q = [&](double f) { return v[std::min(v.size() - 1, size_t(f * double(v.size())))]; };
                std::fprintf(stderr, "[fbs-trace] %-12s %-8s n %5zu  min %6.2f p10 %6.2f p50 %6.2f p90 %6.2f max %6.2f us\n",
                             grp == 0 ? "all waves" : grp == 1 ? "small-bubble" : "qn waves", names[k], v.size(), v[0],
                             q(0.1), q(0.5), q(0.9), v.back());
            }
        }
        // small-bubble phases (stamps 8..11: quads loaded, weights gathered,
        // forward done, backward done), by class (A: chunk below n_small4)
        for (int cls = 0; cls < 2; ++cls) {
            std::vector<double> ph[4];
            for (int w = 0; w < nw; ++w) {
                const int wib = w % wpb, bid = w / wpb;
                if (wib >= small_wpb) continue;
                const int64_t ch = int64_t(wib) * ctx->i_grid + bid;   // (wfsa::small_entry's chunks)
                const int64_t na = (int64_t(ctx->n_small4) + kWave - 1) / kWave;
                if (ch >= wfsa::small_chunks(ctx->n_small4, ctx->n_small) || (ch < na) != (cls == 0)) continue;
                const unsigned long long* r = &t[size_t(w) * 16];
                const unsigned long long st = r[1] ? r[1] : r[0];
                const unsigned long long pts[5] = {st, r[8], r[9], r[10], r[11]};
                for (int k = 0; k < 4; ++k)
                    if (pts[k] && pts[k + 1]) ph[k].push_back(double(pts[k + 1] - pts[k]) / 100.0);
            }
            const char* pn[4] = {"quads", "gathers", "forward", "backward"};
            std::fprintf(stderr, "[fbs-trace] class %c small-bubble phases (p50 / p90 / max us):", cls ? 'B' : 'A');
            for (int k = 0; k < 4; ++k) {
                if (ph[k].empty()) continue;
                std::sort(ph[k].begin(), ph[k].end());
                std::fprintf(stderr, " %s %.2f / %.2f / %.2f;", pn[k], ph[k][ph[k].size() / 2], ph[k][ph[k].size() * 9 / 10],
                             ph[k].back());
            }
            std::fprintf(stderr, "\n");
        }
        {   // the QN waves' phases: poll done (5) -> halt flag + slot chunks summed (8) -> member and
            // constraint sums (9) -> x / weight stores (10) -> done (6)
            std::vector<double> ph[4];
            for (int w = 0; w < nw; ++w) {
                if (!(w % wpb == wpb - 2 && w / wpb < ctx->qw_waves)) continue;
                const unsigned long long* r = &t[size_t(w) * 16];
                const unsigned long long pts[5] = {r[5], r[8], r[9], r[10], r[6]};
                for (int k = 0; k < 4; ++k)
                    if (pts[k] && pts[k + 1] && pts[k + 1] >= pts[k]) ph[k].push_back(double(pts[k + 1] - pts[k]) / 100.0);
            }
            const char* pn[4] = {"chunks", "sums", "stores", "tail"};
            std::fprintf(stderr, "[fbs-trace] QN wave phases (p50 / p90 / max us):");
            for (int k = 0; k < 4; ++k) {
                if (ph[k].empty()) continue;
                std::sort(ph[k].begin(), ph[k].end());
                std::fprintf(stderr, " %s %.2f / %.2f / %.2f;", pn[k], ph[k][ph[k].size() / 2], ph[k][ph[k].size() * 9 / 10],
                             ph[k].back());
            }
            std::fprintf(stderr, "\n");
        }
        {   // the QN waves' polls (11: start, 13: first poll returned, 12: iterations) and the
            // blocks' arrival atomics (wave 0's words 14: the atomic returned, 15: its order)
            std::vector<double> it, per, first;
            for (int w = 0; w < nw; ++w) {
                if (!(w % wpb == wpb - 2 && w / wpb < ctx->qw_waves)) continue;
                const unsigned long long* r = &t[size_t(w) * 16];
                if (!r[11] || !r[5]) continue;
                it.push_back(double(r[12]));
                if (r[12] > 0) per.push_back(double(r[5] - r[11]) / 100.0 / double(r[12]));
                if (r[13]) first.push_back(double(r[13] - r[11]) / 100.0);
            }
            std::vector<std::pair<double, int>> land;
            for (int b = 0; b < ctx->i_grid; ++b) {
                const unsigned long long* r = &t[size_t(b) * wpb * 16];
                if (r[14]) land.push_back({double(r[14] - t0) / 100.0, int(r[15])});
            }
            std::sort(land.begin(), land.end());
            auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v.empty() ? -1.0 : v[v.size() / 2]; };
            auto mx = [](const std::vector<double>& v) { return v.empty() ? -1.0 : *std::max_element(v.begin(), v.end()); };
            std::fprintf(stderr, "[fbs-trace] QN polls: iterations p50 %.0f max %.0f; us per poll p50 %.2f max %.2f; first poll "
                         "p50 %.2f max %.2f us; block arrivals landed: n %zu",
                         med(it), mx(it), med(per), mx(per), med(first), mx(first), land.size());
            for (size_t i = land.size() > 4 ? land.size() - 4 : 0; i < land.size(); ++i)
                std::fprintf(stderr, " (%.2f us, order %d)", land[i].first, land[i].second);
            std::fprintf(stderr, "\n");
        }
        // the deal's calibration: each wave's stream-phase end (stamp 4, from
        // its staging stamp) against its delta rows and its extra work, by
        // least squares: end = c0 + c1 rows + cA [class A] + cB [class B] +
        // cG [big] + cQ [QN wave]; the implied charges in rows are cX / c1
        if (ctx->delta_on && ctx->d_wave_first.ptr && ctx->d_g_base.ptr) {
            std::vector<int32_t> wf(size_t(nw) + 1);
            std::vector<int64_t> gb(size_t(ctx->n_groups) + 1);
            HIP_TRY(ctx->d_wave_first.download(wf.data(), wf.size(), s));
            HIP_TRY(ctx->d_g_base.download(gb.data(), gb.size(), s));
            HIP_TRY(hipStreamSynchronize(s));
            const int64_t nch = wfsa::small_chunks(ctx->n_small4, ctx->n_small);
            const int64_t na = (int64_t(ctx->n_small4) + kWave - 1) / kWave;
            double M[6][6] = {}, v[6] = {};
            double sums[5][3] = {};   // per kind: n, rows, end
            for (int w = 0; w < nw; ++w) {
                const int wib = w % wpb, bid = w / wpb;
                const unsigned long long* r = &t[size_t(w) * 16];
                if (!r[1] || !r[4] || (bid == 0 && wib == wpb - 1)) continue;
                const double end = double(r[4] - r[1]) / 100.0;
                const double rows = double(gb[size_t(wf[size_t(w) + 1])] - gb[size_t(wf[size_t(w)])]) / kWave;
                double x[6] = {1.0, rows, 0, 0, 0, 0};
                const int64_t ch = int64_t(wib) * ctx->i_grid + bid;
                int kind = 0;
                if (wib < small_wpb && ch < nch) {
                    kind = ch >= na ? 2 : 1;
                    x[kind + 1] = 1.0;
                }
                const int64_t rb = wfsa::big_rank(bid, wib, ctx->i_grid, wpb, ctx->qw_waves);
                if (rb < ctx->n_big) {
                    x[4] = 1.0;
                    kind = kind ? kind : 3;
                }
                if (wib == wpb - 2 && bid < ctx->qw_waves) {
                    x[5] = 1.0;
                    kind = 4;
                }
                sums[kind][0] += 1;
                sums[kind][1] += rows;
                sums[kind][2] += end;
                for (int i = 0; i < 6; ++i) {
                    v[i] += x[i] * end;
                    for (int j = 0; j < 6; ++j) M[i][j] += x[i] * x[j];
                }
            }
            for (int i = 0; i < 6; ++i) M[i][i] += 1e-9;   // (a kind absent: its coefficient 0)
            for (int c = 0; c < 6; ++c) {   // Gauss-Jordan
                int p = c;
                for (int i = c + 1; i < 6; ++i)
                    if (std::abs(M[i][c]) > std::abs(M[p][c])) p = i;
                for (int j = 0; j < 6; ++j) std::swap(M[c][j], M[p][j]);
                std::swap(v[c], v[p]);
                for (int i = 0; i < 6; ++i) {
                    if (i == c || M[c][c] == 0.0) continue;
                    const double f = M[i][c] / M[c][c];
                    for (int j = 0; j < 6; ++j) M[i][j] -= f * M[c][j];
                    v[i] -= f * v[c];
                }
            }
            double cf[6];
            for (int i = 0; i < 6; ++i) cf[i] = M[i][i] != 0.0 ? v[i] / M[i][i] : 0.0;
            const char* kn[5] = {"stream only", "class A", "class B", "big", "QN"};
            std::fprintf(stderr, "[fbs-trace] deal fit: end = %.2f + %.4f rows us; charges in rows: A %.1f B %.1f big %.1f "
                         "QN %.1f\n[fbs-trace] deal by kind (n, mean rows, mean end us):", cf[0], cf[1], cf[2] / cf[1],
                         cf[3] / cf[1], cf[4] / cf[1], cf[5] / cf[1]);
            for (int k = 0; k < 5; ++k)
                if (sums[k][0] > 0)
                    std::fprintf(stderr, " %s (%.0f, %.1f, %.2f)", kn[k], sums[k][0], sums[k][1] / sums[k][0],
                                 sums[k][2] / sums[k][0]);
            std::fprintf(stderr, "\n");
        }
        // the slowest bubble waves and QN waves
        auto dt = [&](int w, int a, int b) {
            const unsigned long long x = t[size_t(w) * 16 + size_t(a)], y = t[size_t(w) * 16 + size_t(b)];
            return x && y ? double(y - x) / 100.0 : -1.0;
        };
        std::vector<std::pair<double, int>> bw, qw;
        for (int w = 0; w < nw; ++w) {
            bw.push_back({dt(w, 1, 2), w});
            if (w % wpb == wpb - 2 && w / wpb < ctx->qw_waves) qw.push_back({dt(w, 5, 6), w});
        }
        std::sort(bw.rbegin(), bw.rend());
        std::sort(qw.rbegin(), qw.rend());
        std::fprintf(stderr, "[fbs-trace] small %d/%d big %d, small waves per block %d; slowest bubble phases:", ctx->n_small4,
                     ctx->n_small, ctx->n_big, small_wpb);
        for (size_t i = 0; i < std::min<size_t>(8, bw.size()); ++i)
            std::fprintf(stderr, " (b%d w%d %.2f)", bw[i].second / wpb, bw[i].second % wpb, bw[i].first);
        std::fprintf(stderr, "\n[fbs-trace] slowest QN waves (batch: constraints members chunks):");
        for (size_t i = 0; i < std::min<size_t>(8, qw.size()); ++i) {
            const int b = qw[i].second / wpb;
            if (size_t(2 * b + 1) < ctx->h_qw_batch.size()) {
                const int4 x = ctx->h_qw_batch[size_t(2 * b)], y = ctx->h_qw_batch[size_t(2 * b + 1)];
                std::fprintf(stderr, " (%.2f us: %d %d %d)", qw[i].first, x.y - x.x, x.w - x.z, y.x);
            }
        }
        std::fprintf(stderr, "\n");
    }
#endif
    if (trace) {
        tr_end = clk::now();
        std::fprintf(stderr, "[wfsa] qn_run prologue: prepared %.1f, timing %.1f, (verbose stats) %.1f, flags + fixed %.1f, "
                     "batches %.1f, path %.1f, buffers %.1f us\n", tr_ms(tp[0]), tr_ms(tp[5]), tr_ms(tp[6]), tr_ms(tp[1]),
                     tr_ms(tp[2]), tr_ms(tp[3]), tr_ms(tp[4]));
        std::fprintf(stderr, "[wfsa] qn_run %d steps: prologue %.1f us, first step enqueued %.1f, first row %.1f, "
                     "last row %.1f, end %.1f (start at %lld ns)\n",
                     done, tr_ms(tr_pro), tr_ms(tr_enq1), tr_ms(tr_first), done > 1 ? tr_ms(tr_last) : tr_ms(tr_first),
                     tr_ms(tr_end), (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(tr0.time_since_epoch()).count());
    }
    ctx->qn_flags_clear = st == 0;
    ctx->stats.fb_launches += timed;
    ctx->stats.fb_kernel_ms += fb_ms_sum;
    ctx->stats.compiled_kernel_ms += c_ms_sum;
    if (steps_done) *steps_done = done;
    if (status) *status = st;
    return WFSA_OK;
}

static int hf_setup_impl(wfsa_dev* ctx, int64_t* n_pairs) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->has_model || !ctx->has_corpus) return fail(WFSA_ERR_ARG, "load a model and a corpus first");
    if (ctx->in_flight) return fail(WFSA_ERR_ARG, "an evaluation is in flight");
    if (ctx->dense) return fail(WFSA_ERR_CAPACITY, "second-order terms: not available on the dense path");
    if (ctx->mpath && ctx->comm) return fail(WFSA_ERR_ARG, "second-order terms: matrix-file mode runs on one rank only");
    if (ctx->mpath) {   // the pattern and the slots come from the path matrices
        HIP_TRY(ctx->mpath->hf_setup(ctx->hf_pairs, ctx->stream));
        HIP_TRY(ctx->hf_out.alloc(std::max<size_t>(ctx->hf_pairs.size() / 2, 1)));
        ctx->hf_ready = true;
        ctx->hf_gen = ctx->prep_gen;
        if (n_pairs) *n_pairs = int64_t(ctx->hf_pairs.size() / 2);
        return WFSA_OK;
    }
    if (ctx->prep_level < 2)
        if (int rc = prepare(ctx, 2)) return rc;
    hipStream_t s = ctx->stream;
    const int64_t nfall = int64_t(ctx->n_fall[0]) + ctx->n_fall[1] + ctx->n_fall[2];
    // traversal strings: their equivocal parameters, found on the host from
    // exact min / max counts over each string's trellis (hf_trav_kernel)
    std::vector<int4> tl;
    std::vector<int32_t> tv;
    int64_t bad_string = -1;
    size_t bad_v = 0;
    if (nfall > 0) {
        std::vector<int64_t> off(size_t(ctx->n_strings) + 1);
        HIP_TRY(ctx->off.download(off.data(), off.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<uint8_t> sy(static_cast<size_t>(off.back()));
        HIP_TRY(ctx->sym.download(sy.data(), sy.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<int32_t> V;
        for (int64_t i = 0; i < ctx->n_strings && bad_string < 0; ++i) {
            if (ctx->h_tier[size_t(i)] < 0) continue;
            const int L = int(off[size_t(i) + 1] - off[size_t(i)]);
            if (!equivocal_params(*ctx->h_tm, ctx->h_pptr, ctx->h_pidx, sy.data() + off[size_t(i)], L, V, 4096) ||
                V.size() > size_t(wfsa::kHfTravMaxV)) {
                bad_string = i;
                bad_v = V.size();
                break;
            }
            if (V.empty()) continue;
            tl.push_back(make_int4(int32_t(i), int32_t(tv.size()), int32_t(V.size()), 0));
            tv.insert(tv.end(), V.begin(), V.end());
        }
    }
    const int32_t np = ctx->n_params, nb = ctx->n_bubbles;
    std::vector<int32_t> off(size_t(std::max(nb, 1)));
    std::vector<int32_t> buf(ctx->bub.n);
    if (nb > 0) {
        HIP_TRY(ctx->bub_off.download(off.data(), size_t(nb), s));
        HIP_TRY(ctx->bub.download(buf.data(), buf.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
    }
    auto params = [&](int32_t code, std::vector<int32_t>& out) {   // edge_code -> parameters
        out.clear();
        if (code >= 0) {
            if (code < np) out.push_back(code);
        } else {
            const int32_t g = -code - 2;
            for (int32_t q = ctx->h_pptr[size_t(g)]; q < ctx->h_pptr[size_t(g) + 1]; ++q) out.push_back(ctx->h_pidx[size_t(q)]);
        }
    };
    // slots in the kernel's order: (e, f), j in e, k in f, j <= k
    std::vector<int64_t> base(size_t(nb) + 1, 0), keys;
    std::vector<std::vector<int32_t>> ep;
    std::vector<int32_t> tmp;
    size_t bad_edge_params = 0;   // a bubble edge with more than 8 parameters
    for (int32_t b = 0; b < nb && bad_edge_params == 0; ++b) {
        const int32_t o = off[size_t(b)];
        const int edges = buf[size_t(o)] >> 16;
        ep.assign(size_t(edges), {});
        for (int e = 0; e < edges; ++e) {
            params(buf[size_t(o) + 4 + 2 * size_t(e)], tmp);
            if (tmp.size() > 8 && bad_edge_params == 0) bad_edge_params = tmp.size();
            ep[size_t(e)] = tmp;
        }
        for (int e = 0; e < edges; ++e)
            for (int f = 0; f < edges; ++f)
                for (int32_t j : ep[size_t(e)])
                    for (int32_t k : ep[size_t(f)])
                        if (j <= k) keys.push_back(int64_t(j) * np + k);
        base[size_t(b) + 1] = int64_t(keys.size());
    }
    // every limit is checked before the status all-reduce below, so a rank
    // that fails never leaves the others waiting in a later collective
    const bool local_bad = bad_string >= 0 || bad_edge_params > 0;
    if (ctx->comm) {   // every rank learns whether any cannot build its part (no rank is left in a collective)
        DevBuf<double> t;
        double bad = local_bad ? 1.0 : 0.0;
        HIP_TRY(t.upload(&bad, 1, s));
        COMM_TRY(ctx, t.ptr, 1, wfsa::RedOp::SumF64, s);
        HIP_TRY(t.download(&bad, 1, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (bad > 0 && !local_bad)
            return fail(WFSA_ERR_CAPACITY, "second-order terms: another rank has a string beyond their limits");
    }
    if (bad_edge_params > 0)
        return fail(WFSA_ERR_CAPACITY, "second-order terms: a bubble edge carries %zu parameters (max 8)",
                    bad_edge_params);
    if (local_bad)
        return fail(WFSA_ERR_CAPACITY, "second-order terms: string %lld has %s equivocal parameters (at most %d, "
                    "from at most 4096 parameters on its paths)", (long long)bad_string,
                    bad_v ? std::to_string(bad_v).c_str() : "too many", wfsa::kHfTravMaxV);
    // the traversal strings' slots follow the bubbles': (a <= b) over V_s, row-major
    std::vector<int64_t> tbase;
    for (const int4& t : tl) {
        tbase.push_back(int64_t(keys.size()));
        const int32_t* V = tv.data() + t.y;
        for (int a2 = 0; a2 < t.z; ++a2)
            for (int b2 = a2; b2 < t.z; ++b2) keys.push_back(int64_t(V[a2]) * np + V[b2]);
    }
    const int64_t ns = int64_t(keys.size());
    std::vector<int64_t> order(static_cast<size_t>(ns));
    for (int64_t i = 0; i < ns; ++i) order[size_t(i)] = i;
    std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return keys[size_t(x)] < keys[size_t(y)]; });
    std::vector<int64_t> tptr(1, 0);
    ctx->hf_pairs.clear();
    for (int64_t i = 0; i < ns; ++i) {
        const int64_t key = keys[size_t(order[size_t(i)])];
        if (i == 0 || key != keys[size_t(order[size_t(i) - 1])]) {
            if (i > 0) tptr.push_back(i);
            ctx->hf_pairs.push_back(int32_t(key / np));
            ctx->hf_pairs.push_back(int32_t(key % np));
        }
    }
    tptr.push_back(ns);
    if (ns == 0) tptr.assign(1, 0);
    if (ctx->comm) {
        // the pattern is the union over the ranks: every rank's pairs (keys
        // j*np+k, exact in a double) gathered by a sum into per-rank segments;
        // a global pair this rank never sees gets an empty slot run
        const int nr = ctx->comm->nranks(), me = ctx->comm->rank();
        const size_t nloc = ctx->hf_pairs.size() / 2;
        std::vector<double> cnt(size_t(nr), 0.0);
        cnt[size_t(me)] = double(nloc);
        DevBuf<double> t;
        HIP_TRY(t.upload(cnt.data(), cnt.size(), s));
        COMM_TRY(ctx, t.ptr, cnt.size(), wfsa::RedOp::SumF64, s);
        HIP_TRY(t.download(cnt.data(), cnt.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
        size_t total = 0, mine = 0;
        for (int r = 0; r < nr; ++r) {
            if (r == me) mine = total;
            total += size_t(cnt[size_t(r)]);
        }
        std::vector<double> all(std::max<size_t>(total, 1), 0.0);
        for (size_t i = 0; i < nloc; ++i)
            all[mine + i] = double(int64_t(ctx->hf_pairs[2 * i]) * np + ctx->hf_pairs[2 * i + 1]);
        HIP_TRY(t.upload(all.data(), all.size(), s));
        COMM_TRY(ctx, t.ptr, all.size(), wfsa::RedOp::SumF64, s);
        HIP_TRY(t.download(all.data(), all.size(), s));
        HIP_TRY(hipStreamSynchronize(s));
        std::vector<int64_t> gk(total);
        for (size_t i = 0; i < total; ++i) gk[i] = int64_t(all[i]);
        std::sort(gk.begin(), gk.end());
        gk.erase(std::unique(gk.begin(), gk.end()), gk.end());
        std::vector<int64_t> gptr(gk.size() + 1, 0);
        size_t li = 0;
        int64_t pos = 0;
        for (size_t g = 0; g < gk.size(); ++g) {
            gptr[g] = pos;
            if (li < nloc && int64_t(ctx->hf_pairs[2 * li]) * np + ctx->hf_pairs[2 * li + 1] == gk[g]) {
                pos = tptr[li + 1];
                ++li;
            }
        }
        gptr[gk.size()] = pos;
        tptr = gptr;
        ctx->hf_pairs.clear();
        for (int64_t key : gk) {
            ctx->hf_pairs.push_back(int32_t(key / np));
            ctx->hf_pairs.push_back(int32_t(key % np));
        }
    }
    HIP_TRY(ctx->hf_slot_base.upload(base.data(), base.size(), s));
    HIP_TRY(ctx->hf_t_ptr.upload(tptr.data(), tptr.size(), s));
    HIP_TRY(ctx->hf_t_slot.upload(order.empty() ? base.data() : order.data(), std::max<size_t>(order.size(), 1), s));
    HIP_TRY(ctx->hf_slot_val.alloc(size_t(std::max<int64_t>(ns, 1))));
    HIP_TRY(ctx->hf_out.alloc(std::max<size_t>(ctx->hf_pairs.size() / 2, 1)));
    ctx->hft_n = int32_t(tl.size());
    if (!tl.empty()) {
        HIP_TRY(ctx->hft_list.upload(tl.data(), tl.size(), s));
        HIP_TRY(ctx->hft_v.upload(tv.data(), tv.size(), s));
        HIP_TRY(ctx->hft_base.upload(tbase.data(), tbase.size(), s));
        int32_t vm = kWave, nv_max = 0;
        for (const int4& t : tl) nv_max = std::max(nv_max, t.z);
        while (vm < nv_max) vm *= 2;   // 64, 128, 256, 512: the kernel's column tiers
        ctx->hft_vm = vm;
        ctx->hft_stride = wfsa::hf_trav_stride(ctx->max_len, ctx->n_nodes, vm);
        const int64_t budget = (int64_t(2) << 30) / 8;   // 2 GiB of per-wave scratch
        constexpr int wpb = wfsa::kHfBlock / kWave;
        int64_t waves = std::min<int64_t>(int64_t(tl.size()), int64_t(ctx->n_cu) * 8);
        waves = std::max<int64_t>(1, std::min<int64_t>(waves, budget / ctx->hft_stride));
        ctx->hft_grid = int((waves + wpb - 1) / wpb);
        HIP_TRY(ctx->hft_scratch.alloc(size_t(ctx->hft_grid) * wpb * size_t(ctx->hft_stride)));
    }
    HIP_TRY(hipStreamSynchronize(s));
    ctx->hf_n_slots = ns;
    ctx->hf_ready = true;
    ctx->hf_gen = ctx->prep_gen;
    if (n_pairs) *n_pairs = int64_t(ctx->hf_pairs.size() / 2);
    return WFSA_OK;
}

int wfsa_dev_hf_pairs(wfsa_dev* ctx, int32_t* pairs) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->hf_ready || ctx->hf_gen != ctx->prep_gen) return fail(WFSA_ERR_ARG, "wfsa_dev_hf_setup has not run");
    if (pairs && !ctx->hf_pairs.empty()) std::memcpy(pairs, ctx->hf_pairs.data(), ctx->hf_pairs.size() * sizeof(int32_t));
    return WFSA_OK;
}

static int hf_eval_impl(wfsa_dev* ctx, const double* w_full, double* values) {
    if (int rc = check_ctx(ctx)) return rc;
    if (!ctx->hf_ready || ctx->hf_gen != ctx->prep_gen) return fail(WFSA_ERR_ARG, "wfsa_dev_hf_setup has not run");
    if (ctx->in_flight) return fail(WFSA_ERR_ARG, "an evaluation is in flight");
    if (!w_full && ctx->n_params > 0) return fail(WFSA_ERR_ARG, "null weights");
    hipStream_t s = ctx->stream;
    const int32_t np = ctx->n_params;
    if (np > 0) std::memcpy(ctx->pinned + weights_off(np), w_full, size_t(np) * sizeof(double));
    HIP_TRY(wfsa::launch_stage(ctx->pinned_dev + weights_off(np), ctx->w_full.ptr, ctx->ewp.ptr, np, s));
    if (ctx->mpath) {
        const size_t n_pattern = ctx->hf_pairs.size() / 2;
        HIP_TRY(ctx->mpath->hf_eval(ctx->w_full.ptr, ctx->hf_out.ptr, s));
        if (values && n_pattern > 0) HIP_TRY(ctx->hf_out.download(values, n_pattern, s));
        HIP_TRY(hipStreamSynchronize(s));
        return WFSA_OK;
    }
    wfsa::HfArgs a{};
    a.m = model_view(ctx);
    a.bub = ctx->bub.ptr;
    a.bub_off = ctx->bub_off.ptr;
    a.slot_base = ctx->hf_slot_base.ptr;
    a.n_bubbles = ctx->n_bubbles;
    a.w = ctx->w_full.ptr;
    a.ewp = ctx->ewp.ptr;
    a.slot_val = ctx->hf_slot_val.ptr;
    a.t_ptr = ctx->hf_t_ptr.ptr;
    a.t_slot = ctx->hf_t_slot.ptr;
    a.n_pattern = int64_t(ctx->hf_pairs.size() / 2);
    a.out = ctx->hf_out.ptr;
    wfsa::HfTravArgs t{};
    if (ctx->hft_n > 0) {
        t.m = a.m;
        t.w.c_ptr = ctx->w_cptr.ptr;
        t.w.dst = ctx->w_dst.ptr;
        t.w.e_ptr = ctx->w_eptr.ptr;
        t.w.e_src = ctx->w_esrc.ptr;
        t.w.e_g = ctx->w_eg.ptr;
        t.sym = ctx->sym.ptr;
        t.off = ctx->off.ptr;
        t.p = ctx->p.ptr;
        t.list = ctx->hft_list.ptr;
        t.vlist = ctx->hft_v.ptr;
        t.slot_base = ctx->hft_base.ptr;
        t.n_list = ctx->hft_n;
        t.max_len = ctx->max_len;
        t.wt = ctx->w_full.ptr;
        t.scratch = ctx->hft_scratch.ptr;
        t.stride = ctx->hft_stride;
        t.vm = ctx->hft_vm;
        t.slot_val = ctx->hf_slot_val.ptr;
    }
    HIP_TRY(wfsa::launch_hf(a, s, ctx->hft_n > 0 ? &t : nullptr, ctx->hft_grid));
    if (ctx->comm && a.n_pattern > 0) COMM_TRY(ctx, ctx->hf_out.ptr, size_t(a.n_pattern), wfsa::RedOp::SumF64, s);
    if (values && a.n_pattern > 0) HIP_TRY(ctx->hf_out.download(values, size_t(a.n_pattern), s));
    HIP_TRY(hipStreamSynchronize(s));
    COMM_CHECK(ctx);
    return WFSA_OK;
}

int wfsa_dev_comm_unique_id(uint8_t id[WFSA_COMM_ID_BYTES]) {
    if (!id) return fail(WFSA_ERR_ARG, "null id");
    static_assert(wfsa::kCommIdBytes == WFSA_COMM_ID_BYTES, "communicator id size");
    std::string err;
    if (wfsa::rccl_unique_id(id, err)) return fail(WFSA_ERR_RCCL, "%s", err.c_str());
    return WFSA_OK;
}

int wfsa_dev_comm_local_id(int nranks, uint8_t id[WFSA_COMM_ID_BYTES]) {
    if (!id) return fail(WFSA_ERR_ARG, "null id");
    if (nranks < 1 || nranks > wfsa::kLocalMaxRanks) return fail(WFSA_ERR_ARG, "an in-process group has 1..16 members");
    wfsa::local_group_id(nranks, id);
    return WFSA_OK;
}

int wfsa_dev_comm_init(wfsa_dev* ctx, int nranks, int rank, const uint8_t id[WFSA_COMM_ID_BYTES]) {
    if (int rc = check_ctx(ctx)) return rc;
    if (nranks < 1 || rank < 0 || rank >= nranks || !id) return fail(WFSA_ERR_ARG, "bad communicator arguments");
    ctx->comm.reset();
    std::string err;
    ctx->comm = wfsa::is_local_group_id(id) ? wfsa::make_local_collective(nranks, rank, id, ctx->device, err)
                                            : wfsa::make_rccl_collective(nranks, rank, id, err);
    if (!ctx->comm) return fail(WFSA_ERR_RCCL, "%s", err.c_str());
    ctx->nranks = nranks;
    ctx->rank = rank;
    // the compiled corpus' constant gradient is summed over the ranks at
    // compilation: compile again (every rank does, in the same call order)
    if (ctx->prep_level >= 2) ctx->prep_level = 1;
    ctx->qn_fused = false;   // the per-step all-reduce needs the reduced vector
    return WFSA_OK;
}

int wfsa_dev_comm_init_host(wfsa_dev* ctx, int nranks, int rank, wfsa_host_allreduce_fn fn, void* user) {
    if (int rc = check_ctx(ctx)) return rc;
    if (nranks < 1 || rank < 0 || rank >= nranks || !fn) return fail(WFSA_ERR_ARG, "bad communicator arguments");
    ctx->comm.reset();
    std::string err;
    ctx->comm = wfsa::make_host_collective(nranks, rank, fn, user, err);
    if (!ctx->comm) return fail(WFSA_ERR_RCCL, "%s", err.c_str());
    ctx->nranks = nranks;
    ctx->rank = rank;
    if (ctx->prep_level >= 2) ctx->prep_level = 1;   // (as wfsa_dev_comm_init)
    ctx->qn_fused = false;
    return WFSA_OK;
}

static int allreduce_impl(wfsa_dev* ctx, double* host_buf, int64_t count) {
    if (int rc = check_ctx(ctx)) return rc;
    if (count <= 0) return WFSA_OK;
    if (!host_buf) return fail(WFSA_ERR_ARG, "null buffer");
    if (!ctx->comm) return WFSA_OK;   // single rank: the sum is the input
    DevBuf<double> tmp;
    HIP_TRY(tmp.upload(host_buf, size_t(count), ctx->stream));
    COMM_TRY(ctx, tmp.ptr, size_t(count), wfsa::RedOp::SumF64, ctx->stream);
    HIP_TRY(tmp.download(host_buf, size_t(count), ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    COMM_CHECK(ctx);
    return WFSA_OK;
}

int wfsa_dev_get_stats(wfsa_dev* ctx, wfsa_dev_stats* out) {
    if (!ctx || !out) return fail(WFSA_ERR_ARG, "null argument");
    if (!ctx->in_flight)
        if (int rc = collect_timing(ctx)) return rc;
    *out = ctx->stats;
    out->comm_ranks = ctx->comm ? ctx->comm->nranks() : 1;
    const char* ps = ctx->comm ? ctx->comm->peer_state() : "off";
    out->comm_peer = std::strcmp(ps, "on") == 0 ? 1 : std::strcmp(ps, "failed") == 0 ? -1 : 0;
    return WFSA_OK;
}


// Entry points that take part in rank collectives: a failure on this rank
// (anything but a bad argument, which fails before any collective) aborts
// the communicator, so the other ranks' current or next collective fails at
// once instead of waiting for a member that will not come.
static int rank_guard(wfsa_dev* ctx, int rc) {
    if (rc != WFSA_OK && rc != WFSA_ERR_ARG && ctx && ctx->comm) ctx->comm->abort(g_last_error.c_str());
    return rc;
}
int wfsa_dev_recognize(wfsa_dev* ctx, uint8_t* recognized, double* path_count, uint8_t* used_param) { return rank_guard(ctx, recognize_impl(ctx, recognized, path_count, used_param)); }
int wfsa_dev_rmin(wfsa_dev* ctx, double* rmin, int64_t* string_index) { return rank_guard(ctx, rmin_impl(ctx, rmin, string_index)); }
int wfsa_dev_objective_grad_begin(wfsa_dev* ctx, const double* w_full, int want_logq) { return rank_guard(ctx, objective_grad_begin_impl(ctx, w_full, want_logq)); }
int wfsa_dev_objective_grad_end(wfsa_dev* ctx, double* loglik, double* grad_full, double* logq) { return rank_guard(ctx, objective_grad_end_impl(ctx, loglik, grad_full, logq)); }
int wfsa_dev_qn_setup(wfsa_dev* ctx, const wfsa_qn_desc* d) { return rank_guard(ctx, qn_setup_impl(ctx, d)); }
int wfsa_dev_qn_run(wfsa_dev* ctx, double eta, double tol, int32_t max_steps, double* info_rows, int32_t* steps_done, int32_t* status) { return rank_guard(ctx, qn_run_impl(ctx, eta, tol, max_steps, info_rows, steps_done, status)); }
int wfsa_dev_hf_setup(wfsa_dev* ctx, int64_t* n_pairs) { return rank_guard(ctx, hf_setup_impl(ctx, n_pairs)); }
int wfsa_dev_hf_eval(wfsa_dev* ctx, const double* w_full, double* values) { return rank_guard(ctx, hf_eval_impl(ctx, w_full, values)); }
int wfsa_dev_allreduce(wfsa_dev* ctx, double* host_buf, int64_t count) { return rank_guard(ctx, allreduce_impl(ctx, host_buf, count)); }

int wfsa_dev_comm_abort(wfsa_dev* ctx, const char* why) {
    if (int rc = check_ctx(ctx)) return rc;
    if (ctx->comm) ctx->comm->abort(why ? why : "wfsa_dev_comm_abort");
    return WFSA_OK;
}

int wfsa_dev_peer_selftest(int device, int nranks, int64_t n, double timeout_s, int mode, double out[4]) {
    if (!out) return fail(WFSA_ERR_ARG, "null output");
    const hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail(WFSA_ERR_HIP, "hipSetDevice: %s", hipGetErrorString(e));
    std::string err;
    if (wfsa::peer_selftest(nranks, n, timeout_s, mode, out, err)) return fail(WFSA_ERR_HIP, "%s", err.c_str());
    return WFSA_OK;
}

}  // extern "C"

