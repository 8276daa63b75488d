// Dense-automaton path (BASELINE.json configs[4], SURVEY.md 8d "c5"): when the
// transition matrix is dense, one trellis step of many strings at once is a
// GEMM against the N x N matrix exp(w) -- fp64 MFMA (v_mfma_f64_16x16x4f64).
//
// Model (reference semantics, SURVEY.md 8 "Exact semantics"): the start state
// `^` moves to state T and T emits the first byte; each later byte is a
// transition S->T followed by T's 1-byte emission; `$` is entered once the
// string is consumed.  With a[T] = exp(w(^->T)), A[S][T] = exp(w(S->T)),
// E[T][c] = exp(w(T emits c)), e[S] = exp(w(S->$)):
//   alpha_1 = a (.) E[:, s_0],  alpha_{j+1} = (alpha_j A) (.) E[:, s_j],
//   q = alpha_L . e,  beta_L = e,  beta_j = A (E[:, s_j] (.) beta_{j+1}),
// and the gradient of every parameter is minus its p-weighted posterior
// count (src/QuasiNewtonLearner.cpp:93-125): transitions
// A (.) sum_j alpha_j^T (E (.) beta_{j+1}) / q, emissions / start / end edges
// from gamma_j = alpha_j (.) beta_j / q.
//
// Layout in HBM: strings are packed back to back into R row slots (longest
// first, each to the least loaded slot), so trellis step t of the batch is one
// R x Np row block whatever the string lengths are; every GEMM has M = R.
// alpha, gamma and z (the scaled E (.) beta rows the gradient GEMM consumes)
// are kept for all T steps: T x R x Np doubles each.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "wfsa_dev.h"

namespace wfsa {

// Parameter codes of the dense tables: >= 0 Fsa parameter, kCodeNone no
// such edge (weight 0), kCodeOne an unequivocal edge (weight 1).
constexpr int32_t kCodeNone = -1;
constexpr int32_t kCodeOne = -2;
constexpr int kDenseTile = 128;   // GEMM block tile (rows and columns)

struct DenseModel {
    int32_t n_states = 0;          // interior states (not ^, not $)
    int32_t np = 0;                // n_states padded to kDenseTile
    int32_t vocab = 0;             // distinct emitted bytes
    int32_t n_params = 0;          // Fsa parameters (n_full)
    int16_t sym_of_byte[256];      // byte -> symbol index, vocab = not emitted
    std::vector<int32_t> code_a;   // [np][np] S->T
    std::vector<int32_t> code_s;   // [np] ^->T
    std::vector<int32_t> code_e;   // [np] S->$
    std::vector<int32_t> code_em;  // [vocab+1][np] T emits symbol v (row vocab: none)
    int32_t code_se = kCodeNone;   // ^->$ (the empty string)
    int64_t n_transitions = 0;     // interior S->T edges
};

// Builds the dense tables when the automaton qualifies: every state other
// than ^ and $ emits single bytes only (no epsilon, no multi-byte emission),
// and -- unless force -- at least a quarter of the interior transition matrix
// is present with >= 64 interior states.  Returns "" when dense, else why not.
std::string dense_model_build(const wfsa_model_desc& d, bool force, DenseModel& out);

class DensePath {
public:
    explicit DensePath(int n_cu) : n_cu_(n_cu > 0 ? n_cu : 256) {}
    ~DensePath();
    DensePath(const DensePath&) = delete;
    DensePath& operator=(const DensePath&) = delete;

    hipError_t load_model(const DenseModel& m, hipStream_t s);
    // packs the strings into row slots and allocates the per-step buffers
    hipError_t load_corpus(const uint8_t* sym, const int64_t* off, const double* p, int64_t n_strings,
                           hipStream_t s);
    // One evaluation: out[0] = sum_s p_s log q_s, out[1 + j] = -sum_s p_s
    // E[count_j | s] for every Fsa parameter (the context's out layout);
    // logq (nullable) per string in load order.  ewp[j] = exp(w_full[j]).
    // structural: all weights 1 and all p 1 (path counts and used
    // parameters, wfsa_dev_recognize).  halted (nullable): nonzero = skip.
    hipError_t enqueue(const double* ewp, bool structural, double* out, double* logq, const unsigned* halted,
                       hipStream_t s);
    // The rmin info column at the weights of the evaluation just enqueued
    // (src/QuasiNewtonLearner.cpp:80-84): res[0] = min over strings and
    // their paths of path probability / q, res[1] = the string holding it
    // (lowest index on ties), by a (min, +) trellis pass in the log domain
    // over the same row slots -- one tiled min-plus product per step on the
    // fp64 VALU (a semiring MFMA does not compute).  Empty strings (one path,
    // relative probability 1) are not candidates.
    hipError_t enqueue_rmin(double* res, const unsigned* halted, hipStream_t s);

    // the last evaluation ran at real weights (not the structural pass)
    bool weighted() const { return weighted_; }
    int64_t n_strings() const { return n_strings_; }
    int32_t rows() const { return R_; }
    int32_t steps() const { return T_; }
    int32_t np() const { return np_; }
    // the GEMM engine the evaluations run: 0 fused MFMA kernels, 1 rocBLAS
    // dgemm + epilogue kernels, 2 split-K MFMA kernels + epilogue kernels,
    // 3 LDS-DMA pipelined MFMA kernels + epilogue kernels
    int engine() const { return engine_ == 1 && !blas_ ? 0 : engine_; }
    int64_t total_symbols() const { return total_sym_; }
    // algorithmic fp64 flops of one evaluation: three GEMMs of 2 np^2 per
    // string position (forward, backward, gradient)
    double gemm_flops() const { return 6.0 * double(np_) * double(np_) * double(total_sym_); }
    // flops the GEMM launches execute (slot padding included)
    double issued_flops() const;

private:
    int n_cu_ = 256;
    int grad_cfg_ = 0;   // gradient GEMM: 4-wave blocks, K slices of 16, two blocks per CU (WFSA_DENSE_GRAD_CFG=1: 8-wave, 32; 65.7 vs 69.8 ms, profiles/r04/gemm_cfg_ab.txt)
    // WFSA_DENSE_STEP_CFG: 5 (default) engine 2's step GEMMs as 8-wave 128 x 128 blocks, 64 x 32 per wave,
    // two blocks per CU (c5 0.797 -> 0.814 of the fp64 peak, profiles/r05/c5_step_gemm_8wave.txt); timing
    // experiments: 0 the 4-wave blocks, 6 the gradient GEMM in 8-wave blocks too (0.80), 1 per-step GEMMs with
    // 4-wave blocks, 2 K slices of 16, 3 engine 2 with K slices of 32, 4 engine 3 with its own gradient GEMM
    int step_cfg_ = 5;
    int32_t n_params_ = 0, np_ = 0, vocab_ = 0, nct_ = 0;
    int32_t code_se_ = kCodeNone;
    int16_t sym_of_byte_[256] = {};
    int64_t n_strings_ = 0, total_sym_ = 0;
    int32_t R_ = 0, T_ = 0;
    bool weighted_ = false;
    int32_t ldx_ = 0;                  // row pitch of alpha / gamma / z / Y
    double p0_sum_ = 0.0, n0_ = 0.0;   // sum of p / count of empty strings
    int32_t reduce_chunks_ = 0;
    // model tables
    int32_t* code_a_ = nullptr;
    int32_t* code_s_ = nullptr;
    int32_t* code_e_ = nullptr;
    int32_t* code_em_ = nullptr;
    // per-iteration weights
    double* amat_ = nullptr;   // [np][np]
    double* amat_t_ = nullptr; // [np][np] transposed
    double* et_ = nullptr;     // [vocab+1][np]
    double* a0_ = nullptr;     // [np]
    double* aend_ = nullptr;   // [np]
    double* ones_ = nullptr;   // [n_params + 1] all ones (structural pass)
    // corpus: slots
    int32_t* meta_ = nullptr;  // [T][R] symbol | start << 9 | end << 10 (idle: symbol = vocab)
    int32_t* sid_ = nullptr;   // [T][R] string or -1
    int32_t* end_at_ = nullptr;  // [S] t * R + r of the string's last position, -1 if empty
    double* p_ = nullptr;      // [S]
    double* pones_ = nullptr;  // [S] all ones
    double* logq_ = nullptr;   // [S]
    double* la_ = nullptr;     // [T][R]
    double* lb_ = nullptr;     // [T][R]
    double* alpha_ = nullptr;  // [T][R][np]
    double* gam_ = nullptr;    // [T][R][np]
    double* z_ = nullptr;      // [T][R][np]
    double* y_ = nullptr;      // [2][R][np]
    double* part_ = nullptr;   // [2][nct][R]
    double* ll_part_ = nullptr;
    int32_t n_ll_ = 0;
    double* red_ = nullptr;    // [chunks][vocab+2][np]
    // GEMM engine (WFSA_DENSE_ENGINE=fused|blas|split|dma, default split;
    // WFSA_DENSE_BLAS=0/1 = fused/blas): 1 the GEMMs as plain fp64 library GEMMs (rocBLAS, atomics
    // off: deterministic) with our epilogue kernels; 2 the same flow with our
    // RAW GEMM kernel (K split in two halves: 2 blocks per CU) for the step
    // GEMMs and the fused gradient kernel; 0 the fused MFMA kernels above
    int engine_ = 2;
    void* blas_ = nullptr;     // rocblas_handle
    double* gbuf_ = nullptr;   // [np][np] the gradient GEMM's product (engine 1)
    double* ysplit_ = nullptr; // [R][ldx] the second K half's products (engine 2)
    // rmin pass (allocated by its first call): log tables (+inf: no edge),
    // two row-slot buffers of log min-path weights, per column tile and
    // string the end minima, per block the string minima
    double* lmat_ = nullptr;   // [np][np] log A
    double* let_ = nullptr;    // [vocab+1][np] log E^T
    double* l0_ = nullptr;     // [np] log a
    double* lend_ = nullptr;   // [np] log e
    double* mrow_ = nullptr;   // [2][R][np]
    double* spart_ = nullptr;  // [nct][S]
    double* rpart_ = nullptr;  // [2 * blocks]
    hipError_t enqueue_lib(const double* w, const double* p, bool structural, double* out, double* logq,
                           const unsigned* halted, hipStream_t s);
    void free_corpus();
    void free_model();
};

}  // namespace wfsa
