// Matrix-file mode (Learner::LoadMatrices,
// src/Learner.cpp:125-199, main.cpp -m "<file"): no automaton, the learner
// is handed the path matrices the reference's BuildPaths would have built --
// P (paths x parameters, counts), M (strings x paths, ones), C, p -- and the
// objective is the reference's own SpMV chain (ComputeModeledProbs
// src/Learner.cpp:515-547, ComputeGrad src/QuasiNewtonLearner.cpp:93-125):
//   lw = P x,  log q_s = logsumexp_{l in M_s} lw_l,  rpp_l = exp(lw_l - log q_s),
//   grad = -P^T (rpp (.) M^T p).
// On the device: a path per lane for P x (row walk), a string per lane for the
// log-sum-exp and the coefficients -p_s rpp_l, and a parameter per lane over
// P^T (built once at load) for the gradient -- fixed order throughout (no
// atomics: deterministic).  The string pass also takes the block minima of
// the relative path probabilities of ambiguous strings with their path index
// -- the rmin column exactly as the reference reports it.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace wfsa {

class MatrixPath {
public:
    MatrixPath() = default;
    ~MatrixPath();
    MatrixPath(const MatrixPath&) = delete;
    MatrixPath& operator=(const MatrixPath&) = delete;

    // prow[n_paths+1], pcol/pdata[prow[n_paths]]; mrow[n_strings+1],
    // mcol[mrow[n_strings]] (path indices); p[n_strings].  Validated by the
    // caller.  Host copies of the per-string path counts and the used
    // parameters are kept for the structural queries.
    hipError_t load(int32_t n_params, int64_t n_paths, const int64_t* prow, const int32_t* pcol, const double* pdata,
                    int64_t n_strings, const int64_t* mrow, const int64_t* mcol, const double* p, hipStream_t s);
    // out[0] = sum_s p_s log q_s, out[1 + j] = grad_j; logq nullable;
    // w[n_params] = x.  halted (nullable): nonzero = skip.
    hipError_t enqueue(const double* w, double* out, double* logq, const unsigned* halted, hipStream_t s);
    // rmin of the last enqueue: res[0] = min relative path probability over
    // ambiguous strings, res[1] = its path index (-1: none)
    hipError_t enqueue_rmin(double* res, const unsigned* halted, hipStream_t s);

    // H_f over the paths (HessianLearner::AssembleH :381-446 + ComputeHf
    // :498-547): setup lists the pattern pairs (j <= k, ascending) of the
    // parameters whose counts differ between a string's paths; hf_eval runs
    // the evaluation at w and writes out[t] = sum_s p_s Cov_s(c_j, c_k) for
    // pattern pair t (a lane per (string, pair) slot, then a lane per pair
    // summing its slots in order).
    hipError_t hf_setup(std::vector<int32_t>& pairs, hipStream_t s);
    hipError_t hf_eval(const double* w, double* out, hipStream_t s);

    const std::vector<double>& path_counts() const { return h_counts_; }
    const std::vector<uint8_t>& used() const { return h_used_; }
    int64_t n_paths() const { return n_paths_; }

private:
    void release();
    int32_t n_params_ = 0;
    int64_t n_paths_ = 0, n_strings_ = 0;
    int blocks_s_ = 0;
    int64_t* prow_ = nullptr;
    int32_t* pcol_ = nullptr;
    double* pdata_ = nullptr;
    int64_t* mrow_ = nullptr;
    int64_t* mcol_ = nullptr;
    double* p_ = nullptr;
    int64_t* trow_ = nullptr;    // P^T (CSR over parameters): rows, path ids, counts
    int64_t* tcol_ = nullptr;
    double* tdata_ = nullptr;
    double* lw_ = nullptr;       // [n_paths] P x, then -p_s rpp_l
    double* part_ = nullptr;     // [blocks_s][3]: sum p log q, min rpp, its path
    double* rpp_ = nullptr;      // [n_paths] relative path probabilities of the last evaluation
    std::vector<double> h_counts_;
    std::vector<uint8_t> h_used_;
    // host copies for the H_f pattern
    std::vector<int64_t> h_prow_, h_mrow_, h_mcol_;
    std::vector<int32_t> h_pcol_;
    std::vector<double> h_pdata_;
    // H_f tables: per equivocal string (table offset, paths, equivocal params,
    // first M entry), its dense count table, the slots (string, a, b), and
    // the pair -> slots CSR
    int4* hf_str_ = nullptr;
    double* hf_tab_ = nullptr;
    int4* hf_slot_ = nullptr;
    int64_t* hf_tptr_ = nullptr;
    int64_t* hf_tslot_ = nullptr;
    double* hf_val_ = nullptr;
    int64_t hf_n_slots_ = 0, hf_n_pairs_ = 0;
};

}  // namespace wfsa
