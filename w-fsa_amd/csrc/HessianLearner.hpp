// HessianLearner: host-side mirror of the reference's second-order optimizer
// (inc/HessianLearner.h:24-168, src/HessianLearner.cpp) over the device path.
//
// Each step solves the augmented (KKT) Newton system
//     [ H_g + H_f   J_g ] [dx]   [grad f + J_g lambda]
//     [ J_g^T        0  ] [dl] = [C^T exp(x) - 1     ]
// where grad f comes from the forward-backward kernels, H_f = -sum_s p_s Cov_s
// (the count covariance of each string's paths) from the per-bubble
// second-order kernel (wfsa_dev_hf_eval), and H_g / J_g are diagonal /
// one-entry-per-row.  MKL DSS (symmetric indefinite factorisation, inertia,
// determinant) is replaced by a dense Bunch-Kaufman LDL^T -- on the host for
// small systems, in HBM (wfsa_dev_sym_factor) for large ones up to kMaxDense
// unknowns -- and a sparse LDL^T (SparseLdlt.hpp) where its fill is small or
// the system exceeds the dense limit.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "Learner.hpp"
#include "SparseLdlt.hpp"

namespace wfsa {

// Symmetric indefinite LDL^T with Bunch-Kaufman partial pivoting (1x1 and
// 2x2 pivots) of a dense matrix: P A P^T = L D L^T.  Gives the inertia and
// the determinant (dss_statistics "Inertia" / "Determinant",
// src/HessianLearner.cpp:303, src/Utils.cpp:344) and solves.
class DenseLdlt {
public:
    // a: n x n row-major, symmetric (both triangles); consumed
    void Factor(std::vector<double>& a, int64_t n);
    void Solve(const double* b, double* x) const;
    int64_t positive = 0, negative = 0, zero = 0;
    double log_abs_det = 0.0;
    int det_sign = 1;

private:
    int64_t n_ = 0;
    std::vector<double> a_;        // L strictly below the pivots, D on the pivot blocks
    std::vector<int64_t> perm_;    // position i holds original index perm_[i]
    std::vector<int8_t> block_;    // 1: 1x1 pivot, 2: first of a 2x2, 0: second of a 2x2
};

class HessianLearner : public Learner {
public:
    // n + k of the augmented system: factored on the host (Bunch-Kaufman
    // LDL^T) up to kHostDense, above that in HBM (sym_solver.hip, our own
    // Bunch-Kaufman kernels +
    // wfsa_dev_sym_solve) up to kMaxDense (17 GB of fp64); WFSA_KKT=host /
    // device forces one side
    static constexpr int64_t kHostDense = 1024;
    static constexpr int64_t kMaxDense = 46000;
    // above kHostDense the sparse LDL^T (SparseLdlt.hpp, multifrontal with
    // scalar host fronts at ~1 GFLOP/s) takes systems whose factor costs at
    // most this many flops -- below the dense factorisation in HBM (0.5 s at
    // N = 10k; c3's KKT system fills in too much for the sparse one) -- and
    // every system beyond kMaxDense; WFSA_KKT=sparse forces it
    static constexpr double kSparseFlops = 3e8;
    // a sparse factorisation whose smallest pivot is below this fraction of
    // its row's largest entry leaves the inertia's sign there to rounding
    // (threshold pivots allow more growth than full Bunch-Kaufman): such a
    // system goes to the dense factorisation when it fits
    static constexpr double kSparsePivotFloor = 1e-9;
    char LastKktKind() const { return kkt_kind; }   // h / d / s: the last step's factorisation

    void OptimizationStep(double eta = 1.0, bool verbose = false) override;
    std::vector<double> GetOptimizationInfo() override;      // 9 values
    std::string GetOptimizationHeader() const override;
    std::vector<double> GetOptimizationResult(bool verbose = false) override;
    bool HaltCondition(double tol) override;

    void ComputeExpX();
    void ComputeGrad();
    double ComputeLogDetHessian(bool verbose = false);
    const std::vector<double>& GetGradient() const { return grad; }
    const std::vector<double>& GetLambda() const { return lambda; }
    std::vector<double> GetLagrangeMultipliers() const override { return lambda; }
    void SetLambda(const double* l) { lambda.assign(l, l + lambda.size()); }

protected:
    void FinalizeCallback() override;
    void InitCallback(int flags) override;

private:
    void InitSlackVariables();
    void ComputeRhs();
    void SetupHf();
    // A += -sum_s p_s Cov_s at the current x, on the trimmed parameters
    // (per_weight: over exp(x_j) exp(x_k), the weight-space Hessian); returns
    // whether the pattern has off-diagonal entries
    bool AddHf(SymEntries& A, bool per_weight);
    void PrintKkt(FILE* f, const SymEntries& A, bool with_hf, bool with_jg,
                  const std::vector<double>* rhs_print);
    SymEntries log_det_h;   // the last log-det Hessian, kept for PrintH (verbose)

    std::vector<double> rhs, expx, grad, lambda, step;
    std::vector<int32_t> hf_j, hf_k;   // trimmed indices of the pattern (-1: not a variable)
    std::vector<double> hf_vals, w_hf;
    bool hf_ready = false, include_Hf = false, degenerate = false, exponential_lambda = false, reorder = false;
    char kkt_kind = 0;
    double error = 0.0, lambda_min = 0.0;
    double rmin[2] = {0.0, 0.0};   // rmin column at the step's x
    int64_t inertia_pos = 0, inertia_neg = 0;
};

}  // namespace wfsa
