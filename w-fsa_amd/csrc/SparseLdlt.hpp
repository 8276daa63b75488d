// Sparse symmetric LDL^T for the HessianLearner's KKT system: MKL DSS's
// role (dss_define_structure / dss_reorder / dss_factor_real /
// dss_solve_real, src/HessianLearner.cpp:28-57,100-113; inertia and
// determinant through dss_statistics, :303, src/Utils.cpp:344).
//
// The KKT matrix [[H_g + H_f, J_g], [J_g^T, 0]] is very sparse: H_f holds the
// equivocal pairs, J_g one entry per parameter row.  The factorisation is
// up-looking (row k of L from a sparse triangular solve over the elimination
// tree), with 1x1 pivots in a static order: the identity (the reference's
// MKL_DSS_MY_ORDER with perm = 0..N-1) or, for init flag 16 (the reference's
// METIS ordering), our own minimum-degree ordering.  Without pivoting a tiny
// pivot can lose accuracy, so Factor reports the smallest pivot ratio and the
// caller checks the residual of every solve (HessianLearner falls back to the
// dense Bunch-Kaufman factorisation when either fails).
#pragma once

#include <cstdint>
#include <vector>

namespace wfsa {

// symmetric matrix as upper-triangle coordinates (i <= j); duplicates add
struct SymEntries {
    int64_t n = 0;
    std::vector<int32_t> i, j;
    std::vector<double> v;
    explicit SymEntries(int64_t n_ = 0) : n(n_) {}
    void add(int64_t a, int64_t b, double x) {
        if (a > b) std::swap(a, b);
        i.push_back(int32_t(a));
        j.push_back(int32_t(b));
        v.push_back(x);
    }
    // dense row-major n x n, both triangles
    std::vector<double> dense() const;
    // y = A x
    void multiply(const double* x, double* y) const;
};

class SparseLdlt {
public:
    // the pattern of a (values ignored) and the ordering: 0 identity, 1
    // minimum degree.  false: the ordering's work bound was exceeded (the
    // identity is used instead, still valid)
    bool Analyze(const SymEntries& a, int order);
    // numeric factorisation of a (same pattern as Analyze's); false: a zero or
    // non-finite pivot
    bool Factor(const SymEntries& a);
    void Solve(const double* b, double* x) const;

    int64_t positive = 0, negative = 0, zero = 0;
    double log_abs_det = 0.0;
    int det_sign = 1;
    double min_pivot_ratio = 0.0;   // min_k |d_k| / max |A(k, :)| over the pivots
    int64_t nnz_l = 0;              // strictly below the diagonal
    double flops = 0.0;             // sum over columns of (count of L)^2: the factor's work
    std::vector<int32_t> perm;      // perm[new] = old

private:
    int64_t n_ = 0;
    std::vector<int32_t> pinv_;                // pinv[old] = new
    std::vector<int64_t> ap_;                  // permuted upper pattern by column: rows < k of column k
    std::vector<int32_t> ai_;
    std::vector<int64_t> src_;                 // entry of a feeding each (ap_, ai_) slot; diagonal slots too
    std::vector<int64_t> dp_;                  // per column: entries of a on the diagonal, [dp_[k], dp_[k+1]) in dsrc_
    std::vector<int64_t> dsrc_;
    std::vector<int32_t> parent_, lnz_;
    std::vector<int64_t> lp_;
    std::vector<int32_t> li_;
    std::vector<double> lx_, d_;
};

// minimum-degree ordering of the graph of a (perm[new] = old); false when the
// work bound is exceeded
bool minimum_degree_order(const SymEntries& a, std::vector<int32_t>& perm, double work_bound = 4e8);

}  // namespace wfsa
