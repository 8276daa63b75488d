// Sparse symmetric-indefinite LDL^T for the HessianLearner's KKT system: MKL
// DSS's role (dss_define_structure / dss_reorder / dss_factor_real /
// dss_solve_real, src/HessianLearner.cpp:28-57,100-113; inertia and
// determinant through dss_statistics, :303, src/Utils.cpp:344).
//
// The KKT matrix [[H_g + H_f, J_g], [J_g^T, 0]] is very sparse: H_f holds the
// equivocal pairs, J_g one entry per parameter row.  The factorisation is
// multifrontal and supernodal, like the PARDISO solver behind DSS:
//   * a fill-reducing order -- the identity (the reference's
//     MKL_DSS_MY_ORDER with perm = 0..N-1), exact minimum degree, or
//     approximate minimum degree on the quotient graph (init flag 16, the
//     reference's METIS ordering) -- in which a row with a zero diagonal (a
//     constraint) becomes eligible only once a neighbour is eliminated;
//   * the elimination tree, its postorder and column counts, fundamental
//     supernodes (a chain of columns with nested structure);
//   * per supernode, in postorder: a dense frontal matrix assembled from the
//     entries and the children's update matrices (extend-add), partially
//     factorised with Bunch-Kaufman 1x1 / 2x2 pivots chosen among its fully
//     summed columns and accepted under a threshold test over the whole
//     front column (multipliers at most 1 / u, u = 0.1); columns with no
//     acceptable pivot are delayed -- handed, with the Schur complement, to
//     the parent's front, where they are fully summed again (MA57's
//     threshold pivoting with delayed pivots; PARDISO perturbs such pivots
//     instead), and a root's front pivots over its whole remaining matrix.
// Inertia and log|det| come from the D blocks (Sylvester).  SolveRefined adds
// iterative refinement; the caller checks every solve's residual and falls
// back to the dense factorisation when it is off.
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
    enum Order { kIdentity = 0, kMinimumDegree = 1, kApproxMinimumDegree = 2 };
    // the pattern of a (values ignored), the ordering and the symbolic
    // factorisation.  false: the ordering's work bound was exceeded (the
    // identity is used instead, still valid)
    bool Analyze(const SymEntries& a, int order);
    // numeric factorisation of a (same pattern as Analyze's); false: a zero
    // or non-finite pivot
    bool Factor(const SymEntries& a);
    void Solve(const double* b, double* x) const;
    // Solve, then up to max_steps of iterative refinement against a (as
    // PARDISO does after a pivot it could not make stable), kept while the
    // normwise backward error falls; the steps taken
    int SolveRefined(const SymEntries& a, const double* b, double* x, int max_steps = 2) const;

    int64_t positive = 0, negative = 0, zero = 0;
    double log_abs_det = 0.0;
    int det_sign = 1;
    double min_pivot_ratio = 0.0;   // min over pivots of |pivot| / max |A(k, :)|
    int64_t nnz_l = 0;              // strictly below the diagonal (the supernodal factor's stored entries)
    double flops = 0.0;             // sum over columns of (count of L)^2: the factor's work
    int64_t supernodes = 0, two_by_two = 0, max_front = 0, delayed = 0;   // delayed: columns passed up
    std::vector<int32_t> perm;      // perm[new] = old

private:
    struct Super {
        int32_t first = 0, ncol = 0;     // columns [first, first + ncol) of the postordered matrix
        std::vector<int32_t> rows;       // front rows: the ncol columns, then the structure below
        int32_t parent = -1;
    };
    struct Front {                       // a factorised supernode
        std::vector<int32_t> rows;       // the front's rows in pivot order: the nelim eliminated, then the rest
        int32_t nelim = 0;
        std::vector<int8_t> piv;         // 1: 1x1 pivot, 2: first of a 2x2, 0: its second
        std::vector<double> d;           // [nelim][2]: d11 / d21 of the pivot block at t (2x2: d22 at t + 1)
        std::vector<double> l;           // m x nelim column-major, unit lower (2x2 blocks: identity)
    };
    int64_t n_ = 0;
    std::vector<int32_t> pinv_;          // pinv[old] = new (postordered)
    std::vector<Super> sn_;
    std::vector<Front> fr_;
};

// minimum-degree orderings of the graph of a (perm[new] = old); false when
// the work bound is exceeded
bool minimum_degree_order(const SymEntries& a, std::vector<int32_t>& perm, double work_bound = 4e8);
bool approximate_minimum_degree_order(const SymEntries& a, std::vector<int32_t>& perm);

}  // namespace wfsa
