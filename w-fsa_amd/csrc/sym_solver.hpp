// Dense symmetric-indefinite factorisation on the device for the
// HessianLearner's KKT system (the reference factors it with MKL DSS,
// src/HessianLearner.cpp:28-57,100-113; log-det src/Utils.cpp:296-350).
// Bunch-Kaufman LDL^T (LAPACK dsytf2 semantics, lower, column-major) by our
// own kernels in HBM -- an (n+k)^2 fp64 matrix of 40k unknowns is 12.8 GB,
// well inside 288 GB; rocSOLVER's dsytrf took 118 s at n = 10k -- then the
// inertia and log|det| from D's 1x1 / 2x2 blocks (2n values and the pivots
// come back, not the factor) and the solve by a one-workgroup kernel running
// LAPACK dsytrs' two sweeps with the column updates spread over 1024 lanes.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace wfsa {

struct SymFactor {
    int64_t positive = 0, negative = 0, zero = 0;
    double log_abs_det = 0.0;
    int det_sign = 1;
};

class SymSolver {
public:
    SymSolver() = default;
    ~SymSolver();
    SymSolver(const SymSolver&) = delete;
    SymSolver& operator=(const SymSolver&) = delete;

    // a: n x n symmetric (row- or column-major: both triangles equal).
    // Returns a HIP failure as a message (null on success).
    const char* factor(const double* a, int64_t n, hipStream_t s, SymFactor* out);
    // b[n] in place: x = A^-1 b with the last factorisation
    const char* solve(double* b, hipStream_t s);

    // The same from the matrix's entries (upper-triangle coordinates, i <= j,
    // duplicates add), assembled in HBM: the blocked factorisation
    // (sym_blocked.hip) first; when it takes a pivot under its threshold,
    // shows element growth, or -- with b -- its solve does not refine to a
    // backward error of 1e-12 against the entries, the full Bunch-Kaufman
    // factorisation instead (the result then is the one above).  b (nullable)
    // is solved in place; *method = 1 blocked, 2 full Bunch-Kaufman.
    const char* factor_coo(int64_t n, int64_t nnz, const int32_t* i, const int32_t* j, const double* v, double* b,
                           hipStream_t s, SymFactor* out, int* method);
    double last_growth() const { return last_growth_; }

private:
    const char* alloc(int64_t n);
    const char* bk_factor_device(hipStream_t s, SymFactor* out);   // dsytf2 on a_ as it stands
    // sym_blocked.hip
    const char* ensure_blocked(int64_t n, hipStream_t s);
    const char* assemble(hipStream_t s);
    const char* blocked_factor(hipStream_t s, SymFactor* out, bool* exact);
    const char* blocked_solve(hipStream_t s);
    // r = b - A x over the host entries; false when the backward error per row
    // exceeds tol (|r_i| <= tol (|A||x| + |b|)_i)
    bool residual(const double* b, const double* x, double* r, double tol) const;

    double* a_ = nullptr;
    double* b_ = nullptr;
    double* diag_ = nullptr;   // [2 n]: D's diagonal and subdiagonal
    int32_t* ipiv_ = nullptr;
    void* ctl_ = nullptr;      // the factorisation's step state (sym_solver.hip BkCtl)
    int64_t n_ = 0, cap_ = 0;
    bool factored_ = false;
    // blocked factorisation
    void* blas_ = nullptr;     // rocblas_handle
    double *y_ = nullptr, *bd_ = nullptr, *gmax_ = nullptr, *x_ = nullptr;
    int32_t *perm_ = nullptr, *bpiv_ = nullptr, *bstat_ = nullptr;
    void* coo_ = nullptr;
    size_t coo_bytes_ = 0;
    int64_t bcap_ = 0;
    double last_growth_ = 0.0;
    bool blocked_ok_ = false;            // the last factorisation is the blocked one
    std::vector<int32_t> crow_, ccol_;   // the unique lower entries (row >= col)
    std::vector<double> cval_;
};

}  // namespace wfsa
