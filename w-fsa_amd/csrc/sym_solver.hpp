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

private:
    double* a_ = nullptr;
    double* b_ = nullptr;
    double* diag_ = nullptr;   // [2 n]: D's diagonal and subdiagonal
    int32_t* ipiv_ = nullptr;
    void* ctl_ = nullptr;      // the factorisation's step state (sym_solver.hip BkCtl)
    int64_t n_ = 0, cap_ = 0;
    bool factored_ = false;
};

}  // namespace wfsa
