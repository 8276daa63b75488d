// Dense symmetric-indefinite LDL^T on the device (sym_solver.hpp).
#include "sym_solver.hpp"

#include <rocblas/rocblas.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

namespace wfsa {
namespace {

constexpr int kSolveBlock = 1024;

__global__ void diag_kernel(const double* __restrict__ a, int64_t n, double* __restrict__ d) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    d[k] = a[k * n + k];
    d[n + k] = k + 1 < n ? a[k * n + k + 1] : 0.0;   // column k, row k+1 (lower)
}

// Bunch-Kaufman LDL^T, lower, column-major (LAPACK dsytf2 semantics: the
// same pivot choices, interchanges, D blocks and 1-based ipiv).  Right-looking
// and unblocked: per pivot step one single-workgroup kernel chooses the pivot
// and applies the interchange (O(n)), one grid kernel applies the rank-1/2
// update to the trailing lower triangle (a block per column: coalesced along
// the column, bound by HBM -- sum over steps ~ n^3/6 x 16 B), one
// single-workgroup kernel writes the multipliers and advances k.  The step
// state lives on the device, so the host enqueues n steps blindly (a 2x2
// pivot consumes two columns; surplus steps exit at once).
struct BkCtl {
    int64_t k;        // next column
    int64_t kstep;    // 1 or 2 for the step in progress
    int64_t kp;
    int64_t info;     // first zero pivot column + 1 (0: none)
    double r;         // 1 / d (1x1)
    double d11, d22, d21;   // 2x2 scalars (dsytf2)
};

constexpr int kPivBlock = 1024;

__device__ void argmax_abs(double v, int64_t i, double* rv, int64_t* ri, double& out_v, int64_t& out_i) {
    // block argmax of |v| (first index on ties, as idamax)
    double a = fabs(v);
    for (int o = 32; o > 0; o >>= 1) {
        const double b = __shfl_xor(a, o, 64);
        const int64_t j = __shfl_xor(i, o, 64);
        if (b > a || (b == a && j < i)) {
            a = b;
            i = j;
        }
    }
    const int w = int(threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) {
        rv[w] = a;
        ri[w] = i;
    }
    __syncthreads();
    a = rv[0];
    i = ri[0];
    for (int q = 1; q < int(blockDim.x) / 64; ++q)
        if (rv[q] > a || (rv[q] == a && ri[q] < i)) {
            a = rv[q];
            i = ri[q];
        }
    __syncthreads();
    out_v = a;
    out_i = i;
}

__global__ __launch_bounds__(kPivBlock) void bk_pivot_kernel(double* a, int64_t n, int32_t* ipiv, BkCtl* ctl) {
    __shared__ double rv[kPivBlock / 64];
    __shared__ int64_t ri[kPivBlock / 64];
    const int64_t k = ctl->k;
    if (k >= n) return;
    const int t = int(threadIdx.x);
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    const double* ck = a + k * n;
    const double absakk = fabs(ck[k]);
    double colmax = 0.0;
    int64_t imax = k;
    {
        double v = 0.0;
        int64_t vi = n;
        for (int64_t i = k + 1 + t; i < n; i += kPivBlock)
            if (fabs(ck[i]) > fabs(v) || vi == n) {
                v = ck[i];
                vi = i;
            }
        argmax_abs(v, vi, rv, ri, colmax, imax);
        if (imax >= n) {
            colmax = 0.0;
            imax = k;
        }
    }
    int64_t kp = k, kstep = 1;
    if (fmax(absakk, colmax) == 0.0) {
        if (t == 0 && ctl->info == 0) ctl->info = k + 1;
    } else if (!(absakk >= alpha * colmax)) {
        // largest off-diagonal in row / column imax
        double v = 0.0;
        int64_t vi = n;
        for (int64_t j = k + t; j < imax; j += kPivBlock) {   // row imax, columns k..imax-1
            const double x = a[j * n + imax];
            if (fabs(x) > fabs(v) || vi == n) {
                v = x;
                vi = j;
            }
        }
        for (int64_t i = imax + 1 + t; i < n; i += kPivBlock) {   // column imax below the diagonal
            const double x = a[imax * n + i];
            if (fabs(x) > fabs(v) || vi == n) {
                v = x;
                vi = i;
            }
        }
        double rowmax;
        int64_t jm;
        argmax_abs(v, vi, rv, ri, rowmax, jm);
        if (absakk >= alpha * colmax * (colmax / rowmax)) {
            kp = k;
        } else if (fabs(a[imax * n + imax]) >= alpha * rowmax) {
            kp = imax;
        } else {
            kp = imax;
            kstep = 2;
        }
    }
    const int64_t kk = k + kstep - 1;
    if (kp != kk) {   // interchange rows and columns kk and kp of the trailing matrix
        double* ckk = a + kk * n;
        double* ckp = a + kp * n;
        for (int64_t i = kp + 1 + t; i < n; i += kPivBlock) {
            const double x = ckk[i];
            ckk[i] = ckp[i];
            ckp[i] = x;
        }
        for (int64_t j = kk + 1 + t; j < kp; j += kPivBlock) {
            const double x = ckk[j];
            ckk[j] = a[j * n + kp];
            a[j * n + kp] = x;
        }
        __syncthreads();
        if (t == 0) {
            double x = ckk[kk];
            ckk[kk] = ckp[kp];
            ckp[kp] = x;
            if (kstep == 2) {
                x = a[k * n + k + 1];
                a[k * n + k + 1] = a[k * n + kp];
                a[k * n + kp] = x;
            }
        }
    }
    __syncthreads();
    if (t == 0) {
        ctl->kstep = kstep;
        ctl->kp = kp;
        if (kstep == 1) {
            ipiv[k] = int32_t(kp + 1);
            const double d = a[k * n + k];
            ctl->r = d != 0.0 ? 1.0 / d : 0.0;   // a zero column: no update (dsytf2 skips it)
        } else {
            ipiv[k] = ipiv[k + 1] = -int32_t(kp + 1);
            const double d21 = a[k * n + k + 1];
            const double d11 = a[(k + 1) * n + k + 1] / d21;
            const double d22 = a[k * n + k] / d21;
            const double tt = 1.0 / (d11 * d22 - 1.0);
            ctl->d11 = d11;
            ctl->d22 = d22;
            ctl->d21 = tt / d21;
        }
    }
}

// trailing update, block per column j = n - 1 - blockIdx.x (rows i >= j)
__global__ __launch_bounds__(256) void bk_update_kernel(double* a, int64_t n, const BkCtl* ctl) {
    const int64_t k = ctl->k;
    if (k >= n) return;
    const int64_t kstep = ctl->kstep;
    const int64_t j = n - 1 - int64_t(blockIdx.x);
    if (j < k + kstep) return;
    double* cj = a + j * n;
    const double* ck = a + k * n;
    if (kstep == 1) {
        const double f = ctl->r * ck[j];
        for (int64_t i = j + threadIdx.x; i < n; i += 256) cj[i] -= ck[i] * f;
    } else {
        const double* ck1 = a + (k + 1) * n;
        const double d21 = ctl->d21, d11 = ctl->d11, d22 = ctl->d22;
        const double wk = d21 * (d11 * ck[j] - ck1[j]);
        const double wkp1 = d21 * (d22 * ck1[j] - ck[j]);
        for (int64_t i = j + threadIdx.x; i < n; i += 256) cj[i] -= ck[i] * wk + ck1[i] * wkp1;
    }
}

// the multipliers into columns k (, k+1), then k += kstep
__global__ __launch_bounds__(kPivBlock) void bk_finish_kernel(double* a, int64_t n, BkCtl* ctl) {
    const int64_t k = ctl->k;
    if (k >= n) return;
    const int64_t kstep = ctl->kstep;
    double* ck = a + k * n;
    if (kstep == 1) {
        const double r = ctl->r;
        for (int64_t i = k + 1 + threadIdx.x; i < n; i += kPivBlock) ck[i] *= r;
    } else {
        double* ck1 = a + (k + 1) * n;
        const double d21 = ctl->d21, d11 = ctl->d11, d22 = ctl->d22;
        for (int64_t i = k + 2 + threadIdx.x; i < n; i += kPivBlock) {
            const double x = ck[i], y = ck1[i];
            ck[i] = d21 * (d11 * x - y);
            ck1[i] = d21 * (d22 * y - x);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) ctl->k = k + kstep;
}

__device__ double block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = int(threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double s = 0.0;
    for (int i = 0; i < kSolveBlock / 64; ++i) s += red[i];   // fixed order: every lane the same sum
    __syncthreads();
    return s;
}

// LAPACK dsytrs, uplo = 'L', one right-hand side; a column-major with lda =
// n, ipiv 1-based as dsytrf returns it.  One workgroup: the sweeps are
// sequential over the pivots, each column update / dot product is spread
// over the lanes.
__global__ __launch_bounds__(kSolveBlock) void sytrs_lower_kernel(const double* __restrict__ a, int64_t n,
                                                                   const int32_t* __restrict__ ipiv, double* b) {
    __shared__ double red[kSolveBlock / 64];
    const int t = int(threadIdx.x);
    // L D y = b
    for (int64_t k = 0; k < n;) {
        const int32_t p = ipiv[k];
        if (p > 0) {
            const int64_t kp = int64_t(p) - 1;
            if (t == 0 && kp != k) {
                const double x = b[k];
                b[k] = b[kp];
                b[kp] = x;
            }
            __syncthreads();
            const double bk = b[k];
            const double* col = a + k * n;
            for (int64_t i = k + 1 + t; i < n; i += kSolveBlock) b[i] -= col[i] * bk;
            __syncthreads();
            if (t == 0) b[k] = bk / col[k];
            __syncthreads();
            k += 1;
        } else {
            const int64_t kp = -int64_t(p) - 1;
            if (t == 0 && kp != k + 1) {
                const double x = b[k + 1];
                b[k + 1] = b[kp];
                b[kp] = x;
            }
            __syncthreads();
            const double b0 = b[k], b1 = b[k + 1];
            const double* c0 = a + k * n;
            const double* c1 = a + (k + 1) * n;
            for (int64_t i = k + 2 + t; i < n; i += kSolveBlock) b[i] -= c0[i] * b0 + c1[i] * b1;
            __syncthreads();
            if (t == 0) {
                const double akm1k = c0[k + 1];
                const double akm1 = c0[k] / akm1k, ak = c1[k + 1] / akm1k;
                const double denom = akm1 * ak - 1.0;
                const double bkm1 = b0 / akm1k, bk = b1 / akm1k;
                b[k] = (ak * bkm1 - bk) / denom;
                b[k + 1] = (akm1 * bk - bkm1) / denom;
            }
            __syncthreads();
            k += 2;
        }
    }
    // L^T x = y
    for (int64_t k = n - 1; k >= 0;) {
        const int32_t p = ipiv[k];
        if (p > 0) {
            double s = 0.0;
            const double* col = a + k * n;
            for (int64_t i = k + 1 + t; i < n; i += kSolveBlock) s += col[i] * b[i];
            s = block_sum(s, red);
            if (t == 0) {
                b[k] -= s;
                const int64_t kp = int64_t(p) - 1;
                if (kp != k) {
                    const double x = b[k];
                    b[k] = b[kp];
                    b[kp] = x;
                }
            }
            __syncthreads();
            k -= 1;
        } else {
            double s1 = 0.0, s0 = 0.0;
            const double* c1 = a + k * n;
            const double* c0 = a + (k - 1) * n;
            for (int64_t i = k + 1 + t; i < n; i += kSolveBlock) {
                s1 += c1[i] * b[i];
                s0 += c0[i] * b[i];
            }
            s1 = block_sum(s1, red);
            s0 = block_sum(s0, red);
            if (t == 0) {
                b[k] -= s1;
                b[k - 1] -= s0;
                const int64_t kp = -int64_t(p) - 1;
                if (kp != k) {
                    const double x = b[k];
                    b[k] = b[kp];
                    b[kp] = x;
                }
            }
            __syncthreads();
            k -= 2;
        }
    }
}

}  // namespace

SymSolver::~SymSolver() {
    for (void* p : {static_cast<void*>(a_), static_cast<void*>(b_), static_cast<void*>(diag_),
                    static_cast<void*>(ipiv_), static_cast<void*>(ctl_), static_cast<void*>(y_),
                    static_cast<void*>(bd_), static_cast<void*>(gmax_), static_cast<void*>(x_),
                    static_cast<void*>(perm_), static_cast<void*>(bpiv_), static_cast<void*>(bstat_), coo_})
        if (p) (void)hipFree(p);
    if (blas_) (void)rocblas_destroy_handle(static_cast<rocblas_handle>(blas_));
}

const char* SymSolver::alloc(int64_t n) {
    if (n >= (int64_t(1) << 31)) return "matrix too large";
    if (n <= cap_) return nullptr;
    for (void* p : {static_cast<void*>(a_), static_cast<void*>(b_), static_cast<void*>(diag_),
                    static_cast<void*>(ipiv_), static_cast<void*>(ctl_)})
        if (p) (void)hipFree(p);
    a_ = b_ = diag_ = nullptr;
    ipiv_ = nullptr;
    ctl_ = nullptr;
    cap_ = 0;
    if (hipMalloc(reinterpret_cast<void**>(&a_), size_t(n) * size_t(n) * sizeof(double)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&b_), size_t(n) * sizeof(double)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&diag_), 2 * size_t(n) * sizeof(double)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&ipiv_), size_t(n) * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&ctl_, sizeof(BkCtl)) != hipSuccess)
        return "device allocation failed";
    cap_ = n;
    return nullptr;
}

const char* SymSolver::factor(const double* a, int64_t n, hipStream_t s, SymFactor* out) {
    factored_ = false;
    blocked_ok_ = false;
    if (n <= 0) {
        *out = SymFactor{};
        return nullptr;
    }
    if (const char* e = alloc(n)) return e;
    n_ = n;
    if (hipMemcpyAsync(a_, a, size_t(n) * size_t(n) * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess)
        return "upload failed";
    return bk_factor_device(s, out);
}

const char* SymSolver::bk_factor_device(hipStream_t s, SymFactor* out) {
    const int64_t n = n_;
    if (hipMemsetAsync(ctl_, 0, sizeof(BkCtl), s) != hipSuccess) return "memset failed";
    BkCtl* ctl = static_cast<BkCtl*>(ctl_);
    for (int64_t step = 0; step < n; ++step) {   // each step takes >= 1 column: n steps suffice
        hipLaunchKernelGGL(bk_pivot_kernel, dim3(1), dim3(kPivBlock), 0, s, a_, n, ipiv_, ctl);
        hipLaunchKernelGGL(bk_update_kernel, dim3(unsigned(n - step)), dim3(256), 0, s, a_, n, ctl);
        hipLaunchKernelGGL(bk_finish_kernel, dim3(1), dim3(kPivBlock), 0, s, a_, n, ctl);
    }
    if (hipGetLastError() != hipSuccess) return "factorisation launch failed";
    hipLaunchKernelGGL(diag_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, a_, n, diag_);
    std::vector<double> d(2 * size_t(n));
    std::vector<int32_t> piv(static_cast<size_t>(n));
    if (hipMemcpyAsync(d.data(), diag_, d.size() * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(piv.data(), ipiv_, piv.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return "download failed";
    SymFactor f;
    for (int64_t k = 0; k < n;) {
        if (piv[size_t(k)] > 0) {
            const double v = d[size_t(k)];
            if (v > 0.0) ++f.positive;
            else if (v < 0.0) ++f.negative;
            else ++f.zero;
            if (v < 0.0) f.det_sign = -f.det_sign;
            f.log_abs_det += std::log(std::fabs(v));
            k += 1;
        } else {
            const double x = d[size_t(k)], y = d[size_t(n + k)], z = d[size_t(k) + 1];
            const double det = x * z - y * y;
            if (det < 0.0) {
                ++f.positive;
                ++f.negative;
                f.det_sign = -f.det_sign;
            } else if (det > 0.0) {
                (x + z > 0.0 ? f.positive : f.negative) += 2;
            } else {
                f.zero += 2;
            }
            f.log_abs_det += std::log(std::fabs(det));
            k += 2;
        }
    }
    *out = f;
    factored_ = true;
    return nullptr;
}

bool SymSolver::residual(const double* b, const double* x, double* r, double tol) const {
    const int64_t n = n_;
    std::vector<double> mag(static_cast<size_t>(n), 0.0);
    for (int64_t i = 0; i < n; ++i) r[i] = b[i];
    for (size_t t = 0; t < cval_.size(); ++t) {
        const int64_t i = crow_[t], j = ccol_[t];
        const double v = cval_[t];
        r[i] -= v * x[j];
        mag[size_t(i)] += std::fabs(v * x[j]);
        if (i != j) {
            r[j] -= v * x[i];
            mag[size_t(j)] += std::fabs(v * x[i]);
        }
    }
    bool ok = true;
    for (int64_t i = 0; i < n && ok; ++i) ok = std::isfinite(r[i]) && std::fabs(r[i]) <= tol * (mag[size_t(i)] + std::fabs(b[i]));
    return ok;
}

// componentwise backward error the blocked factor's refined solve must meet
// (the bar HessianLearner.cpp sets for the host sparse LDL^T); a factor that misses it is
// replaced by the full Bunch-Kaufman (WFSA_KKT_TRACE logs that)
constexpr double kRefineTol = 1e-9;

const char* SymSolver::factor_coo(int64_t n, int64_t nnz, const int32_t* ei, const int32_t* ej, const double* ev,
                                  double* b, hipStream_t s, SymFactor* out, int* method) {
    factored_ = false;
    blocked_ok_ = false;
    if (method) *method = 0;
    if (n <= 0) {
        *out = SymFactor{};
        return nullptr;
    }
    if (const char* e = alloc(n)) return e;
    n_ = n;
    // unique lower entries (row = max, col = min), duplicates summed in a fixed order
    {
        std::vector<int64_t> key(static_cast<size_t>(nnz));
        std::vector<int64_t> ord(static_cast<size_t>(nnz));
        for (int64_t t = 0; t < nnz; ++t) {
            const int64_t r = std::max(ei[t], ej[t]), c = std::min(ei[t], ej[t]);
            if (c < 0 || r >= n) return "entry out of range";
            key[size_t(t)] = c * n + r;
            ord[size_t(t)] = t;
        }
        std::stable_sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) { return key[size_t(x)] < key[size_t(y)]; });
        crow_.clear();
        ccol_.clear();
        cval_.clear();
        for (int64_t q = 0; q < nnz; ++q) {
            const int64_t t = ord[size_t(q)];
            if (q > 0 && key[size_t(t)] == key[size_t(ord[size_t(q) - 1])]) {
                cval_.back() += ev[t];
            } else {
                crow_.push_back(int32_t(key[size_t(t)] % n));
                ccol_.push_back(int32_t(key[size_t(t)] / n));
                cval_.push_back(ev[t]);
            }
        }
    }
    {   // the blocked factorisation first; the full Bunch-Kaufman below where it is not exact
        if (const char* e = ensure_blocked(n, s)) return e;
        if (const char* e = assemble(s)) return e;
        bool exact = false;
        SymFactor f;
        if (const char* e = blocked_factor(s, &f, &exact)) return e;
        if (exact) {
            bool ok = true;
            if (b) {   // solve, refine (up to 3 corrections) and check
                std::vector<double> rhs(b, b + n), x(static_cast<size_t>(n)), r(static_cast<size_t>(n));
                auto dev_solve = [&](const double* in, double* outv) -> const char* {
                    if (hipMemcpyAsync(b_, in, size_t(n) * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess)
                        return "upload failed";
                    if (const char* e = blocked_solve(s)) return e;
                    if (hipMemcpyAsync(outv, b_, size_t(n) * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
                        hipStreamSynchronize(s) != hipSuccess)
                        return "download failed";
                    return nullptr;
                };
                if (const char* e = dev_solve(rhs.data(), x.data())) return e;
                ok = residual(rhs.data(), x.data(), r.data(), kRefineTol);
                for (int it = 0; it < 3 && !ok; ++it) {
                    std::vector<double> dx(static_cast<size_t>(n));
                    if (const char* e = dev_solve(r.data(), dx.data())) return e;
                    for (int64_t q = 0; q < n; ++q) x[size_t(q)] += dx[size_t(q)];
                    ok = residual(rhs.data(), x.data(), r.data(), kRefineTol);
                }
                if (ok) std::copy(x.begin(), x.end(), b);
            }
            if (ok) {
                *out = f;
                if (method) *method = 1;
                blocked_ok_ = true;
                return nullptr;
            }
        }
        if (std::getenv("WFSA_VERBOSE"))
            std::fprintf(stderr, "[kkt] n %lld: blocked factor %s; the full Bunch-Kaufman instead\n", (long long)n,
                         exact ? "missed the refined residual bound" : "hit a pivot it cannot take");
    }
    // the full Bunch-Kaufman (LAPACK dsytf2 semantics) on the assembled matrix
    if (const char* e = ensure_blocked(n, s)) return e;
    if (const char* e = assemble(s)) return e;
    if (const char* e = bk_factor_device(s, out)) return e;
    if (method) *method = 2;
    if (b) return solve(b, s);
    return nullptr;
}

const char* SymSolver::solve(double* b, hipStream_t s) {
    if (blocked_ok_) {   // the blocked factor: solve, then refine against the entries
        const int64_t n = n_;
        std::vector<double> rhs(b, b + n), x(static_cast<size_t>(n)), r(static_cast<size_t>(n));
        auto dev_solve = [&](const double* in, double* outv) -> const char* {
            if (hipMemcpyAsync(b_, in, size_t(n) * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess)
                return "upload failed";
            if (const char* e = blocked_solve(s)) return e;
            if (hipMemcpyAsync(outv, b_, size_t(n) * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return "download failed";
            return nullptr;
        };
        if (const char* e = dev_solve(rhs.data(), x.data())) return e;
        bool ok = residual(rhs.data(), x.data(), r.data(), kRefineTol);
        for (int it = 0; it < 3 && !ok; ++it) {
            std::vector<double> dx(static_cast<size_t>(n));
            if (const char* e = dev_solve(r.data(), dx.data())) return e;
            for (int64_t q = 0; q < n; ++q) x[size_t(q)] += dx[size_t(q)];
            ok = residual(rhs.data(), x.data(), r.data(), kRefineTol);
        }
        std::copy(x.begin(), x.end(), b);
        return nullptr;
    }
    if (!factored_) return "no factorisation";
    if (n_ == 0) return nullptr;
    if (hipMemcpyAsync(b_, b, size_t(n_) * sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess) return "upload failed";
    hipLaunchKernelGGL(sytrs_lower_kernel, dim3(1), dim3(kSolveBlock), 0, s, a_, n_, ipiv_, b_);
    if (hipGetLastError() != hipSuccess) return "sytrs launch failed";
    if (hipMemcpyAsync(b, b_, size_t(n_) * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return "download failed";
    return nullptr;
}

}  // namespace wfsa
