// Blocked symmetric-indefinite LDL^T on the device (sym_solver.hpp,
// SymSolver::factor_coo): the KKT system is assembled in HBM from its
// entries, then factored panel by panel (kNb columns):
//   1. the diagonal block in LDS, one workgroup: Bunch-Kaufman 1x1 / 2x2
//      pivots chosen within the block (the supernode-restricted pivoting of
//      MKL DSS / PARDISO, which the reference calls); a pivot below
//      tau = 1e-12 max|A| is not taken -- the factorisation reports
//      "perturbed" and the caller uses the full Bunch-Kaufman instead;
//   2. the block's interchanges applied to the columns of the panel below
//      (into a scratch panel) and to the block's rows of L on the left;
//   3. Y = A21 P L11^-T (rocBLAS dtrsm), L21 = Y D^-1 (a kernel, which also
//      tracks the largest |L21| -- element growth);
//   4. the trailing update A22 -= Y L21^T on the lower triangle (rocBLAS
//      dsyrkx: a plain library GEMM-class call, fp64 MFMA).
// P^T A P = L D L^T with P block-diagonal.  Inertia and log|det| come from
// D's blocks (Sylvester: exact for the congruence).  The solve runs the
// blocks forward and back (rocBLAS dtrsv / dgemv) and the caller refines it
// against the sparse entries.
#include "sym_solver.hpp"

#include <rocblas/rocblas.h>

#include <algorithm>
#include <cmath>

namespace wfsa {
namespace {

constexpr int kNb = 128;          // panel width
constexpr int kDiagThreads = 1024;

__global__ void coo_scatter_kernel(double* a, int64_t n, int64_t nnz, const int32_t* __restrict__ row,
                                   const int32_t* __restrict__ col, const double* __restrict__ val) {
    const int64_t t = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (t < nnz) a[int64_t(col[t]) * n + row[t]] = val[t];
}

// block argmax of |v| over the workgroup (first index on ties)
__device__ void blk_argmax(double v, int i, double* rv, int* ri, double& out_v, int& out_i) {
    double a = fabs(v);
    for (int o = 32; o > 0; o >>= 1) {
        const double b = __shfl_xor(a, o, 64);
        const int j = __shfl_xor(i, o, 64);
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
    for (int q = 1; q < kDiagThreads / 64; ++q)
        if (rv[q] > a || (rv[q] == a && ri[q] < i)) {
            a = rv[q];
            i = ri[q];
        }
    __syncthreads();
    out_v = a;
    out_i = i;
}

// The diagonal block [k0, k0 + m): Bunch-Kaufman (dsytf2's rule) with the
// pivot search restricted to the block; writes the unit lower L11 (zero at a
// 2x2 block's off-diagonal) and D's diagonal into a, D (diag, subdiag) and
// the pivot kinds (1: 1x1, 2: first column of a 2x2, 0: its second) into
// d / piv, and perm[k0 + c] = the global row now at position k0 + c.
__global__ __launch_bounds__(kDiagThreads) void blk_diag_kernel(double* a, int64_t n, int64_t k0, int m, double tau,
                                                                int32_t* perm_out, double* d_out, int32_t* piv_out,
                                                                int32_t* status) {
    __shared__ double B[kNb][kNb + 1];
    __shared__ int perm[kNb];
    __shared__ double rv[kDiagThreads / 64];
    __shared__ int ri[kDiagThreads / 64];
    __shared__ int s_piv[kNb];
    const int t = int(threadIdx.x);
    for (int idx = t; idx < m * m; idx += kDiagThreads) {
        const int r = idx % m, c = idx / m;
        if (r >= c) {
            const double v = a[(k0 + c) * n + k0 + r];
            B[r][c] = v;
            B[c][r] = v;
        }
    }
    for (int c = t; c < m; c += kDiagThreads) perm[c] = c;
    __syncthreads();
    const double alpha = (1.0 + sqrt(17.0)) / 8.0;
    bool small = false;
    for (int k = 0; k < m;) {
        double colmax;
        int imax;
        {
            double v = 0.0;
            int vi = m;
            for (int i = k + 1 + t; i < m; i += kDiagThreads)
                if (fabs(B[i][k]) > fabs(v) || vi == m) {
                    v = B[i][k];
                    vi = i;
                }
            blk_argmax(v, vi, rv, ri, colmax, imax);
            if (imax >= m) {
                colmax = 0.0;
                imax = k;
            }
        }
        const double absakk = fabs(B[k][k]);
        int kp = k, kstep = 1;
        if (fmax(absakk, colmax) > 0.0 && absakk < alpha * colmax) {
            double v = 0.0;
            int vi = m;
            for (int j = k + t; j < m; j += kDiagThreads)
                if (j != imax && (fabs(B[imax][j]) > fabs(v) || vi == m)) {
                    v = B[imax][j];
                    vi = j;
                }
            double rowmax;
            int jm;
            blk_argmax(v, vi, rv, ri, rowmax, jm);
            if (absakk >= alpha * colmax * (colmax / rowmax)) {
                kp = k;
            } else if (fabs(B[imax][imax]) >= alpha * rowmax) {
                kp = imax;
            } else {
                kp = imax;
                kstep = 2;
            }
        }
        const int kk = k + kstep - 1;
        if (kp != kk) {   // symmetric interchange of kk and kp: rows (L part too), then columns >= k
            for (int j = t; j < m; j += kDiagThreads) {
                const double x = B[kk][j];
                B[kk][j] = B[kp][j];
                B[kp][j] = x;
            }
            __syncthreads();
            for (int i = k + t; i < m; i += kDiagThreads) {
                const double x = B[i][kk];
                B[i][kk] = B[i][kp];
                B[i][kp] = x;
            }
            if (t == 0) {
                const int x = perm[kk];
                perm[kk] = perm[kp];
                perm[kp] = x;
            }
        }
        __syncthreads();
        if (kstep == 1) {
            const double d = B[k][k];
            if (!(fabs(d) >= tau)) small = true;   // (every thread sees the same d)
            const double r = (d != 0.0) ? 1.0 / d : 0.0;
            const int w = m - k - 1;
            for (int idx = t; idx < w * w; idx += kDiagThreads) {
                const int i = k + 1 + idx % w, j = k + 1 + idx / w;
                if (i >= j) {
                    const double u = B[i][j] - B[i][k] * B[j][k] * r;
                    B[i][j] = u;
                    B[j][i] = u;
                }
            }
            __syncthreads();
            for (int i = k + 1 + t; i < m; i += kDiagThreads) B[i][k] *= r;
            if (t == 0) s_piv[k] = 1;
        } else {
            const double d11 = B[k][k], d21 = B[k + 1][k], d22 = B[k + 1][k + 1];
            const double det = d11 * d22 - d21 * d21;
            if (!(fabs(det) >= tau * fabs(d21))) small = true;
            const double i11 = d22 / det, i21 = -d21 / det, i22 = d11 / det;
            const int w = m - k - 2;
            for (int idx = t; idx < w * w; idx += kDiagThreads) {
                const int i = k + 2 + idx % w, j = k + 2 + idx / w;
                if (i >= j) {
                    const double ai0 = B[i][k], ai1 = B[i][k + 1], aj0 = B[j][k], aj1 = B[j][k + 1];
                    const double u = B[i][j] - (ai0 * (i11 * aj0 + i21 * aj1) + ai1 * (i21 * aj0 + i22 * aj1));
                    B[i][j] = u;
                    B[j][i] = u;
                }
            }
            __syncthreads();
            for (int i = k + 2 + t; i < m; i += kDiagThreads) {
                const double x = B[i][k], y = B[i][k + 1];
                B[i][k] = x * i11 + y * i21;
                B[i][k + 1] = x * i21 + y * i22;
            }
            if (t == 0) {
                s_piv[k] = 2;
                s_piv[k + 1] = 0;
            }
        }
        __syncthreads();
        k += kstep;
    }
    if (small && t == 0) atomicOr(status, 1);
    // L11 (unit lower) and D's diagonal back into a; D and the pivots out
    for (int idx = t; idx < m * m; idx += kDiagThreads) {
        const int r = idx % m, c = idx / m;
        if (r > c) a[(k0 + c) * n + k0 + r] = (r == c + 1 && s_piv[c] == 2) ? 0.0 : B[r][c];
        else if (r == c) a[(k0 + c) * n + k0 + r] = B[c][c];
    }
    for (int c = t; c < m; c += kDiagThreads) {
        perm_out[k0 + c] = int32_t(k0 + perm[c]);
        piv_out[k0 + c] = s_piv[c];
        d_out[k0 + c] = B[c][c];
        d_out[n + k0 + c] = (s_piv[c] == 2) ? B[c + 1][c] : 0.0;
    }
}

// rows [r0, n) of the panel's columns, permuted (column c <- column perm[c]),
// into the scratch panel Y (column-major, leading dimension ldy)
__global__ void panel_gather_kernel(const double* a, int64_t n, int64_t k0, int m, int64_t r0, const int32_t* perm,
                                    double* y, int64_t ldy) {
    const int64_t i = r0 + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int c = 0; c < m; ++c) y[int64_t(c) * ldy + (i - r0)] = a[int64_t(perm[k0 + c]) * n + i];
}

// L21 = Y D^-1 into a (rows [r0, n) of the panel's columns); the largest
// |L21| of each thread block into gmax (element growth)
__global__ void panel_scale_kernel(double* a, int64_t n, int64_t k0, int m, int64_t r0, const double* y, int64_t ldy,
                                   const double* d, const int32_t* piv, double* gmax) {
    __shared__ double red[256];
    const int64_t i = r0 + int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    double mx = 0.0;
    if (i < n) {
        for (int c = 0; c < m;) {
            const int64_t g = k0 + c;
            if (piv[g] == 1) {
                const double dv = d[g];
                const double l = dv != 0.0 ? y[int64_t(c) * ldy + (i - r0)] / dv : 0.0;
                a[g * n + i] = l;
                mx = fmax(mx, fabs(l));
                c += 1;
            } else {
                const double d11 = d[g], d22 = d[g + 1], d21 = d[n + g];
                const double det = d11 * d22 - d21 * d21;
                const double y0 = y[int64_t(c) * ldy + (i - r0)], y1 = y[int64_t(c + 1) * ldy + (i - r0)];
                const double l0 = (y0 * d22 - y1 * d21) / det, l1 = (y1 * d11 - y0 * d21) / det;
                a[g * n + i] = l0;
                a[(g + 1) * n + i] = l1;
                mx = fmax(mx, fmax(fabs(l0), fabs(l1)));
                c += 2;
            }
        }
    }
    red[threadIdx.x] = mx;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (int(threadIdx.x) < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) gmax[blockIdx.x] = fmax(gmax[blockIdx.x], red[0]);
}

// the block's rows of L to its left (columns [0, k0)) in the block's final order
__global__ void left_rows_kernel(double* a, int64_t n, int64_t k0, int m, const int32_t* perm) {
    __shared__ double col[kNb];
    const int64_t j = blockIdx.x;   // column < k0
    const int c = int(threadIdx.x);
    if (c < m) col[c] = a[j * n + perm[k0 + c]];
    __syncthreads();
    if (c < m) a[j * n + k0 + c] = col[c];
}

__global__ void permute_kernel(const double* src, const int32_t* perm, int64_t n, double* dst, int inverse) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (inverse) dst[perm[i]] = src[i];
    else dst[i] = src[perm[i]];
}

__global__ void dsolve_kernel(double* x, const double* d, const int32_t* piv, int64_t n) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    if (piv[k] == 1) {
        x[k] = d[k] != 0.0 ? x[k] / d[k] : 0.0;
    } else if (piv[k] == 2) {
        const double d11 = d[k], d22 = d[k + 1], d21 = d[n + k];
        const double det = d11 * d22 - d21 * d21;
        const double y0 = x[k], y1 = x[k + 1];
        x[k] = (y0 * d22 - y1 * d21) / det;
        x[k + 1] = (y1 * d11 - y0 * d21) / det;
    }
}

bool rb_ok(rocblas_status st) { return st == rocblas_status_success; }

}  // namespace

// ---- SymSolver::blocked_* (sym_solver.hpp) ---------------------------------

const char* SymSolver::ensure_blocked(int64_t n, hipStream_t s) {
    if (!blas_) {
        rocblas_handle h = nullptr;
        if (!rb_ok(rocblas_create_handle(&h))) return "rocblas_create_handle failed";
        blas_ = h;
    }
    if (!rb_ok(rocblas_set_stream(static_cast<rocblas_handle>(blas_), s))) return "rocblas_set_stream failed";
    if (n > bcap_) {
        for (void* p : {static_cast<void*>(y_), static_cast<void*>(perm_), static_cast<void*>(bpiv_),
                        static_cast<void*>(bd_), static_cast<void*>(gmax_), static_cast<void*>(bstat_),
                        static_cast<void*>(x_), static_cast<void*>(coo_)})
            if (p) (void)hipFree(p);
        y_ = bd_ = gmax_ = x_ = nullptr;
        perm_ = bpiv_ = bstat_ = nullptr;
        coo_ = nullptr;
        bcap_ = 0;
        const int64_t nblk = (n + 255) / 256;
        if (hipMalloc(reinterpret_cast<void**>(&y_), size_t(n) * kNb * sizeof(double)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&perm_), size_t(n) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&bpiv_), size_t(n) * sizeof(int32_t)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&bd_), 2 * size_t(n) * sizeof(double)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&gmax_), size_t(nblk) * sizeof(double)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&bstat_), sizeof(int32_t)) != hipSuccess ||
            hipMalloc(reinterpret_cast<void**>(&x_), 2 * size_t(n) * sizeof(double)) != hipSuccess)
            return "device allocation failed";
        bcap_ = n;
    }
    return nullptr;
}

const char* SymSolver::assemble(hipStream_t s) {
    const int64_t n = n_;
    const int64_t nnz = int64_t(crow_.size());
    if (hipMemsetAsync(a_, 0, size_t(n) * size_t(n) * sizeof(double), s) != hipSuccess) return "memset failed";
    if (nnz == 0) return nullptr;
    if (coo_bytes_ < size_t(nnz) * 16) {
        if (coo_) (void)hipFree(coo_);
        coo_ = nullptr;
        coo_bytes_ = 0;
        if (hipMalloc(&coo_, size_t(nnz) * 16) != hipSuccess) return "device allocation failed";
        coo_bytes_ = size_t(nnz) * 16;
    }
    int32_t* dr = static_cast<int32_t*>(coo_);
    int32_t* dc = dr + nnz;
    double* dv = reinterpret_cast<double*>(dc + nnz);
    if (hipMemcpyAsync(dr, crow_.data(), size_t(nnz) * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dc, ccol_.data(), size_t(nnz) * 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(dv, cval_.data(), size_t(nnz) * 8, hipMemcpyHostToDevice, s) != hipSuccess)
        return "upload failed";
    hipLaunchKernelGGL(coo_scatter_kernel, dim3(unsigned((nnz + 255) / 256)), dim3(256), 0, s, a_, n, nnz, dr, dc, dv);
    return hipGetLastError() == hipSuccess ? nullptr : "scatter launch failed";
}

const char* SymSolver::blocked_factor(hipStream_t s, SymFactor* out, bool* exact) {
    const int64_t n = n_;
    *exact = false;
    rocblas_handle h = static_cast<rocblas_handle>(blas_);
    double amax = 0.0;
    for (double v : cval_) amax = std::max(amax, std::fabs(v));
    const double tau = 1e-12 * std::max(amax, 1e-300);
    const int64_t nblk = (n + 255) / 256;
    if (hipMemsetAsync(bstat_, 0, sizeof(int32_t), s) != hipSuccess ||
        hipMemsetAsync(gmax_, 0, size_t(nblk) * sizeof(double), s) != hipSuccess)
        return "memset failed";
    const double one = 1.0, minus = -1.0;
    for (int64_t k0 = 0; k0 < n; k0 += kNb) {
        const int m = int(std::min<int64_t>(kNb, n - k0));
        const int64_t r0 = k0 + m, rows = n - r0;
        hipLaunchKernelGGL(blk_diag_kernel, dim3(1), dim3(kDiagThreads), 0, s, a_, n, k0, m, tau, perm_, bd_, bpiv_,
                           bstat_);
        if (k0 > 0) hipLaunchKernelGGL(left_rows_kernel, dim3(unsigned(k0)), dim3(kNb), 0, s, a_, n, k0, m, perm_);
        if (rows > 0) {
            const unsigned g = unsigned((rows + 255) / 256);
            hipLaunchKernelGGL(panel_gather_kernel, dim3(g), dim3(256), 0, s, a_, n, k0, m, r0, perm_, y_, rows);
            // Y = (A21 P) L11^-T
            if (!rb_ok(rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower, rocblas_operation_transpose,
                                     rocblas_diagonal_unit, rocblas_int(rows), m, &one, a_ + k0 * n + k0,
                                     rocblas_int(n), y_, rocblas_int(rows))))
                return "rocblas_dtrsm failed";
            hipLaunchKernelGGL(panel_scale_kernel, dim3(g), dim3(256), 0, s, a_, n, k0, m, r0, y_, rows, bd_, bpiv_,
                               gmax_);
            // A22 -= Y L21^T (lower)
            if (!rb_ok(rocblas_dsyrkx(h, rocblas_fill_lower, rocblas_operation_none, rocblas_int(rows), m, &minus, y_,
                                      rocblas_int(rows), a_ + k0 * n + r0, rocblas_int(n), &one, a_ + r0 * n + r0,
                                      rocblas_int(n))))
                return "rocblas_dsyrkx failed";
        }
    }
    if (hipGetLastError() != hipSuccess) return "blocked factorisation launch failed";
    std::vector<double> d(2 * size_t(n)), gm(static_cast<size_t>(nblk));
    std::vector<int32_t> piv(static_cast<size_t>(n));
    int32_t st = 0;
    if (hipMemcpyAsync(d.data(), bd_, d.size() * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(piv.data(), bpiv_, piv.size() * sizeof(int32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(gm.data(), gmax_, gm.size() * sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(&st, bstat_, sizeof st, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return "download failed";
    double growth = 0.0;
    for (double v : gm) growth = std::max(growth, v);
    SymFactor f;
    for (int64_t k = 0; k < n;) {
        if (piv[size_t(k)] == 2) {
            const double x = d[size_t(k)], z = d[size_t(k) + 1], y = d[size_t(n + k)];
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
        } else {
            const double v = d[size_t(k)];
            if (v > 0.0) ++f.positive;
            else if (v < 0.0) ++f.negative;
            else ++f.zero;
            if (v < 0.0) f.det_sign = -f.det_sign;
            f.log_abs_det += std::log(std::fabs(v));
            k += 1;
        }
    }
    *out = f;
    // a pivot under tau, or element growth past 1e8: not trusted (the caller
    // falls back to the full Bunch-Kaufman)
    *exact = st == 0 && growth <= 1e8 && f.zero == 0;
    last_growth_ = growth;
    return nullptr;
}

// x = A^-1 b through the blocked factor (x_, b_ on the device)
const char* SymSolver::blocked_solve(hipStream_t s) {
    const int64_t n = n_;
    rocblas_handle h = static_cast<rocblas_handle>(blas_);
    double* z = x_;       // [n] working vector
    double* tmp = x_ + n;
    const unsigned g = unsigned((n + 255) / 256);
    const double one = 1.0, minus = -1.0;
    hipLaunchKernelGGL(permute_kernel, dim3(g), dim3(256), 0, s, b_, perm_, n, z, 0);   // z = P^T b
    for (int64_t k0 = 0; k0 < n; k0 += kNb) {   // L y = z
        const int m = int(std::min<int64_t>(kNb, n - k0));
        const int64_t r0 = k0 + m, rows = n - r0;
        if (!rb_ok(rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_none, rocblas_diagonal_unit, m,
                                 a_ + k0 * n + k0, rocblas_int(n), z + k0, 1)))
            return "rocblas_dtrsv failed";
        if (rows > 0 && !rb_ok(rocblas_dgemv(h, rocblas_operation_none, rocblas_int(rows), m, &minus, a_ + k0 * n + r0,
                                             rocblas_int(n), z + k0, 1, &one, z + r0, 1)))
            return "rocblas_dgemv failed";
    }
    hipLaunchKernelGGL(dsolve_kernel, dim3(g), dim3(256), 0, s, z, bd_, bpiv_, n);   // D w = y
    const int64_t last = ((n - 1) / kNb) * kNb;
    for (int64_t k0 = last; k0 >= 0; k0 -= kNb) {   // L^T v = w
        const int m = int(std::min<int64_t>(kNb, n - k0));
        const int64_t r0 = k0 + m, rows = n - r0;
        if (rows > 0 && !rb_ok(rocblas_dgemv(h, rocblas_operation_transpose, rocblas_int(rows), m, &minus,
                                             a_ + k0 * n + r0, rocblas_int(n), z + r0, 1, &one, z + k0, 1)))
            return "rocblas_dgemv failed";
        if (!rb_ok(rocblas_dtrsv(h, rocblas_fill_lower, rocblas_operation_transpose, rocblas_diagonal_unit, m,
                                 a_ + k0 * n + k0, rocblas_int(n), z + k0, 1)))
            return "rocblas_dtrsv failed";
    }
    hipLaunchKernelGGL(permute_kernel, dim3(g), dim3(256), 0, s, z, perm_, n, tmp, 1);   // x = P v
    if (hipMemcpyAsync(b_, tmp, size_t(n) * sizeof(double), hipMemcpyDeviceToDevice, s) != hipSuccess)
        return "copy failed";
    return hipGetLastError() == hipSuccess ? nullptr : "solve launch failed";
}

}  // namespace wfsa
