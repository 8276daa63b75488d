// rocBLAS fp64 GEMM at the dense path's shapes (c5: 4096 states, 1024 row
// slots), against the fp64 MFMA peak (78.6 TF): the step GEMM
// (1024 x 4096 x 4096, both operands along memory rows as the dense kernels
// read them) and a slice of the gradient GEMM (4096 x 4096 x 1024*k).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
#define RB(x) do { rocblas_status s_ = (x); if (s_ != rocblas_status_success) { printf("rocblas %d line %d\n", int(s_), __LINE__); return 1; } } while (0)

int main() {
    rocblas_handle h;
    RB(rocblas_create_handle(&h));
    struct Shape { int m, n, k; rocblas_operation ta, tb; const char* what; };
    const Shape shapes[] = {
        {4096, 1024, 4096, rocblas_operation_transpose, rocblas_operation_none, "step: C^T(4096x1024) = A^T alpha^T"},
        {4096, 1024, 4096, rocblas_operation_none, rocblas_operation_none, "step, A not transposed"},
        {4096, 4096, 8192, rocblas_operation_none, rocblas_operation_transpose, "gradient slice K=8192"},
        {4096, 4096, 32768, rocblas_operation_none, rocblas_operation_transpose, "gradient slice K=32768"},
    };
    for (const Shape& sh : shapes) {
        const size_t na = size_t(sh.m) * sh.k, nb = size_t(sh.k) * sh.n, nc = size_t(sh.m) * sh.n;
        double *a, *b, *c;
        CK(hipMalloc(&a, na * 8));
        CK(hipMalloc(&b, nb * 8));
        CK(hipMalloc(&c, nc * 8));
        CK(hipMemset(a, 0, na * 8));
        CK(hipMemset(b, 0, nb * 8));
        CK(hipMemset(c, 0, nc * 8));
        const double one = 1.0, zero = 0.0;
        const int lda = sh.ta == rocblas_operation_none ? sh.m : sh.k;
        const int ldb = sh.tb == rocblas_operation_none ? sh.k : sh.n;
        for (int r = 0; r < 3; ++r) RB(rocblas_dgemm(h, sh.ta, sh.tb, sh.m, sh.n, sh.k, &one, a, lda, b, ldb, &zero, c, sh.m));
        CK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const int reps = 10;
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) RB(rocblas_dgemm(h, sh.ta, sh.tb, sh.m, sh.n, sh.k, &one, a, lda, b, ldb, &zero, c, sh.m));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double t = ms / reps * 1e-3, tf = 2.0 * sh.m * sh.n * double(sh.k) / t / 1e12;
        printf("%-40s %8.3f ms  %6.1f TF/s  %.2f of 78.6\n", sh.what, t * 1e3, tf, tf / 78.6);
        CK(hipFree(a));
        CK(hipFree(b));
        CK(hipFree(c));
    }
    return 0;
}
