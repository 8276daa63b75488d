// Micro-benchmark: what a small kernel costs after a kernel that dirtied
// the L2 (device time per op, hipEvent).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void dirty(double* p, size_t n) {
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) p[i] = double(i);
}
__global__ void empty1() {}
__global__ void sum1(const double* p, int n, double* out) {
    double s = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i];
    if (threadIdx.x == 0) out[0] = s;
}
__global__ void hostflag(unsigned* f, unsigned v) {
    if (threadIdx.x == 0) __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
    double* d;
    const size_t N = size_t(8) << 20;   // 64 MB
    CK(hipMalloc(&d, N * 8));
    unsigned* hf;
    CK(hipHostMalloc(&hf, 64, hipHostMallocMapped | hipHostMallocCoherent));
    unsigned* df;
    CK(hipHostGetDevicePointer((void**)&df, hf, 0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int R = 100;
    for (size_t dirty_bytes : {size_t(0), size_t(1) << 20, size_t(6) << 20, size_t(64) << 20}) {
        for (int kind = 0; kind < 3; ++kind) {
            float tot = 0, base = 0;
            for (int pass = 0; pass < 2; ++pass) {
                CK(hipStreamSynchronize(s));
                CK(hipEventRecord(a, s));
                for (int r = 0; r < R; ++r) {
                    if (dirty_bytes) hipLaunchKernelGGL(dirty, dim3(1024), dim3(256), 0, s, d, dirty_bytes / 8);
                    if (pass == 1) {
                        if (kind == 0) hipLaunchKernelGGL(empty1, dim3(1), dim3(64), 0, s);
                        if (kind == 1) hipLaunchKernelGGL(sum1, dim3(1), dim3(1024), 0, s, d, 12000, d + N - 1);
                        if (kind == 2) hipLaunchKernelGGL(hostflag, dim3(1), dim3(64), 0, s, df, unsigned(r));
                    }
                }
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (pass == 0) base = ms; else tot = ms;
            }
            const char* nm[] = {"empty 1x64", "sum 12k 1x1024", "host flag"};
            printf("dirty %6zu KB  %-16s  added %.2f us per launch (dirty-only %.2f us)\n", dirty_bytes >> 10, nm[kind],
                   (tot - base) * 1e3 / R, base * 1e3 / R);
        }
    }
    return 0;
}
