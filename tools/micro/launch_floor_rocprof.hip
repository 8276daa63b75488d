// Launch floor on gfx950: rocprof durations of kernels that return at entry,
// launched back to back on one stream -- no arguments, a 1 KiB argument
// struct, 16 KiB of dynamic LDS, and after a kernel that stores 5 MB (the
// next kernel's start then follows an end-of-kernel write-back).
// Build: hipcc --offload-arch=gfx950 -O2 launch_floor_rocprof.hip -o launch_floor_rocprof
#include <hip/hip_runtime.h>

#include <cstdio>

struct Big {
    double v[128];
};

__global__ void empty_kernel() {}
__global__ void big_arg_kernel(Big b) {
    if (b.v[0] == 12345.0 && threadIdx.x == 0) b.v[1] = 0.0;
}
__global__ void lds_kernel(int x) {
    extern __shared__ double s[];
    if (x == 12345) s[threadIdx.x] = 0.0;
}
__global__ void empty_s() {}
__global__ void empty_after_flag() {}
__global__ void flag_kernel(unsigned* f, unsigned v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void store_kernel(double* p, size_t n) {
    const size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) p[i] = double(i);
}

int main() {
    const int reps = 200;
    Big b{};
    double* p = nullptr;
    const size_t n = 5u << 17;   // 5 MB of doubles / 8
    if (hipMalloc(&p, n * sizeof(double)) != hipSuccess) return 1;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(empty_kernel, dim3(1025), dim3(256), 0, 0);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(big_arg_kernel, dim3(1025), dim3(256), 0, 0, b);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(lds_kernel, dim3(1025), dim3(256), 16384, 0, 0);
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(store_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, 0, p, n);
        hipLaunchKernelGGL(empty_kernel, dim3(1025), dim3(256), 0, 0);
    }
    hipStream_t s1 = nullptr, s2 = nullptr;
    if (hipStreamCreateWithFlags(&s1, hipStreamNonBlocking) != hipSuccess) return 3;
    if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess) return 3;
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s2);
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(empty_s, dim3(1025), dim3(256), 0, s1);
    unsigned* hf = nullptr;
    unsigned* df = nullptr;
    if (hipHostMalloc(&hf, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 4;
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&df), hf, 0) != hipSuccess) return 4;
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(store_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s1, p, n);
        hipLaunchKernelGGL(flag_kernel, dim3(1025), dim3(256), 0, s1, df, unsigned(r));
        hipLaunchKernelGGL(empty_after_flag, dim3(1025), dim3(256), 0, s1);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    (void)hipHostFree(hf);
    (void)hipFree(p);
    std::printf("ok\n");
    return 0;
}
