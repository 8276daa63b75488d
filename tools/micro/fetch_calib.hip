// FETCH_SIZE / WRITE_SIZE calibration for our access pattern: one kernel
// streams exactly `bytes` with 16-byte-per-lane coalesced loads (the stream
// kernel's pattern), another writes exactly `bytes` with 16-byte stores.
// Run under rocprofv3 --pmc FETCH_SIZE (and WRITE_SIZE) and compare the
// counter (KiB) with the byte count printed here.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

__global__ void stream_read(const uint4* __restrict__ p, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void stream_write(uint4* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
        p[i] = make_uint4(unsigned(i), 1u, 2u, 3u);
}

int main() {
    const size_t bytes = size_t(512) << 20;   // past the 256 MB infinity cache
    uint4* d;
    unsigned* o;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&o, 64));
    CK(hipMemset(d, 1, bytes));
    const size_t n = bytes / 16;
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(stream_read, dim3(4096), dim3(256), 0, 0, d, n, o);
        hipLaunchKernelGGL(stream_write, dim3(4096), dim3(256), 0, 0, d, n);
    }
    CK(hipDeviceSynchronize());
    printf("bytes per launch %zu (%zu KiB)\n", bytes, bytes >> 10);
    return 0;
}
