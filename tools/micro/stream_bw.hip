// Streaming-read rate by footprint: the stream kernel's access shape (each
// wave reads a contiguous run of 1 KiB rows, 16 B per lane, two register sets
// of D rows in flight) over buffers of 16 MB to 1 GB read again and again,
// so the Infinity Cache (256 MiB) holds the small ones between launches.
// Prints the event-timed time per launch and the rate, for 256 x 1024
// threads (16 waves per CU) and for 512 x 1024 (32 waves per CU).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int D, int OCC>
__global__ __launch_bounds__(1024, OCC) void stream_read(const uint4* __restrict__ buf, int64_t rows_per_wave, uint32_t* out) {
    const int lane = threadIdx.x % 64;
    const int64_t w = int64_t(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64;
    const uint4* s = buf + w * rows_per_wave * 64 + lane;
    const int64_t last = rows_per_wave - 1;
    uint4 A[D], B[D];
    uint32_t acc = 0;
    for (int d = 0; d < D; ++d) A[d] = s[64 * min(int64_t(d), last)];
    for (int d = 0; d < D; ++d) B[d] = s[64 * min(int64_t(D + d), last)];
    for (int64_t c0 = 0; c0 < rows_per_wave; c0 += 2 * D) {
        for (int d = 0; d < D; ++d) acc ^= A[d].x ^ A[d].y ^ A[d].z ^ A[d].w;
        for (int d = 0; d < D; ++d) A[d] = s[64 * min(c0 + 2 * D + d, last)];
        for (int d = 0; d < D; ++d) acc ^= B[d].x ^ B[d].y ^ B[d].z ^ B[d].w;
        for (int d = 0; d < D; ++d) B[d] = s[64 * min(c0 + 3 * D + d, last)];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t max_bytes = size_t(1) << 30;
    uint4* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 1, max_bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int occ : {1, 2}) {
        for (size_t mb : {16, 32, 64, 96, 128, 192, 384, 1024}) {
            const int blocks = 256 * occ, waves = blocks * 16;
            const int64_t rows = int64_t(mb << 20) / (int64_t(waves) * 1024);
            auto launch = [&] {
                if (occ == 1) hipLaunchKernelGGL((stream_read<2, 1>), dim3(blocks), dim3(1024), 0, 0, buf, rows, out);
                else hipLaunchKernelGGL((stream_read<2, 2>), dim3(blocks), dim3(1024), 0, 0, buf, rows, out);
            };
            for (int r = 0; r < 5; ++r) launch();
            CK(hipDeviceSynchronize());
            const int reps = 40;
            CK(hipEventRecord(e0, 0));
            for (int r = 0; r < reps; ++r) launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / reps, bytes = double(rows) * waves * 1024;
            printf("%2d waves/CU %6zu MB: %8.2f us per launch  %6.2f TB/s\n", 16 * occ, mb, us, bytes / us / 1e6);
        }
    }
    return 0;
}
