// Micro-benchmark: ways to move ~74 KB of results device -> host (and the
// weights host -> device) per iteration.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void pub8(const double* out, double* host, int n) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) host[i] = out[i];
    __threadfence_system();
}
__global__ void pub16(const double2* out, double2* host, int n2) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += gridDim.x * blockDim.x) host[i] = out[i];
    __threadfence_system();
}
__global__ void pubnt(const double2* out, double2* host, int n2) {
    typedef double v2 __attribute__((ext_vector_type(2)));
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += gridDim.x * blockDim.x)
        __builtin_nontemporal_store(*reinterpret_cast<const v2*>(out + i), reinterpret_cast<v2*>(host + i));
    __threadfence_system();
}
__global__ void empty() {}

int main() {
    const int n = 9216 + 1;
    const size_t bytes = size_t(n) * 8;
    double* d;
    CK(hipMalloc(&d, bytes + 64));
    CK(hipMemset(d, 0, bytes + 64));
    double *hc, *hn, *hd;
    CK(hipHostMalloc(&hc, bytes + 64, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc(&hn, bytes + 64, hipHostMallocMapped | hipHostMallocNonCoherent));
    CK(hipHostMalloc(&hd, bytes + 64));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, auto fn) -> int {
        for (int r = 0; r < 5; ++r) fn();
        CK(hipStreamSynchronize(s));
        const int R = 200;
        auto t0 = std::chrono::steady_clock::now();
        CK(hipEventRecord(a, s));
        for (int r = 0; r < R; ++r) fn();
        CK(hipEventRecord(b, s));
        CK(hipStreamSynchronize(s));
        auto t1 = std::chrono::steady_clock::now();
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        // single-shot round trip: enqueue + synchronize
        double rt = 0;
        for (int r = 0; r < 50; ++r) {
            auto q0 = std::chrono::steady_clock::now();
            fn();
            CK(hipStreamSynchronize(s));
            rt += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - q0).count();
        }
        printf("%-40s device %7.2f us/op  host-loop %7.2f us/op  round-trip %7.2f us\n", name, ms * 1e3 / R,
               std::chrono::duration<double, std::micro>(t1 - t0).count() / R, rt / 50);
        return 0;
    };
    double *dc, *dn, *dd;
    CK(hipHostGetDevicePointer((void**)&dc, hc, 0));
    CK(hipHostGetDevicePointer((void**)&dn, hn, 0));
    CK(hipHostGetDevicePointer((void**)&dd, hd, 0));
    run("empty kernel", [&] { hipLaunchKernelGGL(empty, dim3(1), dim3(64), 0, s); });
    run("memcpy D2H default pinned", [&] { (void)hipMemcpyAsync(hd, d, bytes, hipMemcpyDeviceToHost, s); });
    run("memcpy H2D default pinned", [&] { (void)hipMemcpyAsync(d, hd, bytes, hipMemcpyHostToDevice, s); });
    run("memcpy D2H coherent", [&] { (void)hipMemcpyAsync(hc, d, bytes, hipMemcpyDeviceToHost, s); });
    for (int blocks : {1, 8, 37}) {
        for (int thr : {256, 1024}) {
            char nm[96];
            snprintf(nm, sizeof nm, "pub8 coherent %dx%d", blocks, thr);
            run(nm, [&] { hipLaunchKernelGGL(pub8, dim3(blocks), dim3(thr), 0, s, d, dc, n); });
            snprintf(nm, sizeof nm, "pub16 coherent %dx%d", blocks, thr);
            run(nm, [&] { hipLaunchKernelGGL(pub16, dim3(blocks), dim3(thr), 0, s, (const double2*)d, (double2*)dc, (n + 1) / 2); });
            snprintf(nm, sizeof nm, "pub16 noncoherent %dx%d", blocks, thr);
            run(nm, [&] { hipLaunchKernelGGL(pub16, dim3(blocks), dim3(thr), 0, s, (const double2*)d, (double2*)dn, (n + 1) / 2); });
            snprintf(nm, sizeof nm, "pub16 default %dx%d", blocks, thr);
            run(nm, [&] { hipLaunchKernelGGL(pub16, dim3(blocks), dim3(thr), 0, s, (const double2*)d, (double2*)dd, (n + 1) / 2); });
            snprintf(nm, sizeof nm, "pubnt coherent %dx%d", blocks, thr);
            run(nm, [&] { hipLaunchKernelGGL(pubnt, dim3(blocks), dim3(thr), 0, s, (const double2*)d, (double2*)dc, (n + 1) / 2); });
        }
    }
    // host -> device reads by a kernel
    for (int blocks : {1, 8, 37}) {
        char nm[96];
        snprintf(nm, sizeof nm, "stage16 coherent %dx256", blocks);
        run(nm, [&] { hipLaunchKernelGGL(pub16, dim3(blocks), dim3(256), 0, s, (const double2*)dc, (double2*)d, (n + 1) / 2); });
        snprintf(nm, sizeof nm, "stage16 default %dx256", blocks);
        run(nm, [&] { hipLaunchKernelGGL(pub16, dim3(blocks), dim3(256), 0, s, (const double2*)dd, (double2*)d, (n + 1) / 2); });
    }
    return 0;
}
