// Semantics of gfx950's v_permlane16_swap / v_permlane32_swap (the bubble
// butterfly's cross-row exchanges): prints, for both outputs of each
// builtin with old = src = lane id, which lane's value every lane received.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
    const int l = int(threadIdx.x);
    auto a = __builtin_amdgcn_permlane16_swap(l, l, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(l, l, false, false);
    out[l] = a[0];
    out[64 + l] = a[1];
    out[128 + l] = b[0];
    out[192 + l] = b[1];
}

int main() {
    int* d = nullptr;
    if (hipMalloc(&d, 256 * sizeof(int)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    int h[256];
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[4] = {"perm16[0]", "perm16[1]", "perm32[0]", "perm32[1]"};
    for (int k = 0; k < 4; ++k) {
        std::printf("%s:", names[k]);
        for (int l = 0; l < 64; ++l) std::printf(" %d", h[64 * k + l]);
        std::printf("\n");
    }
    return 0;
}
