// Stream formats for the trivial words of compiled strings, measured in
// isolation (c3-like: 1M strings of 36 edges, 1024 nodes x 9 out-slots):
//   A  16-bit slot index per edge (the current stream): an independent LDS
//      gather of the edge weight per edge, 2 B of stream per edge;
//   B  4-bit out-edge choice per edge: a chain through LDS (slot = base of the
//      current node + choice; weight and the next node's base per slot),
//      0.5 B of stream per edge;
//   B2 B with two strings per lane (two chains in flight);
//   C  B with the weight and the next base in one 16-byte LDS entry.
// Prints the kernel time of each and checks that all three sum the same
// log-likelihood.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kWave = 64;
constexpr int kNodes = 1024, kDeg = 9, kSlots = kNodes * kDeg;
constexpr int kLen = 36;
constexpr int kChA = (kLen + 7) / 8;    // 16-byte chunks per string, 16-bit words
constexpr int kChB = (kLen + 31) / 32;  // ... nibbles

__device__ inline double wave_sum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// one wave per group of 64 strings, groups dealt round-robin over the waves
__global__ __launch_bounds__(512) void walk_a(const uint4* __restrict__ st, int n_groups, const double* __restrict__ w,
                                              const double* __restrict__ p, double* ll_part) {
    __shared__ double lw[kSlots];
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) lw[j] = w[j];
    __syncthreads();
    const int lane = threadIdx.x % kWave;
    const int gw = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    const int nw = gridDim.x * (blockDim.x / kWave);
    double ll = 0.0;
    for (int g = gw; g < n_groups; g += nw) {
        const uint4* s = st + size_t(g) * kChA * kWave + lane;
        uint4 r[kChA];
#pragma unroll
        for (int c = 0; c < kChA; ++c) r[c] = s[c * kWave];
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int c = 0; c < kChA; ++c) {
            const uint32_t v[4] = {r[c].x, r[c].y, r[c].z, r[c].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t lo = v[i] & 0xffffu, hi = v[i] >> 16;
                a0 += lw[min(lo, uint32_t(kSlots - 1))] * (lo != 0xffffu);
                a1 += lw[min(hi, uint32_t(kSlots - 1))] * (hi != 0xffffu);
            }
        }
        ll += p[g * kWave + lane] * (a0 + a1);
    }
    ll = wave_sum(ll);
    if (lane == 0) ll_part[gw] = ll;
}

template <int K>   // strings per lane in flight
__global__ __launch_bounds__(1024) void walk_b(const uint4* __restrict__ st, int n_groups, const double* __restrict__ sw,
                                               const uint16_t* __restrict__ nb, const double* __restrict__ p,
                                               double* ll_part) {
    __shared__ double lw[kSlots];
    __shared__ uint16_t lnb[kSlots];
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) {
        lw[j] = sw[j];
        lnb[j] = nb[j];
    }
    __syncthreads();
    const int lane = threadIdx.x % kWave;
    const int gw = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    const int nw = gridDim.x * (blockDim.x / kWave);
    double ll = 0.0;
    for (int g0 = gw * K; g0 < n_groups; g0 += nw * K) {
        uint4 r[K][kChB];
        double acc[K];
        int base[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int g = min(g0 + k, n_groups - 1);
            const uint4* s = st + size_t(g) * kChB * kWave + lane;
#pragma unroll
            for (int c = 0; c < kChB; ++c) r[k][c] = s[c * kWave];
            acc[k] = 0.0;
            base[k] = 0;
        }
#pragma unroll
        for (int c = 0; c < kChB; ++c) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    if (c * 32 + i * 8 + h >= kLen) break;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const uint32_t v = (i == 0 ? r[k][c].x : i == 1 ? r[k][c].y : i == 2 ? r[k][c].z : r[k][c].w);
                        const int slot = base[k] + int((v >> (4 * h)) & 0xfu);
                        acc[k] += lw[slot];
                        base[k] = lnb[slot];
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (g0 + k < n_groups) ll += p[(g0 + k) * kWave + lane] * acc[k];
    }
    ll = wave_sum(ll);
    if (lane == 0) ll_part[gw] = ll;
}

// the same with the next group's chunks loaded before the current group is
// applied (software pipelining across groups, as the real stream kernel does)
template <bool GATHER>
__global__ __launch_bounds__(1024) void walk_a_pf(const uint4* __restrict__ st, int n_groups, const double* __restrict__ w,
                                                  const double* __restrict__ p, double* ll_part) {
    __shared__ double lw[kSlots];
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) lw[j] = w[j];
    __syncthreads();
    const int lane = threadIdx.x % kWave;
    const int gw = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    const int nw = gridDim.x * (blockDim.x / kWave);
    double ll = 0.0;
    uint4 r[kChA], nx[kChA];
    auto ld = [&](uint4 (&d)[kChA], int g) {
        const uint4* s = st + size_t(min(g, n_groups - 1)) * kChA * kWave + lane;
#pragma unroll
        for (int c = 0; c < kChA; ++c) d[c] = s[c * kWave];
    };
    if (gw < n_groups) ld(r, gw);
    for (int g = gw; g < n_groups; g += nw) {
        ld(nx, g + nw);
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int c = 0; c < kChA; ++c) {
            const uint32_t v[4] = {r[c].x, r[c].y, r[c].z, r[c].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint32_t lo = v[i] & 0xffffu, hi = v[i] >> 16;
                if (GATHER) {
                    a0 += lw[min(lo, uint32_t(kSlots - 1))] * (lo != 0xffffu);
                    a1 += lw[min(hi, uint32_t(kSlots - 1))] * (hi != 0xffffu);
                } else {
                    a0 += double(lo ^ hi);
                }
            }
        }
        ll += p[g * kWave + lane] * (a0 + a1);
#pragma unroll
        for (int c = 0; c < kChA; ++c) r[c] = nx[c];
    }
    ll = wave_sum(ll);
    if (lane == 0) ll_part[gw] = ll;
}

template <int K>
__global__ __launch_bounds__(1024) void walk_b_pf(const uint4* __restrict__ st, int n_groups, const double* __restrict__ sw,
                                                  const uint16_t* __restrict__ nb, const double* __restrict__ p,
                                                  double* ll_part) {
    __shared__ double lw[kSlots];
    __shared__ uint16_t lnb[kSlots];
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) {
        lw[j] = sw[j];
        lnb[j] = nb[j];
    }
    __syncthreads();
    const int lane = threadIdx.x % kWave;
    const int gw = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    const int nw = gridDim.x * (blockDim.x / kWave);
    double ll = 0.0;
    uint4 r[K][kChB], nx[K][kChB];
    auto ld = [&](uint4 (&d)[K][kChB], int g0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint4* s = st + size_t(min(g0 + k, n_groups - 1)) * kChB * kWave + lane;
#pragma unroll
            for (int c = 0; c < kChB; ++c) d[k][c] = s[c * kWave];
        }
    };
    if (gw * K < n_groups) ld(r, gw * K);
    for (int g0 = gw * K; g0 < n_groups; g0 += nw * K) {
        ld(nx, g0 + nw * K);
        double acc[K];
        int base[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc[k] = 0.0;
            base[k] = 0;
        }
#pragma unroll
        for (int c = 0; c < kChB; ++c) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    if (c * 32 + i * 8 + h >= kLen) break;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const uint32_t v = (i == 0 ? r[k][c].x : i == 1 ? r[k][c].y : i == 2 ? r[k][c].z : r[k][c].w);
                        const int slot = base[k] + int((v >> (4 * h)) & 0xfu);
                        acc[k] += lw[slot];
                        base[k] = lnb[slot];
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (g0 + k < n_groups) ll += p[(g0 + k) * kWave + lane] * acc[k];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int c = 0; c < kChB; ++c) r[k][c] = nx[k][c];
    }
    ll = wave_sum(ll);
    if (lane == 0) ll_part[gw] = ll;
}

// C: B's chain with the weight and the next node's base in ONE 16-byte LDS
// entry (one ds_read_b128 per edge instead of an 8-byte and a 2-byte read);
// the table (147 KB) takes the CU's LDS: one 1024-thread block per CU
template <int K>
__global__ __launch_bounds__(1024) void walk_c_pf(const uint4* __restrict__ st, int n_groups,
                                                  const double2* __restrict__ tab, const double* __restrict__ p,
                                                  double* ll_part) {
    extern __shared__ double2 lt[];
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) lt[j] = tab[j];
    __syncthreads();
    const int lane = threadIdx.x % kWave;
    const int gw = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    const int nw = gridDim.x * (blockDim.x / kWave);
    double ll = 0.0;
    uint4 r[K][kChB], nx[K][kChB];
    auto ld = [&](uint4 (&d)[K][kChB], int g0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint4* s = st + size_t(min(g0 + k, n_groups - 1)) * kChB * kWave + lane;
#pragma unroll
            for (int c = 0; c < kChB; ++c) d[k][c] = s[c * kWave];
        }
    };
    if (gw * K < n_groups) ld(r, gw * K);
    for (int g0 = gw * K; g0 < n_groups; g0 += nw * K) {
        ld(nx, g0 + nw * K);
        double acc[K];
        int base[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc[k] = 0.0;
            base[k] = 0;
        }
#pragma unroll
        for (int c = 0; c < kChB; ++c)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int h = 0; h < 8; ++h) {
                    if (c * 32 + i * 8 + h >= kLen) break;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const uint32_t v = (i == 0 ? r[k][c].x : i == 1 ? r[k][c].y : i == 2 ? r[k][c].z : r[k][c].w);
                        const double2 e = lt[base[k] + int((v >> (4 * h)) & 0xfu)];
                        acc[k] += e.x;
                        base[k] = int(__double_as_longlong(e.y));
                    }
                }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (g0 + k < n_groups) ll += p[(g0 + k) * kWave + lane] * acc[k];
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int c = 0; c < kChB; ++c) r[k][c] = nx[k][c];
    }
    ll = wave_sum(ll);
    if (lane == 0) ll_part[gw] = ll;
}

// A with the weight table split into its high and low 32-bit words (two
// tables, two 4-byte gathers per word instead of one 8-byte gather): the
// bank-conflict pattern of random ds_read_b32 vs ds_read_b64
__global__ __launch_bounds__(1024) void walk_a_split(const uint4* __restrict__ st, int n_groups,
                                                     const double* __restrict__ w, const double* __restrict__ p,
                                                     double* ll_part) {
    __shared__ uint32_t lhi[kSlots], llo[kSlots];
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) {
        const long long b = __double_as_longlong(w[j]);
        lhi[j] = uint32_t(b >> 32);
        llo[j] = uint32_t(b);
    }
    __syncthreads();
    const int lane = threadIdx.x % kWave;
    const int gw = blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave;
    const int nw = gridDim.x * (blockDim.x / kWave);
    double ll = 0.0;
    uint4 r[kChA], nx[kChA];
    auto ld = [&](uint4 (&d)[kChA], int g) {
        const uint4* s = st + size_t(min(g, n_groups - 1)) * kChA * kWave + lane;
#pragma unroll
        for (int c = 0; c < kChA; ++c) d[c] = s[c * kWave];
    };
    auto wt = [&](uint32_t x) {
        const uint32_t i = min(x, uint32_t(kSlots - 1));
        return x != 0xffffu ? __hiloint2double(int(lhi[i]), int(llo[i])) : 0.0;
    };
    if (gw < n_groups) ld(r, gw);
    for (int g = gw; g < n_groups; g += nw) {
        ld(nx, g + nw);
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int c = 0; c < kChA; ++c) {
            const uint32_t v[4] = {r[c].x, r[c].y, r[c].z, r[c].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a0 += wt(v[i] & 0xffffu);
                a1 += wt(v[i] >> 16);
            }
        }
        ll += p[g * kWave + lane] * (a0 + a1);
#pragma unroll
        for (int c = 0; c < kChA; ++c) r[c] = nx[c];
    }
    ll = wave_sum(ll);
    if (lane == 0) ll_part[gw] = ll;
}

// both formats in one kernel: the first nb waves of each block walk nibble
// groups [0, GB), the others 16-bit groups [GB, G) -- HBM and LDS at once
__global__ __launch_bounds__(1024) void walk_mix(const uint4* __restrict__ stA, const uint4* __restrict__ stB, int GB,
                                                 int G, int nbw, const double* __restrict__ w,
                                                 const double* __restrict__ sw, const uint16_t* __restrict__ nb,
                                                 const double* __restrict__ p, double* ll_part) {
    __shared__ double lw[kSlots];
    __shared__ uint16_t lnb[kSlots];
    for (int j = threadIdx.x; j < kSlots; j += blockDim.x) {
        lw[j] = sw[j];
        lnb[j] = nb[j];
    }
    __syncthreads();
    const int lane = threadIdx.x % kWave;
    const int wv = threadIdx.x / kWave, wpb = blockDim.x / kWave;
    double ll = 0.0;
    if (wv < nbw) {   // nibble waves
        const int gw = blockIdx.x * nbw + wv, nw = gridDim.x * nbw;
        uint4 r[kChB], nx[kChB];
        auto ld = [&](uint4 (&d)[kChB], int g) {
            const uint4* s = stB + size_t(min(g, GB - 1)) * kChB * kWave + lane;
#pragma unroll
            for (int c = 0; c < kChB; ++c) d[c] = s[c * kWave];
        };
        if (gw < GB) ld(r, gw);
        for (int g = gw; g < GB; g += nw) {
            ld(nx, g + nw);
            double acc = 0.0;
            int base = 0;
#pragma unroll
            for (int c = 0; c < kChB; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int h = 0; h < 8; ++h) {
                        if (c * 32 + i * 8 + h >= kLen) break;
                        const uint32_t v = (i == 0 ? r[c].x : i == 1 ? r[c].y : i == 2 ? r[c].z : r[c].w);
                        const int slot = base + int((v >> (4 * h)) & 0xfu);
                        acc += lw[slot];
                        base = lnb[slot];
                    }
            ll += p[g * kWave + lane] * acc;
#pragma unroll
            for (int c = 0; c < kChB; ++c) r[c] = nx[c];
        }
    } else {   // 16-bit waves
        const int na = wpb - nbw;
        const int gw = blockIdx.x * na + (wv - nbw), nw = gridDim.x * na;
        uint4 r[kChA], nx[kChA];
        auto ld = [&](uint4 (&d)[kChA], int g) {
            const uint4* s = stA + size_t(min(g, G - 1)) * kChA * kWave + lane;
#pragma unroll
            for (int c = 0; c < kChA; ++c) d[c] = s[c * kWave];
        };
        if (GB + gw < G) ld(r, GB + gw);
        for (int g = GB + gw; g < G; g += nw) {
            ld(nx, g + nw);
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int c = 0; c < kChA; ++c) {
                const uint32_t v[4] = {r[c].x, r[c].y, r[c].z, r[c].w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t lo = v[i] & 0xffffu, hi = v[i] >> 16;
                    a0 += lw[min(lo, uint32_t(kSlots - 1))] * (lo != 0xffffu);
                    a1 += lw[min(hi, uint32_t(kSlots - 1))] * (hi != 0xffffu);
                }
            }
            ll += p[g * kWave + lane] * (a0 + a1);
#pragma unroll
            for (int c = 0; c < kChA; ++c) r[c] = nx[c];
        }
    }
    ll = wave_sum(ll);
    if (lane == 0) ll_part[blockIdx.x * wpb + wv] = ll;
}

int main() {
    const int S = 1 << 20, G = S / kWave;
    std::mt19937_64 rng(7);
    std::vector<int> succ(kSlots);
    std::vector<double> sw(kSlots), p(S);
    std::vector<uint16_t> nb(kSlots);
    for (int u = 0; u < kNodes; ++u)
        for (int d = 0; d < kDeg; ++d) {
            succ[u * kDeg + d] = int(rng() % kNodes);
            sw[u * kDeg + d] = -1.0 - double(rng() % 1000) * 1e-3;
            nb[u * kDeg + d] = uint16_t(succ[u * kDeg + d] * kDeg);
        }
    for (int s = 0; s < S; ++s) p[s] = 1.0 / S;
    std::vector<uint32_t> A(size_t(G) * kChA * kWave * 4, 0xffffffffu), B(size_t(G) * kChB * kWave * 4, 0u);
    double ref = 0.0;
    for (int s = 0; s < S; ++s) {
        const int g = s / kWave, l = s % kWave;
        int u = 0;
        double acc = 0.0;
        for (int e = 0; e < kLen; ++e) {
            const int d = int(rng() % 8);
            const int slot = u * kDeg + d;
            acc += sw[slot];
            // A: word e of the string at chunk e/8, u32 (e%8)/2, half e%2
            uint32_t& wa = A[((size_t(g) * kChA + e / 8) * kWave + l) * 4 + (e % 8) / 2];
            wa = (e % 2) ? ((wa & 0xffffu) | (uint32_t(slot) << 16)) : ((wa & 0xffff0000u) | uint32_t(slot));
            uint32_t& wb = B[((size_t(g) * kChB + e / 32) * kWave + l) * 4 + (e % 32) / 8];
            wb |= uint32_t(d) << (4 * (e % 8));
            u = succ[slot];
        }
        ref += p[s] * acc;
    }
    uint4 *dA, *dB;
    double *dsw, *dp, *dll;
    uint16_t* dnb;
    CK(hipMalloc(&dA, A.size() * 4));
    CK(hipMalloc(&dB, B.size() * 4));
    CK(hipMalloc(&dsw, kSlots * 8));
    CK(hipMalloc(&dnb, kSlots * 2));
    CK(hipMalloc(&dp, size_t(S) * 8));
    CK(hipMalloc(&dll, 1 << 20));
    CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dsw, sw.data(), kSlots * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dnb, nb.data(), kSlots * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dp, p.data(), size_t(S) * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch, int nwaves, double bytes) -> int {
        for (int r = 0; r < 3; ++r) launch();
        CK(hipDeviceSynchronize());
        const int reps = 50;
        CK(hipEventRecord(e0, 0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<double> part(nwaves);
        CK(hipMemcpy(part.data(), dll, size_t(nwaves) * 8, hipMemcpyDeviceToHost));
        double ll = 0.0;
        for (double v : part) ll += v;
        const double us = ms * 1e3 / reps;
        printf("%-28s %8.2f us  stream %6.1f MB  %7.1f GB/s  ll %.15g (ref %.15g, rel %.1e)\n", name, us, bytes / 1e6,
               bytes / us / 1e3, ll, ref, std::abs(ll - ref) / std::abs(ref));
        return 0;
    };
    const double bA = double(A.size()) * 4, bB = double(B.size()) * 4;
    for (int bpc : {1, 2, 4}) {   // blocks of 512 threads per CU
        const int grid = 256 * bpc;
        char nm[64];
        snprintf(nm, sizeof nm, "A 16-bit, %d x 512 / CU", bpc);
        if (run(nm, [&] { hipLaunchKernelGGL(walk_a, dim3(grid), dim3(512), 0, 0, dA, G, dsw, dp, dll); }, grid * 8, bA)) return 1;
    }
    for (int bpc : {1}) {
        const int grid = 256 * bpc;
        if (run("B nibble, K=1", [&] { hipLaunchKernelGGL(walk_b<1>, dim3(grid), dim3(1024), 0, 0, dB, G, dsw, dnb, dp, dll); },
                grid * 16, bB)) return 1;
        if (run("B nibble, K=2", [&] { hipLaunchKernelGGL(walk_b<2>, dim3(grid), dim3(1024), 0, 0, dB, G, dsw, dnb, dp, dll); },
                grid * 16, bB)) return 1;
        if (run("B nibble, K=4", [&] { hipLaunchKernelGGL(walk_b<4>, dim3(grid), dim3(1024), 0, 0, dB, G, dsw, dnb, dp, dll); },
                grid * 16, bB)) return 1;
    }
    {
        const int grid = 256;
        if (run("A 16-bit prefetch, 16 w/CU", [&] { hipLaunchKernelGGL(walk_a_pf<true>, dim3(grid), dim3(1024), 0, 0, dA, G, dsw, dp, dll); },
                grid * 16, bA)) return 1;
        if (run("B nibble prefetch, K=1", [&] { hipLaunchKernelGGL(walk_b_pf<1>, dim3(grid), dim3(1024), 0, 0, dB, G, dsw, dnb, dp, dll); },
                grid * 16, bB)) return 1;
        if (run("B nibble prefetch, K=2", [&] { hipLaunchKernelGGL(walk_b_pf<2>, dim3(grid), dim3(1024), 0, 0, dB, G, dsw, dnb, dp, dll); },
                grid * 16, bB)) return 1;
    }
    for (int nbw : {4, 5, 6, 8}) {   // mixed: nibble waves per block / 16, groups split in the same ratio
        for (double f : {0.25, 0.3, 0.35, 0.4}) {
            const int GB = int(G * f);
            char nm[64];
            snprintf(nm, sizeof nm, "mix %d/16 waves nibble, %.2f", nbw, f);
            const double bytes = bA * (1.0 - f) + bB * f;
            if (run(nm, [&] { hipLaunchKernelGGL(walk_mix, dim3(256), dim3(1024), 0, 0, dA, dB, GB, G, nbw, dsw, dsw, dnb,
                                                 dp, dll); }, 256 * 16, bytes)) return 1;
        }
    }
    if (run("A 16-bit prefetch, split hi/lo", [&] { hipLaunchKernelGGL(walk_a_split, dim3(256), dim3(1024), 0, 0, dA, G, dsw, dp, dll); },
            256 * 16, bA)) return 1;
    {   // C: one 16-byte LDS entry per edge (weight, next base)
        std::vector<double2> tab(kSlots);
        for (int j = 0; j < kSlots; ++j) {
            long long nbv = nb[j];
            double nbd;
            memcpy(&nbd, &nbv, 8);
            tab[j] = make_double2(sw[j], nbd);
        }
        double2* dtab;
        CK(hipMalloc(&dtab, kSlots * sizeof(double2)));
        CK(hipMemcpy(dtab, tab.data(), kSlots * sizeof(double2), hipMemcpyHostToDevice));
        const size_t lds = kSlots * sizeof(double2);
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&walk_c_pf<1>), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&walk_c_pf<2>), hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)));
        if (run("C nibble, 16-B entry, K=1", [&] { hipLaunchKernelGGL(walk_c_pf<1>, dim3(256), dim3(1024), lds, 0, dB, G, dtab, dp, dll); },
                256 * 16, bB)) return 1;
        if (run("C nibble, 16-B entry, K=2", [&] { hipLaunchKernelGGL(walk_c_pf<2>, dim3(256), dim3(1024), lds, 0, dB, G, dtab, dp, dll); },
                256 * 16, bB)) return 1;
    }
    {   // stream loads alone: the HBM floor of each format
        const int grid = 256;
        if (run("A loads only (no LDS)", [&] { hipLaunchKernelGGL(walk_a_pf<false>, dim3(grid), dim3(1024), 0, 0, dA, G, dsw, dp, dll); },
                grid * 16, bA)) return 1;
    }
    return 0;
}
