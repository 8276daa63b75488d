// Device helpers shared by the QN kernels and the stream kernel: block
// reductions and the finish of a device-resident QuasiNewton step (the info
// row from qn_update's per-block partials, the halt decision, publication).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#include "fb_kernels.hpp"

namespace wfsa {

__device__ inline double block_reduce(double v, int op, double* red) {   // op 0 min, 1 max
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_xor(v, o, 64);
        v = op == 0 ? fmin(v, t) : fmax(v, t);
    }
    const int w = int(threadIdx.x) / 64, lane = int(threadIdx.x) & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = red[0];
        for (int i = 1; i < int(blockDim.x) / 64; ++i) r = op == 0 ? fmin(r, red[i]) : fmax(r, red[i]);
        red[32] = r;
    }
    __syncthreads();
    return red[32];
}

__device__ inline double block_sum(double v, double* red) {   // fixed order for a fixed block size
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = int(threadIdx.x) / 64, lane = int(threadIdx.x) & 63;
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double r = red[0];
        for (int i = 1; i < int(blockDim.x) / 64; ++i) r += red[i];
        red[32] = r;
    }
    __syncthreads();
    return red[32];
}

// The finish of one step by one block (any size, a multiple of 64).
__device__ inline void qn_finish_block(const QnArgs& a) {
    __shared__ double red[33];
    const unsigned state = *a.halted;
    const int t = int(threadIdx.x), nt = int(blockDim.x);
    double gmin = INFINITY, gmax = -INFINITY, lmin = INFINITY, gerr = 0.0, ll = 0.0;
    if (state == 0) {
        for (int b = t; b < a.n_partial; b += nt) {
            const double* p = a.partial + size_t(b) * 4;
            gmin = fmin(gmin, p[0]);
            gmax = fmax(gmax, p[1]);
            lmin = fmin(lmin, p[2]);
            gerr = fmax(gerr, p[3]);
        }
        if (a.ll_part)
            ll = strided_sum(a.ll_part, a.n_ll, t, nt);
    }
    gmin = block_reduce(gmin, 0, red);
    gmax = block_reduce(gmax, 1, red);
    lmin = block_reduce(lmin, 0, red);
    gerr = block_reduce(gerr, 1, red);
    ll = block_sum(ll, red);
    if (t == 0) {
        unsigned status = kQnSkipped;
        double info[7] = {0, 0, 0, 0, 0, 0, 0};
        if (state == 0) {
            if (a.k == 0) gmin = gmax = lmin = 0.0;
            info[0] = a.plogp - (a.ll_part ? ll : *a.ll_val);
            info[1] = gerr;
            info[2] = gmin;
            info[3] = gmax;
            info[4] = lmin;
            bool finite = true;
            for (int i = 0; i < 7; ++i) finite = finite && isfinite(info[i]);
            const bool halt = gerr <= a.tol && fabs(gmin) <= a.tol && fabs(gmax) <= a.tol;
            status = !finite ? kQnNonFinite : (halt ? kQnHalted : kQnRan);
        }
        double* row = a.host_ring + size_t(a.ring_slot) * kQnRow;
        for (int i = 0; i < 7; ++i) row[i] = info[i];
        row[7] = double(status);
        if (status == kQnHalted || status == kQnNonFinite) *a.halted = status;
        const unsigned v = *a.seq + 1u;
        *a.seq = v;
        // the system-scope release orders the row before the flag
        __hip_atomic_store(a.host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace wfsa
