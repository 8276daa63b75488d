// Device helpers shared by the QN kernels and the stream kernel: wave
// reductions and the finish of a device-resident QuasiNewton step (the info
// row from qn_update's per-block partials, the halt decision, publication).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

#include "fb_kernels.hpp"

namespace wfsa {

__device__ inline double wave_reduce(double v, int op) {   // op 0 min, 1 max, 2 sum (fixed order)
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_xor(v, o, 64);
        v = op == 0 ? fmin(v, t) : (op == 1 ? fmax(v, t) : v + t);
    }
    return v;
}

// The finish of one step by one wavefront (it runs inside the next step's
// stream kernel, beside the streams, or as its own one-wave launch).
__device__ inline void qn_finish_wave(const QnArgs& a) {
    const int lane = int(threadIdx.x) & 63;
    const unsigned state = *a.halted;
    double gmin = INFINITY, gmax = -INFINITY, lmin = INFINITY, gerr = 0.0, ll = 0.0;
    if (state == 0) {
        for (int b = lane; b < a.n_partial; b += 64) {
            const double* p = a.partial + size_t(b) * 4;
            gmin = fmin(gmin, p[0]);
            gmax = fmax(gmax, p[1]);
            lmin = fmin(lmin, p[2]);
            gerr = fmax(gerr, p[3]);
        }
        if (a.ll_part) ll = strided_sum(a.ll_part, a.n_ll, lane, 64);
    }
    double rv = INFINITY, ri = -1.0;   // rmin column from block minima, ties to the lower string
    if (state == 0 && a.rmin_part)
        for (int b = lane; b < a.rmin_n_part; b += 64) {
            const double v = a.rmin_part[2 * b], i = a.rmin_part[2 * b + 1];
            if (v < rv || (v == rv && i < ri)) {
                rv = v;
                ri = i;
            }
        }
    for (int o = 32; o > 0; o >>= 1) {
        const double v = __shfl_xor(rv, o, 64), i = __shfl_xor(ri, o, 64);
        if (v < rv || (v == rv && i < ri)) {
            rv = v;
            ri = i;
        }
    }
    gmin = wave_reduce(gmin, 0);
    gmax = wave_reduce(gmax, 1);
    lmin = wave_reduce(lmin, 0);
    gerr = wave_reduce(gerr, 1);
    ll = wave_reduce(ll, 2);
    if (lane == 0) {
        unsigned status = kQnSkipped;
        double info[7] = {0, 0, 0, 0, 0, 0, 0};
        if (state == 0) {
            if (a.k == 0) gmin = gmax = lmin = 0.0;
            info[0] = a.plogp - (a.ll_part ? ll : *a.ll_val);
            info[1] = gerr;
            info[2] = gmin;
            info[3] = gmax;
            info[4] = lmin;
            if (a.rmin_part) {
                info[5] = ri >= 0.0 ? exp(rv) : 0.0;
                info[6] = ri;
            } else if (a.rmin) {
                info[5] = a.rmin[0];
                info[6] = a.rmin[1];
            }
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
