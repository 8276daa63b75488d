// Device-resident QuasiNewton step: the KKT-diagonal update of
// QuasiNewtonLearner::OptimizationStep (src/QuasiNewtonLearner.cpp:162-201,
// with ComputeExpX :53-56, ComputeG :148-160, ComputeLambdaNext :127-146,
// Learner::LambdaUpdate src/Learner.cpp:438-462, HaltCondition :88-91 and
// GetOptimizationInfo :68-86) after the objective/gradient kernels of the
// same step: qn_update (thread per constraint) + qn_finish (one workgroup).  It keeps x, lambda and the next step's w_full in
// HBM, so consecutive steps need nothing from the host; each step publishes
// its info row to host-mapped memory and bumps the completion flag.
//
// The arithmetic follows the host code operation for operation (the same
// summation orders, no FMA contraction) so the device and host trajectories
// agree to the last bits up to exp()'s rounding.
#include "fb_kernels.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#pragma clang fp contract(off)

namespace wfsa {

namespace {

constexpr int kQnUpdateBlock = 64;    // one wavefront: registers for whole groups
constexpr int kQnFinishBlock = 1024;
constexpr int kQnRegMembers = 16;     // constraint groups up to this size stay in registers

__device__ double block_reduce(double v, int op, double* red) {   // op 0 min, 1 max
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

__device__ double block_sum(double v, double* red) {   // fixed order for a fixed block size
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

// qn_update: one thread per constraint, one wavefront per block (so a
// thread may keep a whole group in registers).  Every quantity of the update
// is local to a constraint -- its members are a contiguous, ascending range
// of parameters -- so the blocks are independent; each writes its partial
// (g_min, g_max, lambda_min, graderr) and qn_finish reduces them.
__global__ __launch_bounds__(kQnUpdateBlock) void qn_update_kernel(QnArgs a) {
    if (*a.halted) return;
    const int c = int(blockIdx.x) * kQnUpdateBlock + int(threadIdx.x);
    double gmin = INFINITY, gmax = -INFINITY, lmin = INFINITY, gerr = 0.0;
    if (c < a.k) {
        const double* __restrict__ out = a.out;
        const int32_t* __restrict__ full_of = a.full_of;
        double* __restrict__ x = a.x;
        double* __restrict__ expx = a.expx;
        double* __restrict__ grad = a.grad;
        double* __restrict__ w_full = a.w_full;
        const int b = a.cptr[c], e = a.cptr[c + 1];
        const double lam = a.lambda[c];
        double g = -1.0, laux;
        if (e - b <= kQnRegMembers) {
            // members in registers: every load issued before the first use
            double xv[kQnRegMembers], gv[kQnRegMembers], ev[kQnRegMembers];
#pragma unroll
            for (int m = 0; m < kQnRegMembers; ++m)
                if (b + m < e) {
                    xv[m] = x[b + m];
                    const int fo = full_of[b + m];
                    gv[m] = out[1 + fo] + (a.fixed ? a.fixed[fo] : 0.0);
                }
            // ComputeExpX, ComputeG: g = -1 + sum exp(x) in member order
#pragma unroll
            for (int m = 0; m < kQnRegMembers; ++m)
                if (b + m < e) {
                    ev[m] = exp(xv[m]);
                    g += ev[m];
                }
            // ComputeLambdaNext: (lambda g - sum grad) / (g + 1)
            double r = lam * g;
#pragma unroll
            for (int m = 0; m < kQnRegMembers; ++m)
                if (b + m < e) r -= gv[m];
            laux = r / (g + 1.0);
            // graderr (old lambda), x update (lambda_next), next weights
#pragma unroll
            for (int m = 0; m < kQnRegMembers; ++m)
                if (b + m < e) {
                    const double aux = ev[m] * lam;
                    gerr = fmax(gerr, fabs(gv[m] + aux));
                    const double xi = xv[m] - a.eta * ((gv[m] + ev[m] * laux) / aux);
                    x[b + m] = xi;
                    grad[b + m] = gv[m];
                    w_full[full_of[b + m]] = xi;   // GetWeight for the next step
                }
        } else {   // large groups (dense automata): the same through memory
            for (int i = b; i < e; ++i) {
                const double ex = exp(x[i]);
                expx[i] = ex;
                g += ex;
            }
            double r = lam * g;
            for (int i = b; i < e; ++i) {
                const double gi = out[1 + full_of[i]] + (a.fixed ? a.fixed[full_of[i]] : 0.0);
                grad[i] = gi;
                r -= gi;
            }
            laux = r / (g + 1.0);
            for (int i = b; i < e; ++i) {
                const double ex = expx[i], gi = grad[i];
                const double aux = ex * lam;
                gerr = fmax(gerr, fabs(gi + aux));
                const double xi = x[i] - a.eta * ((gi + ex * laux) / aux);
                x[i] = xi;
                w_full[full_of[i]] = xi;
            }
        }
        // LambdaUpdate (src/Learner.cpp:438-462)
        const double d = lam - laux;
        a.lambda[c] = a.exp_lambda ? lam * exp(-a.eta * (d / lam)) : lam - a.eta * d;
        gmin = g;
        gmax = g;
        lmin = lam;
    }
    for (int o = 32; o > 0; o >>= 1) {
        gmin = fmin(gmin, __shfl_xor(gmin, o, 64));
        gmax = fmax(gmax, __shfl_xor(gmax, o, 64));
        lmin = fmin(lmin, __shfl_xor(lmin, o, 64));
        gerr = fmax(gerr, __shfl_xor(gerr, o, 64));
    }
    if (threadIdx.x == 0) {
        double* p = a.partial + size_t(blockIdx.x) * 4;
        p[0] = gmin;
        p[1] = gmax;
        p[2] = lmin;
        p[3] = gerr;
    }
}

// qn_finish: the info row of the step (the reductions of qn_update's
// partials and, without the tail kernel, of the per-wave log-likelihood
// partials in a fixed order), the halt decision, then the publication.
__global__ __launch_bounds__(kQnFinishBlock) void qn_finish_kernel(QnArgs a) {
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
            info[0] = a.plogp - (a.ll_part ? ll : a.out[0]);
            info[1] = gerr;
            info[2] = gmin;
            info[3] = gmax;
            info[4] = lmin;
            bool finite = true;
            for (int i = 0; i < 7; ++i) finite = finite && isfinite(info[i]);
            const bool halt = gerr <= a.tol && fabs(gmin) <= a.tol && fabs(gmax) <= a.tol;
            status = !finite ? kQnNonFinite : (halt ? kQnHalted : kQnRan);
        }
        double* row = a.host_ring + size_t(a.slot) * kQnRow;
        for (int i = 0; i < 7; ++i) row[i] = info[i];
        row[7] = double(status);
        if (status == kQnHalted || status == kQnNonFinite) *a.halted = status;
        const unsigned v = *a.seq + 1u;
        *a.seq = v;
        // the system-scope release orders the row before the flag
        __hip_atomic_store(a.host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// initial w_full from x (qn_set_state)
__global__ void qn_weights_kernel(const double* x, const int32_t* trim, int32_t n_full, double* w_full) {
    const int j = int(blockIdx.x * blockDim.x + threadIdx.x);
    if (j < n_full) {
        const int tj = trim[j];
        w_full[j] = tj >= 0 ? x[tj] : (tj == -1 ? 0.0 : -INFINITY);
    }
    if (j == n_full) w_full[j] = 0.0;   // the zero slot of the stream kernel
}

}  // namespace

int qn_update_blocks(int32_t k) { return std::max(1, (k + kQnUpdateBlock - 1) / kQnUpdateBlock); }

hipError_t launch_qn(const QnArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(qn_update_kernel, dim3(unsigned(qn_update_blocks(a.k))), dim3(kQnUpdateBlock), 0, stream, a);
    hipLaunchKernelGGL(qn_finish_kernel, dim3(1), dim3(kQnFinishBlock), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_qn_weights(const double* x, const int32_t* trim, int32_t n_full, double* w_full,
                             hipStream_t stream) {
    const unsigned blocks = unsigned((n_full + 1 + 255) / 256);
    hipLaunchKernelGGL(qn_weights_kernel, dim3(blocks), dim3(256), 0, stream, x, trim, n_full, w_full);
    return hipGetLastError();
}

}  // namespace wfsa
