// Device-resident QuasiNewton step: the KKT-diagonal update of
// QuasiNewtonLearner::OptimizationStep (src/QuasiNewtonLearner.cpp:162-201,
// with ComputeExpX :53-56, ComputeG :148-160, ComputeLambdaNext :127-146,
// Learner::LambdaUpdate src/Learner.cpp:438-462, HaltCondition :88-91 and
// GetOptimizationInfo :68-86) after the objective/gradient kernels of the
// same step, in ONE launch: qn_step_kernel, one block per constraint, and the
// step's finish by the last block to arrive.  It keeps x, lambda and the next
// step's w_full in HBM, so consecutive steps need nothing from the host; each
// step publishes its info row to host-mapped memory and bumps the flag.
//
// Fused form: the members' gradients are completed here from the bubble
// contribution slots (the slots are laid out in trimmed-parameter order, so a
// constraint's members own one contiguous run, summed by seg_sums in a fixed
// order) -- no separate reduction launch.
//
// The arithmetic follows the host code operation for operation (the same
// summation orders, no FMA contraction) so the device and host trajectories
// agree to the last bits up to exp()'s rounding and the gradient's summation.
#include "fb_kernels.hpp"
#include "qn_device.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#pragma clang fp contract(off)

namespace wfsa {

namespace {

constexpr int kW = kQnBlock / 64;

// the info row of a step into its host ring slot, then the flag; the
// system-scope release orders the row before the flag
__device__ void publish_row(const QnArgs& a, const double* info, unsigned status) {
    double* row = a.host_ring + size_t(a.ring_slot) * kQnRow;
    for (int i = 0; i < 7; ++i) row[i] = info ? info[i] : 0.0;
    row[7] = double(status);
    const unsigned v = *a.seq + 1u;
    *a.seq = v;
    __hip_atomic_store(a.host_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ double block_reduce(double v, int op, double* red) {   // fixed tree, every thread gets the result
    const int t = int(threadIdx.x);
    v = wave_reduce(v, op);
    __syncthreads();
    if ((t & 63) == 0) red[t >> 6] = v;
    __syncthreads();
    double r = red[0];
    for (int i = 1; i < kW; ++i) r = op == 0 ? fmin(r, red[i]) : (op == 1 ? fmax(r, red[i]) : r + red[i]);
    return r;
}

template <bool FUSED>
__global__ __launch_bounds__(kQnBlock) void qn_step_kernel(QnArgs a) {
    const int t = int(threadIdx.x);
    const int c = int(blockIdx.x);
    // halted is written only by an earlier launch's finish: every block of
    // this launch sees the same value
    if (*a.halted) {   // a step enqueued after the halt: published as skipped
        if (c == 0 && t == 0) publish_row(a, nullptr, kQnSkipped);
        return;
    }
    __shared__ double sg[kQnMaxSeg], se[kQnMaxSeg];
    __shared__ int sp[kQnMaxSeg + 1];
    __shared__ SegScratch<kQnBlock> sc;
    __shared__ double bc[2], red[kW];
    __shared__ unsigned last;
    double gerr = 0.0, g = 0.0, lam = 0.0;
    const bool have = c < a.k;
    if (have) {
        const int b = a.cptr[c], e = a.cptr[c + 1], nm = e - b;
        lam = a.lambda[c];
        double laux;
        const bool slots = FUSED && a.contrib;
        if (slots) {   // the members' bubble slot sums (the host guarantees nm <= kQnMaxSeg)
            const int s0 = a.seg_ptr[b];
            for (int i = t; i <= nm; i += kQnBlock) sp[i] = a.seg_ptr[b + i] - s0;
            __syncthreads();
            seg_sums<kQnBlock>(a.contrib + s0, sp, nm, seg_piece(sp[nm], kQnBlock), sg, sc);
        }
        if (nm <= kQnMaxSeg) {
            for (int m = t; m < nm; m += kQnBlock) {
                const int fo = a.full_of[b + m];
                double gi = a.out[1 + fo];
                if (a.fixed) gi += a.fixed[fo];
                if (slots) gi += sg[m];
                sg[m] = gi;
                se[m] = exp(a.x[b + m]);
            }
            __syncthreads();
            if (t == 0) {   // ComputeG, ComputeLambdaNext in member order
                double gg = -1.0;
                for (int m = 0; m < nm; ++m) gg += se[m];
                double r = lam * gg;
                for (int m = 0; m < nm; ++m) r -= sg[m];
                bc[0] = gg;
                bc[1] = r / (gg + 1.0);
            }
            __syncthreads();
            g = bc[0];
            laux = bc[1];
            for (int m = t; m < nm; m += kQnBlock) {   // graderr (old lambda), x update (lambda_next)
                const double gi = sg[m], ei = se[m];
                const double aux = ei * lam;
                gerr = fmax(gerr, fabs(gi + aux));
                const double xn = a.x[b + m] - a.eta * ((gi + ei * laux) / aux);
                const int fo = a.full_of[b + m];
                a.x[b + m] = xn;
                a.grad[b + m] = gi;
                a.w_full[fo] = xn;   // GetWeight for the next step
                a.ewp[fo] = exp(xn);
            }
        } else {   // large groups (dense automata; never fused): members strided
                   // over the threads, sums by a fixed tree (deterministic; the
                   // host's member-order sums differ from it by rounding only)
            double gs = 0.0, gv = 0.0;
            for (int i = b + t; i < e; i += kQnBlock) {
                const double ex = exp(a.x[i]);
                const int fo = a.full_of[i];
                double gi = a.out[1 + fo];
                if (a.fixed) gi += a.fixed[fo];
                a.expx[i] = ex;
                a.grad[i] = gi;
                gs += ex;
                gv += gi;
            }
            gs = block_reduce(gs, 2, red);
            gv = block_reduce(gv, 2, red);
            g = -1.0 + gs;
            laux = (lam * g - gv) / (g + 1.0);
            for (int i = b + t; i < e; i += kQnBlock) {
                const double ex = a.expx[i], gi = a.grad[i];
                const double aux = ex * lam;
                gerr = fmax(gerr, fabs(gi + aux));
                const double xn = a.x[i] - a.eta * ((gi + ex * laux) / aux);
                a.x[i] = xn;
                a.w_full[a.full_of[i]] = xn;
                a.ewp[a.full_of[i]] = exp(xn);
            }
        }
        if (t == 0) {   // LambdaUpdate (src/Learner.cpp:438-462)
            const double d = lam - laux;
            a.lambda[c] = a.exp_lambda ? lam * exp(-a.eta * (d / lam)) : lam - a.eta * d;
        }
    }
    gerr = block_reduce(gerr, 1, red);
    // the block's partial, write-through, then the arrival ticket; the block
    // whose arrival is the last finishes the step
    if (t == 0) {
        double* p = a.partial + size_t(c) * 4;
        const double pv[4] = {have ? g : INFINITY, have ? g : -INFINITY, have ? lam : INFINITY, gerr};
        for (int i = 0; i < 4; ++i) __hip_atomic_store(p + i, pv[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned nb = gridDim.x;
        last = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1u;
    }
    __syncthreads();
    if (!last) return;
    // finish: the info row from the block partials (write-through loads) and
    // the log-likelihood partials (written by earlier launches), fixed order
    double gmin = INFINITY, gmax = -INFINITY, lmin = INFINITY, ge = 0.0;
    for (int j = t; j < int(gridDim.x); j += kQnBlock) {
        const double* p = a.partial + size_t(j) * 4;
        gmin = fmin(gmin, __hip_atomic_load(p + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        gmax = fmax(gmax, __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        lmin = fmin(lmin, __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        ge = fmax(ge, __hip_atomic_load(p + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    gmin = block_reduce(gmin, 0, red);
    gmax = block_reduce(gmax, 1, red);
    lmin = block_reduce(lmin, 0, red);
    ge = block_reduce(ge, 1, red);
    double ll = a.ll_part ? strided_sum(a.ll_part, a.n_ll, t, kQnBlock) : 0.0;
    ll = block_reduce(ll, 2, red);
    double rv = INFINITY, ri = -1.0;   // rmin column from block minima, ties to the lower string
    if (a.rmin_part)
        for (int j = t; j < a.rmin_n_part; j += kQnBlock) {
            const double v = a.rmin_part[2 * j], i = a.rmin_part[2 * j + 1];
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
    __shared__ double rr[kW][2];
    if ((t & 63) == 0) {
        rr[t >> 6][0] = rv;
        rr[t >> 6][1] = ri;
    }
    __syncthreads();
    if (t == 0) {
        for (int w = 1; w < kW; ++w)
            if (rr[w][0] < rv || (rr[w][0] == rv && rr[w][1] < ri)) {
                rv = rr[w][0];
                ri = rr[w][1];
            }
        if (a.k == 0) gmin = gmax = lmin = 0.0;
        double info[7];
        info[0] = a.plogp - (a.ll_part ? ll : a.out[0]);
        info[1] = ge;
        info[2] = gmin;
        info[3] = gmax;
        info[4] = lmin;
        info[5] = 0.0;
        info[6] = 0.0;
        if (a.rmin_part) {
            info[5] = ri >= 0.0 ? exp(rv) : 0.0;
            info[6] = ri;
        } else if (a.rmin) {
            info[5] = a.rmin[0];
            info[6] = a.rmin[1];
        }
        bool finite = true;
        for (int i = 0; i < 7; ++i) finite = finite && isfinite(info[i]);
        const bool halt = ge <= a.tol && fabs(gmin) <= a.tol && fabs(gmax) <= a.tol;
        const unsigned status = !finite ? kQnNonFinite : (halt ? kQnHalted : kQnRan);
        if (status != kQnRan) *a.halted = status;   // read by the next launches only
        *a.ticket = 0u;
        publish_row(a, info, status);
    }
}

// initial w_full from x (qn_set_state)
__global__ void qn_weights_kernel(const double* x, const int32_t* trim, int32_t n_full, double* w_full, double* ewp) {
    const int j = int(blockIdx.x * blockDim.x + threadIdx.x);
    if (j < n_full) {
        const int tj = trim[j];
        w_full[j] = tj >= 0 ? x[tj] : (tj == -1 ? 0.0 : -INFINITY);
        ewp[j] = exp(w_full[j]);
    }
    if (j == n_full) {   // the zero slot of the stream kernel
        w_full[j] = 0.0;
        ewp[j] = 1.0;
    }
}

}  // namespace

hipError_t launch_qn_step(const QnArgs& a, bool fused, hipStream_t stream) {
    const dim3 grid(unsigned(std::max(a.k, 1)));
    if (fused) hipLaunchKernelGGL(qn_step_kernel<true>, grid, dim3(kQnBlock), 0, stream, a);
    else hipLaunchKernelGGL(qn_step_kernel<false>, grid, dim3(kQnBlock), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_qn_weights(const double* x, const int32_t* trim, int32_t n_full, double* w_full, double* ewp,
                             hipStream_t stream) {
    const unsigned blocks = unsigned((n_full + 1 + 255) / 256);
    hipLaunchKernelGGL(qn_weights_kernel, dim3(blocks), dim3(256), 0, stream, x, trim, n_full, w_full, ewp);
    return hipGetLastError();
}

}  // namespace wfsa
